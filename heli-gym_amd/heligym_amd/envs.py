"""Single-environment drop-ins for the reference classes `Heli`, `HeliHover`, `HeliForwardFlight`
(heligym/envs/helicopter.py:28-243, heligym/envs/helicopter_with_tasks.py:5-115).

Same constructor argument, reset()/step() signatures and return types, same setters.  Each
instance is a one-env `HeliVecEnv` without auto-reset (the reference never resets by itself), so
its step runs in the same gfx950 kernel as the batched env.  Rendering (the reference's OpenGL
window) is not part of this package: render() raises NotImplementedError.
"""
import ctypes

import numpy as np

from . import _abi, config
from .vector import HeliVecEnv

try:   # the reference's lineage, class Heli(gym.Env, EzPickle) (helicopter.py:28), when gymnasium is installed
    import gymnasium as _gym
    from gymnasium.utils import EzPickle as _EzPickle
    _BASES = (_gym.Env, _EzPickle)
except ImportError:   # gymnasium is optional: the same surface, duck-typed
    _EzPickle = None
    _BASES = (object,)


class Heli(*_BASES):
    """helicopter.py:28 — base task: reward 0, never succeeds on its own."""

    _task = "heli"
    _IO = {"act": 0, "obs": 16, "rew": 96, "flags": 112, "eta": 116}   # host-mapped I/O block layout
    _IO_BYTES = 128
    metadata = {"render.modes": ["human", "rgb_array"], "video.frames_per_second": config.FPS}
    default_max_time = config.DEFAULT_MAX_TIME
    default_trim_cond = dict(config.DEFAULT_TRIM_COND)

    def __init__(self, heli_name: str = "aw109", dt: float = config.DT, seed: int = 0, device=None):
        if _EzPickle is not None:   # helicopter.py:48
            _EzPickle.__init__(self, heli_name, dt, seed, device)
        # reset_mode "retrim": like the reference, every reset() trims against the wind of the last
        # step (helicopter.py:208-212 -> helicopter_dynamics.py:66-71), on the device
        self._env = HeliVecEnv(1, task=self._task, dt=dt, heli_name=heli_name, seed=seed, device=device,
                               autoreset=False, reset_mode="retrim")
        self.observation_space = self._env.single_observation_space   # helicopter.py:56-57
        self.action_space = self._env.single_action_space
        self.normalizers = self._env.normalizers
        self.max_time = self._env.max_time
        self.success_duration = self.max_time / 4
        self.task_duration = self.max_time / 4
        # Host-mapped I/O (hg_host_alloc): the kernel reads the action from and writes the
        # observation, reward and flags to pinned host memory directly, so a step is one launch
        # and one stream synchronisation, with no copies.
        lib = self._env.lib
        host, dev = ctypes.c_void_p(), ctypes.c_void_p()
        _abi.check(lib.hg_host_alloc(self._IO_BYTES, ctypes.byref(host), ctypes.byref(dev)), lib)
        self._io_host, self._io_dev = host.value, dev.value
        buf = (ctypes.c_uint8 * self._IO_BYTES).from_address(self._io_host)
        raw = np.frombuffer(buf, dtype=np.uint8)
        o = self._IO
        self._io_act = raw[o["act"]:o["act"] + 16].view(np.float32)
        self._io_obs = raw[o["obs"]:o["obs"] + 68].view(np.float32)
        self._io_rew = raw[o["rew"]:o["rew"] + 4].view(np.float32)
        self._io_flags = raw[o["flags"]:o["flags"] + 3]
        self._io_eta = raw[o["eta"]:o["eta"] + 12].view(np.float32)

    # setters (helicopter.py:89-111)
    def set_max_time(self, max_time=None):
        self._env.set_max_time(max_time)
        self.max_time = self._env.max_time
        self.success_duration = self.max_time / 4
        self.task_duration = self.max_time / 4

    def set_target(self, target={}):
        self._env.set_target(target)

    def get_target(self):
        return self._env.get_target()

    def set_trim_cond(self, trim_cond={}):
        self._env.set_trim_cond(trim_cond)

    def get_trim_cond(self):
        return self._env.get_trim_cond()

    def set_reward_weights(self, base_reward_weight=None, terminal_reward_weight=None):
        # stored but unused, as in the reference (helicopter.py:108-111)
        zero = np.zeros((17, 17))
        self.base_reward_weight = zero if base_reward_weight is None else base_reward_weight
        self.terminal_reward_weight = zero if terminal_reward_weight is None else terminal_reward_weight

    def reset(self, seed=None, options=None):
        """helicopter.py:208-217 -> (obs float32[17], info).  The reference takes no arguments;
        `seed` / `options` are accepted (and ignored: the noise is keyed by the constructor's seed)
        so that gymnasium's wrappers, which pass them, work."""
        obs, info = self._env.reset()
        return obs[0].cpu().numpy().copy(), {k: bool(v[0]) for k, v in info.items()}

    def step(self, actions, eta=None):
        """helicopter.py:192-206 -> (obs, reward, terminated, truncated, info).  `eta`: optional
        turbulence noise [3] (already scaled by 1/sqrt(dt)) instead of the in-kernel Philox draw --
        the reference's `wind_dyn.eta` (wind_dynamics.py:49-52), for replaying recorded episodes."""
        e = self._env
        self._io_act[:] = np.asarray(actions, dtype=np.float32).reshape(4)
        d, o = self._io_dev, self._IO
        if eta is not None:
            self._io_eta[:] = np.asarray(eta, dtype=np.float32).reshape(3)
        stream = e.torch.cuda.current_stream(e.device)
        e._check(e.lib.hg_step(e._h, d + o["act"], d + o["obs"], d + o["rew"], d + o["flags"],
                               d + o["flags"] + 1, d + o["flags"] + 2, None if eta is None else d + o["eta"],
                               None, None, None, ctypes.c_void_p(stream.cuda_stream)))
        stream.synchronize()
        fl = self._io_flags
        bits = int(fl[2])
        info = {"failed": bool(bits & _abi.HG_INFO_FAILED), "successed": bool(bits & _abi.HG_INFO_SUCCESSED),
                "time_up": bool(bits & _abi.HG_INFO_TIME_UP)}
        return self._io_obs.copy(), float(self._io_rew[0]), bool(fl[0]), bool(fl[1]), info

    def render(self):
        raise NotImplementedError("rendering is outside heligym_amd (the reference renders with OpenGL)")

    def close(self):
        if getattr(self, "_io_host", None):
            self._env.lib.hg_host_free(self._io_host)
            self._io_host = None
        self._env.close()


class HeliHover(Heli):
    """helicopter_with_tasks.py:5-52"""

    _task = "hover"


class HeliForwardFlight(Heli):
    """helicopter_with_tasks.py:54-115"""

    _task = "forward_flight"
