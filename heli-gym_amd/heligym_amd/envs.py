"""Single-environment drop-ins for the reference classes `Heli`, `HeliHover`, `HeliForwardFlight`
(heligym/envs/helicopter.py:28-243, heligym/envs/helicopter_with_tasks.py:5-115).

Same constructor argument, reset()/step() signatures and return types, same setters.  Each
instance is a one-env `HeliVecEnv` without auto-reset (the reference never resets by itself), so
its step runs in the same gfx950 kernel as the batched env.  Rendering (the reference's OpenGL
window) is not part of this package: render() raises NotImplementedError.
"""
import numpy as np

from . import _abi, config
from .vector import HeliVecEnv


class Heli:
    """helicopter.py:28 — base task: reward 0, never succeeds on its own."""

    _task = "heli"
    metadata = {"render.modes": ["human", "rgb_array"], "video.frames_per_second": config.FPS}
    default_max_time = config.DEFAULT_MAX_TIME
    default_trim_cond = dict(config.DEFAULT_TRIM_COND)

    def __init__(self, heli_name: str = "aw109", dt: float = config.DT, seed: int = 0, device=None):
        self._env = HeliVecEnv(1, task=self._task, dt=dt, heli_name=heli_name, seed=seed, device=device,
                               autoreset=False)
        self.observation_space = self._env.observation_space
        self.action_space = self._env.action_space
        self.normalizers = self._env.normalizers
        self.max_time = self._env.max_time
        self.success_duration = self.max_time / 4
        self.task_duration = self.max_time / 4
        t = self._env.torch
        self._act = t.zeros((1, 4), dtype=t.float32, device=self._env.device)
        # pinned host staging: one async H2D copy of the action, async D2H copies of the results
        # and a single stream synchronisation per step
        self._h_act = t.zeros((1, 4), dtype=t.float32).pin_memory()
        self._h_obs = t.zeros((1, 17), dtype=t.float32).pin_memory()
        self._h_rew = t.zeros((1,), dtype=t.float32).pin_memory()
        self._h_flags = t.zeros((3,), dtype=t.uint8).pin_memory()

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

    def reset(self):
        """helicopter.py:208-217 -> (obs float32[17], info)."""
        obs, info = self._env.reset()
        return obs[0].cpu().numpy().copy(), {k: bool(v[0]) for k, v in info.items()}

    def step(self, actions):
        """helicopter.py:192-206 -> (obs, reward, terminated, truncated, info)."""
        e = self._env
        self._h_act.numpy()[0] = np.asarray(actions, dtype=np.float32).reshape(4)
        self._act.copy_(self._h_act, non_blocking=True)
        e.step_async(self._act, with_reset_info=False)
        self._h_obs.copy_(e.obs, non_blocking=True)
        self._h_rew.copy_(e.reward, non_blocking=True)
        self._h_flags[0:1].copy_(e.terminated_u8, non_blocking=True)
        self._h_flags[1:2].copy_(e.truncated_u8, non_blocking=True)
        self._h_flags[2:3].copy_(e.info_u8, non_blocking=True)
        e.torch.cuda.current_stream(e.device).synchronize()
        fl = self._h_flags.numpy()
        bits = int(fl[2])
        info = {"failed": bool(bits & _abi.HG_INFO_FAILED), "successed": bool(bits & _abi.HG_INFO_SUCCESSED),
                "time_up": bool(bits & _abi.HG_INFO_TIME_UP)}
        return self._h_obs.numpy()[0].copy(), float(self._h_rew.numpy()[0]), bool(fl[0]), bool(fl[1]), info

    def render(self):
        raise NotImplementedError("rendering is outside heligym_amd (the reference renders with OpenGL)")

    def close(self):
        self._env.close()


class HeliHover(Heli):
    """helicopter_with_tasks.py:5-52"""

    _task = "hover"


class HeliForwardFlight(Heli):
    """helicopter_with_tasks.py:54-115"""

    _task = "forward_flight"
