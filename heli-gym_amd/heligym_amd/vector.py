"""Batched heli-gym environment on one MI355X: N helicopters advanced by one HIP kernel per step.

`HeliVecEnv` is the vectorised counterpart of the reference's `Heli` gymnasium env
(heligym/envs/helicopter.py:28-243): same 17-observation / 4-action contract, same reward, flags and
setters, with same-step auto-reset.  All buffers are PyTorch-ROCm tensors on the env's device; the
step itself runs in `libheligym_amd.so` (no CPU path exists).
"""
import ctypes

import numpy as np

from . import _abi, config


class Box:
    """Minimal stand-in for gymnasium.spaces.Box (gymnasium is optional)."""

    def __init__(self, low, high, shape, dtype=np.float32):
        self.low = np.full(shape, low, dtype=dtype)
        self.high = np.full(shape, high, dtype=dtype)
        self.shape = tuple(shape)
        self.dtype = np.dtype(dtype)

    def sample(self, rng=np.random):
        lo = np.where(np.isfinite(self.low), self.low, -1.0)
        hi = np.where(np.isfinite(self.high), self.high, 1.0)
        return rng.uniform(lo, hi).astype(self.dtype)

    def contains(self, x):
        x = np.asarray(x)
        return x.shape == self.shape and bool(np.all(x >= self.low) and np.all(x <= self.high))


def _make_box(low, high, shape):
    try:  # use the real class when gymnasium is installed
        from gymnasium import spaces
        return spaces.Box(low, high, shape=shape, dtype=np.float32)
    except ImportError:
        return Box(low, high, shape)


class LazyInfo(dict):
    """The info dict of HeliVecEnv.step(): keys present at once, each value computed on first
    access (then cached).  `valid()` says whether the step's buffers still hold its values; reading
    a field after they were reused raises instead of returning another step's data."""

    def __init__(self, thunks, valid, gen=None):
        """thunks: key -> f(info) computing the value (shared between steps: per-step state goes
        on the info object).  valid: () -> bool; or, with `gen`, the env whose step `gen` this is:
        the values stay readable while env._gen - gen < 2 (the step's buffer set is not reused
        before the step after next)."""
        super().__init__(dict.fromkeys(thunks))
        self._thunks = thunks
        self._pending = set(thunks)
        self._src = valid
        self._gen = gen

    def _valid(self):
        return self._src() if self._gen is None else self._src._gen - self._gen < 2

    def _get(self, k):
        if k in self._pending:
            if not self._valid():
                raise _abi.HeliGymError(f"info[{k!r}] read after its buffers were reused (read info before "
                                        "the step after next)")
            dict.__setitem__(self, k, self._thunks[k](self))
            self._pending.discard(k)
        return dict.__getitem__(self, k)

    def __getitem__(self, k):
        return self._get(k)

    def get(self, k, default=None):
        return self._get(k) if k in self else default

    def __iter__(self):
        return iter(list(dict.keys(self)))

    def items(self):
        return [(k, self._get(k)) for k in list(dict.keys(self))]

    def values(self):
        return [self._get(k) for k in list(dict.keys(self))]

    def copy(self):
        return {k: self._get(k) for k in list(dict.keys(self))}

    # every other read path goes through _get as well, so no caller ever sees a None placeholder
    def __setitem__(self, k, v):
        self._pending.discard(k)
        dict.__setitem__(self, k, v)

    def update(self, *args, **kw):
        for k, v in dict(*args, **kw).items():
            self[k] = v

    _MISSING = object()

    def pop(self, k, default=_MISSING):
        if k not in self:
            if default is LazyInfo._MISSING:
                raise KeyError(k)
            return default
        v = self._get(k)
        dict.pop(self, k)
        return v

    def popitem(self):
        if not len(self):
            raise KeyError("popitem(): dictionary is empty")
        k = list(dict.keys(self))[-1]
        return k, self.pop(k)

    def setdefault(self, k, default=None):
        if k in self:
            return self._get(k)
        dict.__setitem__(self, k, default)
        return default

    def __reduce__(self):   # pickles / deep-copies as the plain dict of its values
        return (dict, (self.copy(),))

    def __deepcopy__(self, memo):
        import copy
        return copy.deepcopy(self.copy(), memo)

    def __repr__(self):
        return repr(self.copy())

    def __eq__(self, other):
        return self.copy() == (other.copy() if isinstance(other, LazyInfo) else other)

    __hash__ = None


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


OBS_NAMES = ("POWER", "LON_AIR_SPD", "LAT_AIR_SPD", "DWN_AIR_SPD", "N_VEL", "E_VEL", "DES_RATE",
             "ROLL", "PITCH", "YAW", "ROLL_RATE", "PITCH_RATE", "YAW_RATE",
             "N_POS", "E_POS", "ALTITUDE", "GROUND_ALTITUDE")   # helicopter_dynamics.py:23-25


try:   # gymnasium.vector.VectorEnv lineage when gymnasium is installed (optional)
    from gymnasium.vector import VectorEnv as _VectorEnv
    _VEC_BASES = (_VectorEnv,)
except ImportError:
    _VEC_BASES = (object,)


class HeliVecEnv(*_VEC_BASES):
    """N independent helicopters (one `hg_env` handle) on one GPU.

    task: "hover" (HeliHover), "forward_flight" (HeliForwardFlight) or "heli" (Heli, reward 0).
    autoreset: finished envs are reset inside the step kernel; the returned observation row is
      the reset observation and the terminal one is in info["final_obs"] (rows of
      info["reset_index"]).  With autoreset=False, finished envs keep integrating until reset().
    env_offset: global id of env 0 (multi-GPU sharding keeps the noise stream of each env fixed).
    """

    metadata = {"render.modes": [], "video.frames_per_second": config.FPS}   # helicopter.py:29-32

    def __init__(self, num_envs, task="hover", dt=config.DT, heli_name="aw109", seed=0, device=None,
                 autoreset=True, env_offset=0, max_time=None, target=None, trim_cond=None,
                 turbulence_level=None, reset_mode="template", autoreset_mode="same_step",
                 max_episode_steps=None, terrain=None, specialize=False):
        import torch
        self.torch = torch
        self.lib = _abi.load_library()
        if not torch.cuda.is_available():
            raise _abi.HeliGymError("HeliVecEnv needs a HIP device (no CPU fallback)")
        self.device = torch.device(device if device is not None else f"cuda:{torch.cuda.current_device()}")
        self.num_envs = int(num_envs)
        self.task = task
        self.dt = float(dt)
        self.autoreset = bool(autoreset)
        self.cfg, doc = config.make_config(task=task, dt=dt, heli_name=heli_name, max_time=max_time,
                                           target=target, trim_cond=trim_cond, autoreset=autoreset,
                                           seed=seed, env_offset=env_offset,
                                           turbulence_level=turbulence_level, reset_mode=reset_mode,
                                           autoreset_mode=autoreset_mode, max_episode_steps=max_episode_steps)
        self.reset_mode = reset_mode
        self.autoreset_mode = autoreset_mode
        self.max_episode_steps = max_episode_steps
        # terrain: the airframe document's map, or a path / uint16 samples / float heights in ft
        if terrain is None or isinstance(terrain, str):
            u16 = config.load_terrain(doc) if terrain is None else config.read_terrain(terrain)
            self.terrain_ft = config.terrain_ft(u16, self.cfg.af.env_MAX_GR_ALT)
        else:
            t = np.asarray(terrain)
            self.terrain_ft = (config.terrain_ft(t, self.cfg.af.env_MAX_GR_ALT) if t.dtype == np.uint16
                               else np.ascontiguousarray(t, dtype=np.float64))
        if self.terrain_ft.ndim != 2:
            raise ValueError("terrain must be a 2-D map")
        self._target = dict(config.DEFAULT_TARGETS[task])
        self._target.update(target or {})
        self._trim_cond = config.fill_trim(_abi.hg_trim_cond(), trim_cond)
        self.max_time = self.cfg.max_time
        h = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            _abi.check(self.lib.hg_create(ctypes.byref(self.cfg), self.terrain_ft.ctypes.data,
                                          self.terrain_ft.shape[0], self.terrain_ft.shape[1],
                                          self.num_envs, ctypes.byref(h)), self.lib)
        self._h = h
        self._specialized = bool(self.lib.hg_set_specialized(h, 1))
        if specialize and not self._specialized:
            self.specialize()
        N, dev = self.num_envs, self.device
        f32, u8, i32 = torch.float32, torch.uint8, torch.int32
        self.obs = torch.empty((N, _abi.HG_N_OBS), dtype=f32, device=dev)
        self.reward = torch.empty((N,), dtype=f32, device=dev)
        self.terminated_u8 = torch.empty((N,), dtype=u8, device=dev)
        self.truncated_u8 = torch.empty((N,), dtype=u8, device=dev)
        # info bits and reset info alternate between two buffer sets from step to step, so that the
        # lazily evaluated info of step() stays valid until the step after next (no copies, no sync)
        self._sets = [dict(info=torch.zeros((N,), dtype=u8, device=dev),
                           index=torch.empty((N,), dtype=i32, device=dev),
                           final=torch.empty((N, _abi.HG_N_OBS), dtype=f32, device=dev)) for _ in range(2)]
        # reset counts rotate over three buffers: step k counts into ring[k % 3], which step k-1
        # zeroed from inside its kernel (hg_step_chained: no separate zeroing launch), and zeroes
        # ring[(k + 1) % 3]; step k's count is so readable until the step after next
        self._count_ring = torch.zeros((3,), dtype=i32, device=dev)
        self._ring_views = [self._count_ring[j:j + 1] for j in range(3)]
        self._p_ring = [v.data_ptr() for v in self._ring_views]
        # the per-step host path passes plain addresses (no per-call tensor -> pointer conversions)
        # and reads the current stream through torch's raw-stream accessor
        self._dev_index = dev.index if dev.index is not None else torch.cuda.current_device()
        self._raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None)
        self._p_obs, self._p_rew = self.obs.data_ptr(), self.reward.data_ptr()
        self._p_term, self._p_trunc = self.terminated_u8.data_ptr(), self.truncated_u8.data_ptr()
        self._term_b, self._trunc_b = self.terminated_u8.view(torch.bool), self.truncated_u8.view(torch.bool)
        self._act_shape = (N, _abi.HG_N_ACT)
        for b in self._sets:
            b["count"] = self._ring_views[0]
            b["p"] = tuple(b[k].data_ptr() for k in ("info", "index", "final"))
            b["thunks"] = self._info_thunks(b)
            b["thunks_rows"] = self._info_thunks(b, rows=True)
            # step()'s hg_step_rows arguments after the actions, before the stream
            b["rows_args"] = (self._p_obs, self._p_rew, self._p_term, self._p_trunc, b["p"][0], None, b["p"][2])
        self._f32 = torch.float32
        self._step_rows = self.lib.hg_step_rows
        # step()'s direct path: same-step auto-reset with reset info (what _launch(rows=True) does),
        # and a raw-stream accessor to read the current stream with
        self._rows_fast = self.autoreset and self.autoreset_mode == "same_step" and self._raw_stream is not None
        self._gen = 0
        self._use_set(0)
        # gymnasium.vector's convention: one env's spaces (helicopter.py:56-57) and the batched ones
        self.single_observation_space = _make_box(-np.inf, np.inf, (_abi.HG_N_OBS,))
        self.single_action_space = _make_box(-1.0, 1.0, (_abi.HG_N_ACT,))
        self.observation_space = _make_box(-np.inf, np.inf, (N, _abi.HG_N_OBS))
        self.action_space = _make_box(-1.0, 1.0, (N, _abi.HG_N_ACT))
        self.normalizers = {                                                     # helicopter.py:63-68
            "t": float(np.sqrt(2 * self.cfg.af.mr_R / self.cfg.af.env_GRAV)),
            "x": 2 * self.cfg.af.mr_R,
            "v": float(np.sqrt(2 * self.cfg.af.mr_R * self.cfg.af.env_GRAV)),
            "a": self.cfg.af.env_GRAV,
        }

    # ------------------------------------------------------------------ plumbing
    def _use_set(self, g):
        b = self._sets[g & 1]
        b["count"] = self._ring_views[g % 3]
        self.info_u8, self.reset_count, self.reset_index, self.final_obs = b["info"], b["count"], b["index"], b["final"]
        return b

    def _stream(self):
        if self._raw_stream is not None:
            return ctypes.c_void_p(self._raw_stream(self._dev_index))
        return ctypes.c_void_p(self.torch.cuda.current_stream(self.device).cuda_stream)

    def _info_thunks(self, b, rows=False):
        """The lazy info fields of a step that used buffer set b: key -> f(info).  rows: the step
        went through hg_step_rows (reset envs flagged by HG_INFO_RESET, terminal observations at
        their own rows of b["final"]), else its reset info is the compacted one."""
        bits, index, final = b["info"], b["index"], b["final"]
        th = {"failed": lambda i: (bits & _abi.HG_INFO_FAILED) != 0,
              "successed": lambda i: (bits & _abi.HG_INFO_SUCCESSED) != 0,
              "time_up": lambda i: (bits & _abi.HG_INFO_TIME_UP) != 0,
              "success_step": lambda i: (bits & _abi.HG_INFO_SUCCESS_STEP) != 0}
        if self.autoreset and self.autoreset_mode == "same_step" and rows:
            def resets(i):   # (sorted env ids, their terminal observations); one nonzero per step
                r = getattr(i, "_resets", None)
                if r is None:
                    idx = self.torch.nonzero(bits & _abi.HG_INFO_RESET).flatten()
                    r = i._resets = (idx, final.index_select(0, idx))
                return r
            th["reset_index"] = lambda i: resets(i)[0]
            th["final_obs"] = lambda i: resets(i)[1]
        elif self.autoreset and self.autoreset_mode == "same_step":
            def resets(i):   # (sorted env ids, their terminal observations); one host read per step
                r = getattr(i, "_resets", None)
                if r is None:
                    k = int(b["count"].item())   # this set's step's ring slot
                    idx = index[:k].long()
                    order = self.torch.argsort(idx)
                    r = i._resets = (idx[order], final[:k][order])
                return r
            th["reset_index"] = lambda i: resets(i)[0]
            th["final_obs"] = lambda i: resets(i)[1]
        return th

    def _check(self, rc):
        return _abi.check(rc, self.lib)

    def close(self):
        if getattr(self, "_h", None):
            self.lib.hg_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ------------------------------------------------------------------ gym surface
    def reset(self, seed=None, options=None, mask=None):
        """Heli.reset (helicopter.py:208-217) for all envs, or for the envs where `mask` != 0.
        Returns (obs [N,17], info) like the reference (obs rows of unmasked envs untouched)."""
        m = None
        if mask is not None:
            m = self.torch.as_tensor(mask, device=self.device).to(self.torch.uint8).contiguous()
        self._check(self.lib.hg_reset(self._h, _ptr(m), _ptr(self.obs), self._stream()))
        tr = self.template()
        N = self.num_envs
        info = {"failed": self.torch.full((N,), bool(tr["failed"]), device=self.device),
                "successed": self.torch.zeros((N,), dtype=self.torch.bool, device=self.device),
                "time_up": self.torch.zeros((N,), dtype=self.torch.bool, device=self.device)}
        return self.obs, info

    def step_async(self, actions, eta=None, with_reset_info=True, obs_out=None):
        """Launch one step on the current stream and return immediately (no host sync).
        actions: float32 [N,4] device tensor.  eta: optional float32 [N,3] injected turbulence noise
        (already scaled by 1/sqrt(dt)), else in-kernel Philox.  obs_out: optional float32 [N,17]
        device tensor (16-byte aligned) the observations go to instead of `self.obs` (double
        buffering, e.g. while a previous step's observations are being gathered)."""
        self._launch(actions, eta, with_reset_info, obs_out)

    def _launch(self, actions, eta, with_reset_info, obs_out, rows=False):
        """step_async's launch; returns the buffer set the step's info went to.  rows: the reset
        info uncompacted (hg_step_rows, step()'s path), else compacted (hg_step_chained)."""
        a = actions
        if a.dtype != self.torch.float32 or not a.is_contiguous() or a.device != self.device:
            a = a.to(device=self.device, dtype=self.torch.float32).contiguous()
        if a.shape != self._act_shape:
            raise ValueError(f"actions must be [{self.num_envs}, 4], got {tuple(a.shape)}")
        e = None
        if eta is not None:
            e = eta.to(device=self.device, dtype=self.torch.float32).contiguous()
            if tuple(e.shape) != (self.num_envs, 3):
                raise ValueError("eta must be [N, 3]")
        p_obs = self._p_obs
        if obs_out is not None:
            if (obs_out.dtype != self.torch.float32 or obs_out.device != self.device or not obs_out.is_contiguous()
                    or tuple(obs_out.shape) != (self.num_envs, _abi.HG_N_OBS)):
                raise ValueError(f"obs_out must be a contiguous float32 [{self.num_envs}, 17] tensor on {self.device}")
            p_obs = obs_out.data_ptr()
        self._keep = (a, e, obs_out)
        self._gen += 1
        b = self._use_set(self._gen)
        p = b["p"]
        rs = with_reset_info and self.autoreset and self.autoreset_mode == "same_step"
        g = self._gen
        if not rs or rows:
            # only a compacted step (step_async with reset info) fills these; after any other step
            # they would hold another step's data
            self.reset_count = self.reset_index = self.final_obs = None
        if rs and rows:
            rc = self.lib.hg_step_rows(self._h, a.data_ptr(), p_obs, self._p_rew, self._p_term, self._p_trunc, p[0],
                                       None if e is None else e.data_ptr(), p[2], self._stream())
        elif rs:
            rc = self.lib.hg_step_chained(self._h, a.data_ptr(), p_obs, self._p_rew, self._p_term, self._p_trunc,
                                          p[0], None if e is None else e.data_ptr(), self._p_ring[g % 3], p[1], p[2],
                                          self._p_ring[(g + 1) % 3], self._stream())
        else:
            rc = self.lib.hg_step(self._h, a.data_ptr(), p_obs, self._p_rew, self._p_term, self._p_trunc, p[0],
                                  None if e is None else e.data_ptr(), None, None, None, self._stream())
        if rc:
            self._check(rc)
        return b

    def step(self, actions, eta=None):
        """Heli.step (helicopter.py:192-206) for all envs: (obs, reward, terminated, truncated, info).
        Returned tensors are the env's buffers, overwritten by the next step.  `info` is evaluated
        lazily: a field costs its device ops (and, for the same-step reset info, a read of the reset
        count) only when it is read, which must happen before the step after next.  The reset info
        comes uncompacted (hg_step_rows: the reset envs' info bytes carry HG_INFO_RESET and their
        terminal observations sit at their own rows), so the step is the plain kernel launch."""
        a = actions
        # the common call (a float32 [N,4] contiguous tensor on the env's device, in-kernel noise) goes
        # straight to hg_step_rows with the buffer set's addresses packed at construction: the host
        # cost per call is then the launch's, not the argument handling's
        if (eta is None and self._rows_fast and a.dtype is self._f32 and a.is_contiguous()
                and a.shape == self._act_shape and a.get_device() == self._dev_index):
            g = self._gen = self._gen + 1
            b = self._sets[g & 1]
            self.info_u8 = b["info"]
            if self.reset_count is not None:   # (only a compacted step fills these)
                self.reset_count = self.reset_index = self.final_obs = None
            self._keep = (a, None, None)
            rc = self._step_rows(self._h, a.data_ptr(), *b["rows_args"], self._raw_stream(self._dev_index))
            if rc:
                self._check(rc)
            return self.obs, self.reward, self._term_b, self._trunc_b, LazyInfo(b["thunks_rows"], self, g)
        b = self._launch(actions, eta, True, None, rows=True)
        return self.obs, self.reward, self._term_b, self._trunc_b, LazyInfo(b["thunks_rows"], self, self._gen)

    # ------------------------------------------------------------------ setters (helicopter.py:89-111)
    def set_max_time(self, max_time=None):
        self.max_time = config.DEFAULT_MAX_TIME if max_time is None else float(max_time)
        self._check(self.lib.hg_set_max_time(self._h, self.max_time))

    def set_target(self, target=None):
        self._target.update(target or {})
        tg = _abi.hg_target()
        config.fill_target(tg, self._target)
        self._check(self.lib.hg_set_target(self._h, ctypes.byref(tg)))

    def get_target(self):
        return dict(self._target)

    def set_specialized(self, enable=True):
        """Allow / forbid the step kernel with the default airframe's constants compiled in
        (csrc/baked.h; bitwise-identical results).  Returns whether it is in use."""
        rc = self.lib.hg_set_specialized(self._h, 1 if enable else 0)
        if rc < 0:
            self._check(rc)
        self._specialized = bool(rc)
        return self._specialized

    def set_retrim_overlap(self, enable=True):
        """reset_mode="retrim": with next-step auto-reset, trim the episodes a step ends while the next
        step runs (True, the default; False: always serial).  enable=2 also trims, with same-step
        auto-reset, a step's resets in the step's own launch as soon as each env's step is done (opt-in:
        bitwise the serial results but slower on MI355X).  hg_set_retrim_overlap.  Returns whether the
        next-step overlap is in effect."""
        mode = 2 if (enable == 2 and enable is not True) else (1 if enable else 0)
        rc = self.lib.hg_set_retrim_overlap(self._h, mode)
        if rc < 0:
            self._check(rc)
        return bool(rc)

    @property
    def specialized(self):
        """True when steps run a constant-specialised kernel: the library's own for the default AW109
        airframe (its constants compiled in; every step and rollout, with or without the optional
        features), or a run-time specialised one for any other airframe (specialize())."""
        return self._specialized

    def specialize(self):
        """Step this env with a kernel specialised for its airframe's constants (heligym_amd._rtc:
        compiled with hipcc on the first request for these constants, ~4 s, then cached), the way the
        default airframe always is: per-step launches with in-kernel noise use it, results bitwise
        those of the generic kernel.  Returns whether a specialised kernel is in use."""
        if self._specialized:
            return True
        from . import _rtc
        rows, cols = self.terrain_ft.shape
        path, img = _rtc.build(self.lib, self.cfg, rows, cols, self.cfg.task)
        buf = ctypes.create_string_buffer(img, len(img))
        rc = self.lib.hg_load_specialized(self._h, path.encode(), self.cfg.task, buf, len(img))
        if rc < 0:
            self._check(rc)
        self._specialized = bool(rc)
        return self._specialized

    def set_trim_cond(self, trim_cond=None):
        cur = self.get_trim_cond()
        cur.update(trim_cond or {})
        tc = _abi.hg_trim_cond()
        self._trim_cond = config.fill_trim(tc, cur)
        self._check(self.lib.hg_set_trim_cond(self._h, ctypes.byref(tc)))

    def get_trim_cond(self):
        import copy
        return copy.deepcopy(self._trim_cond)

    def template(self):
        r = _abi.hg_trim_result()
        self._check(self.lib.hg_get_template(self._h, ctypes.byref(r)))
        return {"state": np.array(r.state), "action": np.array(r.action), "obs": np.array(r.obs),
                "state_dots": np.array(r.state_dots), "residual": r.residual,
                "iterations": r.iterations, "failed": bool(r.failed)}

    # ------------------------------------------------------------------ state access
    def get_state(self):
        """(state [N,27] float32, counters [N,3] int32): heli 18 | wind 5 | carry 4.

        The rotor azimuths (columns 2, 3) are reconstructed from a per-env record (each step adds
        dt * Omega and wraps, bitwise what the step would have carried); the cost is one add-and-wrap
        per step since the env's last reset, set_state or get_state, and each call re-anchors the
        records, so a run that reads its state now and then keeps every read short."""
        t = self.torch
        s = t.empty((self.num_envs, _abi.HG_STATE_COLS), dtype=t.float32, device=self.device)
        c = t.empty((self.num_envs, _abi.HG_COUNTER_COLS), dtype=t.int32, device=self.device)
        self._check(self.lib.hg_get_state(self._h, _ptr(s), _ptr(c), self._stream()))
        return s, c

    def set_state(self, state=None, counters=None):
        t = self.torch
        s = None if state is None else t.as_tensor(state, device=self.device, dtype=t.float32).contiguous()
        c = None if counters is None else t.as_tensor(counters, device=self.device, dtype=t.int32).contiguous()
        if s is not None and tuple(s.shape) != (self.num_envs, _abi.HG_STATE_COLS):
            raise ValueError("state must be [N, 27]")
        if c is not None and tuple(c.shape) != (self.num_envs, _abi.HG_COUNTER_COLS):
            raise ValueError("counters must be [N, 3]")
        self._check(self.lib.hg_set_state(self._h, _ptr(s), _ptr(c), self._stream()))
        self._keep_state = (s, c)

    def rollout(self, actions, eta=None, out=None):
        """Open-loop rollout (hg_rollout): actions [K,N,4] applied over K consecutive steps in one
        launch, identical to K step() calls.  Returns (obs [K,N,17], reward [K,N], terminated,
        truncated [K,N] bool, info bits [K,N] uint8) device tensors (`out` buffers are reused if
        given, as returned by a previous call)."""
        t = self.torch
        a = actions
        if a.dtype != t.float32 or not a.is_contiguous() or a.device != self.device:
            a = a.to(device=self.device, dtype=t.float32).contiguous()
        if a.ndim != 3 or tuple(a.shape[1:]) != (self.num_envs, _abi.HG_N_ACT):
            raise ValueError(f"actions must be [K, {self.num_envs}, 4], got {tuple(a.shape)}")
        K, N = a.shape[0], self.num_envs
        e = None
        if eta is not None:
            e = eta.to(device=self.device, dtype=t.float32).contiguous()
            if tuple(e.shape) != (K, N, 3):
                raise ValueError("eta must be [K, N, 3]")
        if out is None or out[0].shape[0] != K:
            out = (t.empty((K, N, _abi.HG_N_OBS), dtype=t.float32, device=self.device),
                   t.empty((K, N), dtype=t.float32, device=self.device),
                   t.empty((K, N), dtype=t.uint8, device=self.device),
                   t.empty((K, N), dtype=t.uint8, device=self.device),
                   t.empty((K, N), dtype=t.uint8, device=self.device))
        obs, rew, term, trunc, info = out
        self._keep = (a, e)
        self._check(self.lib.hg_rollout(self._h, _ptr(a), K, _ptr(obs), _ptr(rew), _ptr(term), _ptr(trunc),
                                        _ptr(info), _ptr(e), self._stream()))
        return out

    def trim_batch(self, wind_ned):
        """Device batched trim (hg_trim_batch) of this env's trim condition against each row of
        `wind_ned` [K,3] (ft/s NED): the reset the reference computes from its second episode on.
        Returns dict of float32 device tensors state [K,18], action [K,4], obs [K,17] and int32
        status [K] (0 or HG_E_TRIM)."""
        t = self.torch
        w = t.as_tensor(wind_ned, device=self.device, dtype=t.float32).contiguous()
        if w.ndim != 2 or w.shape[1] != 3:
            raise ValueError("wind_ned must be [K, 3]")
        K = w.shape[0]
        out = {"state": t.empty((K, _abi.HG_N_HELI), dtype=t.float32, device=self.device),
               "action": t.empty((K, _abi.HG_N_ACT), dtype=t.float32, device=self.device),
               "obs": t.empty((K, _abi.HG_N_OBS), dtype=t.float32, device=self.device),
               "status": t.full((K,), -99, dtype=t.int32, device=self.device)}
        self._check(self.lib.hg_trim_batch(self._h, _ptr(w), K, _ptr(out["state"]), _ptr(out["action"]),
                                           _ptr(out["obs"]), _ptr(out["status"]), self._stream()))
        self._keep_trim = w
        return out

    def trim_conds(self, conds, wind_ned=None):
        """Device trims (hg_trim_conds_batch) for a list of trim-condition dicts (the reference's
        set_trim_cond keys, missing keys from the defaults), against `wind_ned` [K,3] or the mean
        wind.  Returns dict of device tensors state [K,18], action [K,4], obs [K,17], status [K]."""
        t = self.torch
        K = len(conds)
        arr = (_abi.hg_trim_cond * K)()
        for j, c in enumerate(conds):
            config.fill_trim(arr[j], c)
        w = None
        if wind_ned is not None:
            w = t.as_tensor(wind_ned, device=self.device, dtype=t.float32).contiguous()
            if tuple(w.shape) != (K, 3):
                raise ValueError("wind_ned must be [K, 3]")
        out = {"state": t.empty((K, _abi.HG_N_HELI), dtype=t.float32, device=self.device),
               "action": t.empty((K, _abi.HG_N_ACT), dtype=t.float32, device=self.device),
               "obs": t.empty((K, _abi.HG_N_OBS), dtype=t.float32, device=self.device),
               "status": t.full((K,), -99, dtype=t.int32, device=self.device)}
        self._check(self.lib.hg_trim_conds_batch(self._h, arr, K, _ptr(w), _ptr(out["state"]), _ptr(out["action"]),
                                                 _ptr(out["obs"]), _ptr(out["status"]), self._stream()))
        return out

    def set_trim_conds(self, conds):
        """Batched set_trim_cond (helicopter.py:101-103): env i resets to the trim of conds[i] (a
        list of N dicts).  Trims all on the device; raises if any trim fails.  `None` reverts to
        the shared condition (set_trim_cond)."""
        if conds is None:
            self._check(self.lib.hg_set_reset_templates(self._h, None, self._stream()))
            return None
        if len(conds) != self.num_envs:
            raise ValueError(f"need {self.num_envs} trim conditions, got {len(conds)}")
        r = self.trim_conds(conds)
        bad = (r["status"] != 0).nonzero().flatten()
        if len(bad):
            raise _abi.HeliGymError(f"trim failed for envs {bad[:10].tolist()}")
        obs = r["obs"]
        tmpl = self.torch.cat([r["state"], obs[:, 4:7], obs[:, 16:17], obs], dim=1).contiguous()
        self._check(self.lib.hg_set_reset_templates(self._h, _ptr(tmpl), self._stream()))
        return r

    def retrim_failures(self):
        """Auto-resets in reset_mode="retrim" whose trim did not converge (they got the template)."""
        c = ctypes.c_int64()
        self._check(self.lib.hg_retrim_failures(self._h, ctypes.byref(c)))
        return c.value

    LAUNCH_KINDS = ("steps", "overlapped_retrim", "specialized", "helper", "lone_wave", "bulk")

    def debug_launches(self):
        """Diagnostic: host-side launch counts of this env (hg_debug_launches): step calls, steps that
        held the previous step's re-trims, and the kernel kinds that ran."""
        out = (ctypes.c_int64 * 6)()
        self._check(self.lib.hg_debug_launches(self._h, out))
        return dict(zip(self.LAUNCH_KINDS, (int(v) for v in out)))

    def retrim_solve_stats(self):
        """Diagnostic: (solves tried with the host trim's pivot order, of them re-solved with the pivot
        search after failing the residual test) over the device trims of this env (hg_debug_retrim_solves)."""
        c = (ctypes.c_int64 * 2)()
        self._check(self.lib.hg_debug_retrim_solves(self._h, c))
        return int(c[0]), int(c[1])

    def retrim_invalid_jobs(self):
        """Diagnostic: re-trim job records that named no env (skipped); 0 in a correct run."""
        c = ctypes.c_int64()
        self._check(self.lib.hg_debug_retrim_invalid(self._h, ctypes.byref(c)))
        return c.value

    def debug_eta(self, out=None):
        """Diagnostic: the turbulence noise [N,3] (scaled by 1/sqrt(dt), wind_dynamics.py:49-52) each
        env's next step draws in-kernel, from its current counters (hg_debug_eta).  Injecting it as
        `eta` gives bitwise the in-kernel step."""
        t = self.torch
        if out is None:
            out = t.empty((self.num_envs, 3), dtype=t.float32, device=self.device)
        elif (tuple(out.shape) != (self.num_envs, 3) or out.dtype != t.float32 or out.device != t.device(self.device)
              or not out.is_contiguous()):
            # the kernel writes 3 * num_envs floats: never hand it a buffer that does not hold them
            raise ValueError(f"debug_eta: out must be a contiguous float32 ({self.num_envs}, 3) tensor on "
                             f"{self.device}, got {tuple(out.shape)} {out.dtype} on {out.device}")
        self._check(self.lib.hg_debug_eta(self._h, _ptr(out), self._stream()))
        return out

    def random_actions(self, out, seed, step, lo=-1.0, hi=1.0):
        self._check(self.lib.hg_random_actions(self._h, _ptr(out), int(seed), int(step), float(lo),
                                               float(hi), self._stream()))
        return out
