"""heligym_amd — MI355X-native vectorised heli-gym (HeliHover / HeliForwardFlight) step().

Drop-in for the reference's environment surface (ugurcanozalp/heli-gym v2,
heligym/__init__.py:1-18 and heligym/envs/*): `Heli`, `HeliHover`, `HeliForwardFlight`
single-env classes with the reference's reset()/step()/setters, and `HeliVecEnv` for N envs per
GPU.  Every step runs in the gfx950 kernels of libheligym_amd.so.
"""
from ._abi import HeliGymError, load_library  # noqa: F401
from .config import DT, FPS, make_config  # noqa: F401
from .envs import Heli, HeliForwardFlight, HeliHover  # noqa: F401
from .vector import OBS_NAMES, HeliVecEnv  # noqa: F401

__all__ = ["Heli", "HeliHover", "HeliForwardFlight", "HeliVecEnv", "OBS_NAMES", "register_envs",
           "make_vec", "HeliGymError"]

# gymnasium ids of the reference registry (heligym/__init__.py:4-18) -> task
ENV_IDS = {"Heli-v0": "heli", "HeliHover-v0": "hover", "HeliForwardFlight-v0": "forward_flight"}
MAX_EPISODE_STEPS = 5000   # heligym/__init__.py:4-18
REWARD_THRESHOLD = 0.95


def make_vec(env_id, num_envs, autoreset_mode="next_step", max_episode_steps=MAX_EPISODE_STEPS,
             reset_mode="retrim", **kwargs):
    """`gymnasium.make_vec(env_id, num_envs)` for the heligym ids: one batched GPU env with the
    registry's TimeLimit (max_episode_steps=5000), gymnasium's vector autoreset default (next step)
    and the reference's resets: every reset re-trimmed against the env's last wind, as N reference
    envs in a gymnasium vector env reset (helicopter.py:208-212; reset_mode="template" is the
    faster mean-wind template); kwargs go to HeliVecEnv (dt, seed, device,
    trim_cond, ...)."""
    if env_id not in ENV_IDS:
        raise ValueError(f"unknown env id {env_id!r}; one of {sorted(ENV_IDS)}")
    env = HeliVecEnv(num_envs, task=ENV_IDS[env_id], autoreset=True, autoreset_mode=autoreset_mode,
                     max_episode_steps=max_episode_steps, reset_mode=reset_mode, **kwargs)
    env.spec_id = env_id
    env.reward_threshold = REWARD_THRESHOLD
    return env


def register_envs():
    """gymnasium ids like heligym/__init__.py:4-18 (plus HeliForwardFlight-v0, which the reference
    defines but never registers).  No-op when gymnasium is not installed."""
    try:
        from gymnasium.envs.registration import register
    except ImportError:
        return False
    import functools
    for name, cls in (("Heli-v0", "Heli"), ("HeliHover-v0", "HeliHover"),
                      ("HeliForwardFlight-v0", "HeliForwardFlight")):
        kw = dict(id=name, entry_point=f"heligym_amd.envs:{cls}", max_episode_steps=MAX_EPISODE_STEPS,
                  reward_threshold=REWARD_THRESHOLD, nondeterministic=False)
        try:
            register(vector_entry_point=functools.partial(make_vec, name), **kw)
        except TypeError:   # gymnasium < 1.0 has no vector entry points
            register(**kw)
    return True
