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
           "HeliGymError"]


def register_envs():
    """gymnasium ids like heligym/__init__.py:4-18 (plus HeliForwardFlight-v0, which the reference
    defines but never registers).  No-op when gymnasium is not installed."""
    try:
        from gymnasium.envs.registration import register
    except ImportError:
        return False
    for name, cls in (("Heli-v0", "Heli"), ("HeliHover-v0", "HeliHover"),
                      ("HeliForwardFlight-v0", "HeliForwardFlight")):
        register(id=name, entry_point=f"heligym_amd.envs:{cls}", max_episode_steps=5000,
                 reward_threshold=0.95, nondeterministic=False)
    return True
