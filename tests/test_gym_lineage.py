"""gymnasium lineage of the drop-in classes (helicopter.py:28: class Heli(gym.Env, EzPickle)) and
the registry wiring (heligym/__init__.py:4-18).  gymnasium is not installed in this image, so a
minimal stand-in package (Env, EzPickle, spaces.Box, vector.VectorEnv, registration.register) is
put on sys.path in a subprocess; only the class wiring is checked (constructing an env needs a
GPU).  Without gymnasium the same classes are plain duck-typed ones."""
import os
import subprocess
import sys
import textwrap

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

STUB = {
    "gymnasium/__init__.py": "class Env:\n    metadata = {}\nfrom . import spaces, utils, vector  # noqa\n",
    "gymnasium/utils/__init__.py": "class EzPickle:\n    def __init__(self, *a, **k):\n        self._ezpickle_args = a\n",
    "gymnasium/spaces/__init__.py": textwrap.dedent("""
        import numpy as np
        class Box:
            def __init__(self, low, high, shape=None, dtype=np.float32):
                self.shape, self.dtype = tuple(shape), np.dtype(dtype)
        """),
    "gymnasium/vector/__init__.py": "class VectorEnv:\n    pass\n",
    "gymnasium/envs/__init__.py": "",
    "gymnasium/envs/registration.py": "CALLS = []\ndef register(**kw):\n    CALLS.append(kw)\n",
}

CHECK = textwrap.dedent("""
    import gymnasium, heligym_amd
    from gymnasium.envs import registration
    from heligym_amd import Heli, HeliHover, HeliForwardFlight, HeliVecEnv
    from heligym_amd.vector import _make_box
    assert issubclass(HeliHover, gymnasium.Env) and issubclass(HeliForwardFlight, gymnasium.utils.EzPickle)
    assert issubclass(Heli, gymnasium.Env) and issubclass(HeliVecEnv, gymnasium.vector.VectorEnv)
    assert isinstance(_make_box(-1.0, 1.0, (4,)), gymnasium.spaces.Box)
    assert heligym_amd.register_envs() is True
    ids = sorted(c["id"] for c in registration.CALLS)
    assert ids == ["Heli-v0", "HeliForwardFlight-v0", "HeliHover-v0"], ids
    for c in registration.CALLS:
        assert c["max_episode_steps"] == 5000 and c["reward_threshold"] == 0.95
        assert c["entry_point"].startswith("heligym_amd.envs:") and callable(c["vector_entry_point"])
    print("ok")
    """)


def test_gymnasium_lineage_with_stand_in(tmp_path):
    for rel, text in STUB.items():
        p = tmp_path / rel
        p.parent.mkdir(parents=True, exist_ok=True)
        p.write_text(text)
    env = dict(os.environ, PYTHONPATH=os.pathsep.join([str(tmp_path), os.path.join(ROOT, "heli-gym_amd")]))
    r = subprocess.run([sys.executable, "-c", CHECK], capture_output=True, text=True, env=env, timeout=120)
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), r.stderr[-2000:]


def test_without_gymnasium_classes_are_plain():
    import heligym_amd
    from heligym_amd import HeliHover, HeliVecEnv
    try:
        import gymnasium  # noqa: F401
    except ImportError:
        assert HeliHover.__mro__[-1] is object and HeliVecEnv.__bases__ == (object,)
        assert heligym_amd.register_envs() is False
