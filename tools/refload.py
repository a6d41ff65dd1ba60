"""Load the read-only reference heli-gym dynamics in THIS container (golden generation only).

Test infrastructure, never shipped and never imported on the GPU box: it reads
`/root/reference` at run time.  `import heligym` itself is unusable here (it needs
gymnasium, its renderer package may `os.execv` the interpreter and `Heli.__init__`
opens an OpenGL window via a prebuilt `libHeligym.so`, which is never loaded), so
this module builds a synthetic package whose `__path__` is the reference's
`heligym/envs` directory and pre-registers inert stand-ins for the three
non-physics imports:

* `imageio.imread`  -> Pillow decode of the terrain PNG (uint16, 1024x1024), the
  same array imageio's Pillow plugin returns
  (used at /root/reference/heligym/envs/dynamics/helicopter_dynamics.py:39-42);
* `gymnasium` (`Env`, `spaces.Box`, `utils.EzPickle`, `utils.seeding`) -- only
  class scaffolding for /root/reference/heligym/envs/helicopter.py:10-12,28,48,56-57;
* `<pkg>.renderer.api.Renderer` -> no-op object (helicopter.py:16,70-84).

Physics, trim, reward and flag code all run unmodified from the reference files.
"""
import importlib
import os
import sys
import types

import numpy as np

REF_ROOT = os.environ.get("HELIGYM_REFERENCE", "/root/reference")
ENVS_DIR = os.path.join(REF_ROOT, "heligym", "envs")
RESOURCE_DIR = os.path.join(ENVS_DIR, "renderer", "resources")
PKG = "_hgref"


class _NoOp:
    def __init__(self, *a, **k):
        pass

    def __getattr__(self, name):
        if name.startswith("__"):
            raise AttributeError(name)
        return lambda *a, **k: _NoOp()

    def get_fps(self):
        return 0.0


def _install_stubs():
    if PKG in sys.modules:
        return
    # imageio stand-in (Pillow decode)
    from PIL import Image
    imageio = types.ModuleType("imageio")
    imageio.imread = lambda p: np.asarray(Image.open(p))
    sys.modules.setdefault("imageio", imageio)

    # gymnasium scaffolding
    gym = types.ModuleType("gymnasium")
    spaces = types.ModuleType("gymnasium.spaces")
    utils = types.ModuleType("gymnasium.utils")

    class Env:
        pass

    class Box:
        def __init__(self, low, high, shape=None, dtype=np.float32):
            self.low, self.high, self.shape, self.dtype = low, high, shape, dtype

    class EzPickle:
        def __init__(self, *a, **k):
            pass

    spaces.Box = Box
    utils.EzPickle = EzPickle
    utils.seeding = types.SimpleNamespace()
    gym.Env = Env
    gym.spaces = spaces
    gym.utils = utils
    sys.modules["gymnasium"] = gym
    sys.modules["gymnasium.spaces"] = spaces
    sys.modules["gymnasium.utils"] = utils

    os.environ["HELIGYM_RESOURCE_DIR"] = RESOURCE_DIR

    pkg = types.ModuleType(PKG)
    pkg.__path__ = [ENVS_DIR]
    sys.modules[PKG] = pkg
    rnd = types.ModuleType(PKG + ".renderer")
    rnd.__path__ = []
    api = types.ModuleType(PKG + ".renderer.api")
    api.Renderer = _NoOp
    rnd.api = api
    sys.modules[PKG + ".renderer"] = rnd
    sys.modules[PKG + ".renderer.api"] = api


def load():
    """Return a namespace with the reference modules (dynamics + envs)."""
    _install_stubs()
    ns = types.SimpleNamespace()
    ns.lookup = importlib.import_module(PKG + ".dynamics.lookup")
    ns.utils = importlib.import_module(PKG + ".dynamics.utils")
    ns.kinematic = importlib.import_module(PKG + ".dynamics.kinematic")
    ns.dynamics = importlib.import_module(PKG + ".dynamics.dynamics")
    ns.helicopter_dynamics = importlib.import_module(PKG + ".dynamics.helicopter_dynamics")
    ns.wind_dynamics = importlib.import_module(PKG + ".dynamics.wind_dynamics")
    ns.helicopter = importlib.import_module(PKG + ".helicopter")
    ns.tasks = importlib.import_module(PKG + ".helicopter_with_tasks")
    return ns
