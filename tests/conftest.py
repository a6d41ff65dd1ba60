import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "heli-gym_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")


def load_golden(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


def trim_dict(c):
    """Golden trim-condition vector -> trim_cond dict (tools/gen_goldens.py:trim_vec)."""
    return {"yaw": float(c[0]), "yaw_rate": float(c[1]), "ned_vel": [float(v) for v in c[2:5]],
            "gr_alt": float(c[5]), "xy": [float(c[6]), float(c[7])], "psi_mr": float(c[8]),
            "psi_tr": float(c[9])}


@pytest.fixture(scope="session")
def terrain_u16():
    from heligym_amd import config
    _, doc = config.make_config()
    return config.load_terrain(doc)


@pytest.fixture(scope="session")
def traj002():
    return load_golden("traj_dt0.02.npz")


@pytest.fixture(scope="session")
def traj001():
    return load_golden("traj_dt0.01.npz")
