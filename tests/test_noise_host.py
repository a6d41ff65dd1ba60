"""CPU: the host restatement of the kernel's turbulence noise (tests/philox_ref.py) pinned to the
published Philox4x32-10 known-answer vectors (Random123 kat_vectors), and its Box-Muller normals
checked for the reference's distribution (wind_dynamics.py:49-52: eta = randn(3) / sqrt(dt))."""
import math

import numpy as np

import philox_ref as pr


def test_philox_kat_vectors():
    for inp, out in pr.KAT_PHILOX4X32_10:
        got = pr.philox4x32_10(np.array([inp], dtype=np.uint64))[0]
        assert tuple(int(x) for x in got) == out


def test_box_muller_restatement_is_standard_normal_over_dt():
    n, dt = 200_000, 0.02
    gid = np.arange(n)
    eta = pr.eta_ref(gid, np.full(n, 3), np.full(n, 1), 0x5EED, dt) * math.sqrt(dt)
    M = eta.size
    assert abs(eta.mean()) <= 4 / math.sqrt(M)
    assert abs(eta.var() - 1) <= 4 * math.sqrt(2 / M)
    # same key, another step: a different draw
    eta2 = pr.eta_ref(gid, np.full(n, 4), np.full(n, 1), 0x5EED, dt) * math.sqrt(dt)
    r = np.corrcoef(eta[:, 0], eta2[:, 0])[0, 1]
    assert abs(r) <= 4 / math.sqrt(n)


def test_random_actions_restatement_range():
    a = pr.random_actions_ref(np.arange(4096), 8, 0).reshape(-1, 4)
    assert a.dtype == np.float32 and a.min() > -1 and a.max() < 1
    assert abs(float(a.mean())) < 0.02
