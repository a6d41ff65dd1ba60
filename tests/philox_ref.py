"""Host restatement of the step kernel's turbulence noise and synthetic actions (TEST INFRASTRUCTURE).

The reference draws `eta = randn(3) / sqrt(dt)` from NumPy's global generator once per step
(heligym/envs/dynamics/wind_dynamics.py:49-52).  The kernel replaces that generator with a
counter-based one ("eta from Philox -> Box-Muller"), keyed so that every env's stream
is fixed whatever the batch or the rank count:

  * Philox4x32-10 (Salmon et al., "Parallel random numbers: as easy as 1, 2, 3", SC'11; the
    Random123 library's philox4x32 with R = 10) on the counter (gid_lo, gid_hi, episode step,
    episode index) with the 64-bit key `seed` (csrc/heligym_amd.hip philox, draw_eta);
  * Box-Muller: u = ((x >> 8) + 0.5) 2^-24 (float32, in (0, 1], see u01) from words 0 and 2, angles from the top 23 bits
    of words 1 and 3 as a fraction of a turn; eta0 = r0 cos(2 pi a1), eta1 = r0 sin(2 pi a1),
    eta2 = r1 cos(2 pi a3), r = sqrt(-2 ln u / dt).

This module restates both in NumPy: Philox exactly (uint32 arithmetic), Box-Muller in float64 (the
kernel's hardware log2 / sqrt / sin / cos are approximations, so the comparison carries a stated
tolerance).  The published Random123 known-answer vectors pin the Philox restatement.
"""
import numpy as np

M0, M1 = 0xD2511F53, 0xCD9E8D57          # Philox4x32 multipliers
W0, W1 = 0x9E3779B9, 0xBB67AE85          # Weyl key increments
MASK = 0xFFFFFFFF

# Random123 kat_vectors, "philox4x32 10": (ctr0..3, key0..1) -> out0..3
KAT_PHILOX4X32_10 = [
    ((0x00000000, 0x00000000, 0x00000000, 0x00000000, 0x00000000, 0x00000000),
     (0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8)),
    ((0xffffffff, 0xffffffff, 0xffffffff, 0xffffffff, 0xffffffff, 0xffffffff),
     (0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd)),
    ((0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344, 0xa4093822, 0x299f31d0),
     (0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1)),
]


def philox4x32_10(rows):
    """rows [M,6] {c0, c1, c2, c3, k0, k1} (any integer dtype, values < 2^32) -> [M,4] uint32."""
    r = np.asarray(rows, dtype=np.uint64).reshape(-1, 6)
    x, y, z, w, k0, k1 = (r[:, j].copy() for j in range(6))
    for _ in range(10):
        p0 = np.uint64(M0) * x       # exact: a 32 x 32-bit product fits 64 bits
        p1 = np.uint64(M1) * z
        hi0, lo0 = p0 >> np.uint64(32), p0 & np.uint64(MASK)
        hi1, lo1 = p1 >> np.uint64(32), p1 & np.uint64(MASK)
        x, y, z, w = hi1 ^ y ^ k0, lo1, hi0 ^ w ^ k1, lo0
        k0 = (k0 + np.uint64(W0)) & np.uint64(MASK)
        k1 = (k1 + np.uint64(W1)) & np.uint64(MASK)
    return np.stack([x, y, z, w], axis=1).astype(np.uint32)


def noise_words(gid, step, epi, seed):
    """The four Philox words of the step noise of global env ids `gid` at (episode step, episode
    index) = (step, epi) (the raw counters: an env waiting for its next-step reset keys on its
    negative step counter)."""
    gid = np.asarray(gid, dtype=np.int64).astype(np.uint64)
    n = len(gid)
    rows = np.empty((n, 6), dtype=np.uint64)
    rows[:, 0] = gid & np.uint64(MASK)
    rows[:, 1] = gid >> np.uint64(32)
    rows[:, 2] = np.asarray(step, dtype=np.int64).astype(np.uint64) & np.uint64(MASK)
    rows[:, 3] = np.asarray(epi, dtype=np.int64).astype(np.uint64) & np.uint64(MASK)
    rows[:, 4] = np.uint64(seed & MASK)
    rows[:, 5] = np.uint64((seed >> 32) & MASK)
    return philox4x32_10(rows)


def u01(x):
    """The kernel's ((float)(x >> 8) + 0.5f) * 2^-24 in float32 arithmetic: the 24-bit integer converts
    exactly, but from 2^23 on the + 0.5 rounds (to even), so u is in (0, 1] and only half of the
    upper values sit mid-cell (the device measured this: a float64 restatement differed by one ulp
    in half the values past 0.5)."""
    a = (np.asarray(x, dtype=np.uint32) >> np.uint32(8)).astype(np.float32)
    return ((a + np.float32(0.5)) * np.float32(1.0 / 16777216.0)).astype(np.float64)


def turn_frac(x):
    """Fraction of a turn from the top 23 bits (the kernel builds 1.f in [1, 2) and hands it to the
    hardware sin / cos, which take revolutions)."""
    return (np.asarray(x, dtype=np.uint32) >> np.uint32(9)).astype(np.float64) / 8388608.0


def eta_ref(gid, step, epi, seed, dt):
    """float64 Box-Muller of the Philox words: [n,3] eta already scaled by 1/sqrt(dt)."""
    r = noise_words(gid, step, epi, seed)
    r0 = np.sqrt(-2.0 * np.log(u01(r[:, 0])) / dt)
    r1 = np.sqrt(-2.0 * np.log(u01(r[:, 2])) / dt)
    a1, a3 = 2 * np.pi * turn_frac(r[:, 1]), 2 * np.pi * turn_frac(r[:, 3])
    return np.stack([r0 * np.cos(a1), r0 * np.sin(a1), r1 * np.cos(a3)], axis=1)


def random_actions_ref(gid, seed, step, lo=-1.0, hi=1.0):
    """hg_random_actions (csrc/heligym_amd.hip random_actions_kernel): Philox on (gid, step) with the
    key seed ^ (0xA511E9B3, 0x63D83595), each word u01 -> lo + (hi - lo) u, one fused multiply-add in
    float32.  Restated in float64 then rounded to float32: for (lo, hi) = (-1, 1) every value is
    -1 + 2u with u a multiple of 2^-25 in (0, 1], exact in both, so the restatement is bitwise (other
    bounds could differ by a double rounding)."""
    gid = np.asarray(gid, dtype=np.int64).astype(np.uint64)
    n = len(gid)
    rows = np.empty((n, 6), dtype=np.uint64)
    rows[:, 0] = gid & np.uint64(MASK)
    rows[:, 1] = gid >> np.uint64(32)
    rows[:, 2] = np.uint64(step & MASK)
    rows[:, 3] = np.uint64((step >> 32) & MASK)
    rows[:, 4] = np.uint64((seed & MASK) ^ 0xA511E9B3)
    rows[:, 5] = np.uint64(((seed >> 32) & MASK) ^ 0x63D83595)
    w = np.float64(np.float32(hi) - np.float32(lo))
    u = u01(philox4x32_10(rows))
    return (np.float64(np.float32(lo)) + np.float64(np.float32(w)) * u).astype(np.float32)
