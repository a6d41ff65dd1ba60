"""GPU: the turbulence noise of the kernels the benchmark times.

Every oracle and golden parity test injects the reference's eta (ETA instantiations of the step
kernel).  The benchmark's kernels draw it in-kernel instead (wind_dynamics.py:49-52 restated as
Philox4x32-10 + Box-Muller, tests/philox_ref.py).  These tests join the two:
  * the device Philox against the Random123 known-answer vectors and the host restatement (exact),
  * the exported in-kernel eta (hg_debug_eta) against the host Box-Muller restatement,
  * its moments, shape and independence across steps, episodes, envs and components,
  * each timed launch variant -- the small-batch helper kernel (4 096 envs), the lone-wave kernel
    (65 536) and the bulk kernel (262 144) -- stepped with in-kernel noise, bitwise equal to the same
    population stepped by the injected-noise kernel fed the exported eta, every step, through
    crashes, resets and episode-index changes.
Run with -m gpu."""
import math

import numpy as np
import pytest

import philox_ref as pr

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch():
    import torch as t
    if not t.cuda.is_available():
        pytest.skip("no HIP device")
    return t


def _env(torch, n, task="hover", **kw):
    from heligym_amd import HeliVecEnv
    kw.setdefault("seed", 0x5EED_7E4B_0000_0017)
    return HeliVecEnv(n, task=task, dt=0.01, autoreset=True, device="cuda:0", **kw)


def test_device_philox_matches_kat_and_host(torch):
    """hg_debug_philox (the step kernel's philox()) on the Random123 KAT inputs and on 65 536 random
    counters / keys: bitwise the published outputs and the host restatement."""
    from heligym_amd import _abi
    lib = _abi.load_library()
    rng = np.random.RandomState(11)
    kat_in = np.array([k for k, _ in pr.KAT_PHILOX4X32_10], dtype=np.uint32)
    rows = np.concatenate([kat_in, rng.randint(0, 2**32, size=(65536, 6), dtype=np.uint64).astype(np.uint32)])
    d_in = torch.as_tensor(rows.view(np.int32), device="cuda:0")
    d_out = torch.empty((len(rows), 4), dtype=torch.int32, device="cuda:0")
    _abi.check(lib.hg_debug_philox(d_in.data_ptr(), d_out.data_ptr(), len(rows), None), lib)
    torch.cuda.synchronize()
    got = d_out.cpu().numpy().view(np.uint32)
    for j, (_, o) in enumerate(pr.KAT_PHILOX4X32_10):
        assert tuple(int(x) for x in got[j]) == o
    np.testing.assert_array_equal(got, pr.philox4x32_10(rows))


def test_random_actions_match_host(torch):
    """hg_random_actions (the bench's policy stand-in) bitwise the host restatement, with a global env
    id past 2^32 (the counter's high word) and a 64-bit step."""
    off = (1 << 32) + 12345
    env = _env(torch, 1000, env_offset=off)
    act = torch.empty((1000, 4), dtype=torch.float32, device=env.device)
    for seed, step in ((8, 0), (0xDEADBEEF12345678, (1 << 33) + 7)):
        env.random_actions(act, seed=seed, step=step)
        got = act.cpu().numpy()
        ref = pr.random_actions_ref(off + np.arange(1000), seed, step).reshape(1000, 4)
        np.testing.assert_array_equal(got.view(np.int32), ref.view(np.int32))
    env.close()


# In-kernel eta against the float64 restatement.  The kernel forms sqrt(log2(u) (-2 ln 2 / dt)) and
# cos / sin of the turn fraction with the hardware v_log / v_sqrt / v_cos / v_sin (fp32); the
# restatement is float64.  Tolerance: 1e-4 absolute (1e-5 of the noise's standard deviation 10 at
# dt 0.01) plus 4e-6 relative.
ETA_ABS, ETA_REL = 1e-4, 4e-6


def test_in_kernel_eta_matches_host_restatement(torch):
    """hg_debug_eta over 65 536 envs with counters set to random (step, episode) -- negative steps (an
    env waiting for its next-step reset) and episode indices past 2^16 included -- and global env ids
    past 2^32: within ETA_ABS + ETA_REL |eta| of the host Box-Muller of the host Philox words."""
    n, off = 65536, (1 << 33) + 5
    env = _env(torch, n, env_offset=off)
    rng = np.random.RandomState(3)
    ctr = np.zeros((n, 3), np.int32)
    ctr[:, 0] = rng.randint(-5000, 5000, size=n)
    ctr[:, 2] = rng.randint(0, 1 << 20, size=n)
    env.set_state(counters=ctr)
    got = env.debug_eta().cpu().numpy().astype(np.float64)
    ref = pr.eta_ref(off + np.arange(n), ctr[:, 0], ctr[:, 2], env.cfg.seed, 0.01)
    err = np.abs(got - ref)
    tol = ETA_ABS + ETA_REL * np.abs(ref)
    print(f"\n[eta] max|d| {err.max():.3e}, max |d|/tol {(err / tol).max():.3f}")
    assert np.all(err <= tol), np.argwhere(err > tol)[:10]
    env.close()


def test_debug_eta_rejects_a_wrong_buffer(torch):
    """debug_eta writes 3 * N floats: a buffer of another shape, dtype, device or layout is refused
    before the kernel runs (ValueError), never written out of bounds."""
    env = _env(torch, 100)
    bad = [torch.zeros((99, 3), device="cuda:0"), torch.zeros((100, 3), dtype=torch.float64, device="cuda:0"),
           torch.zeros((100, 3)), torch.zeros((3, 100), device="cuda:0").t()]
    for out in bad:
        with pytest.raises(ValueError):
            env.debug_eta(out)
    assert env.debug_eta().shape == (100, 3)
    env.close()


def _ks_normal(x):
    """Kolmogorov-Smirnov distance of the sample x (a torch tensor) from N(0, 1)."""
    import torch
    s, _ = torch.sort(x.double())
    m = s.numel()
    cdf = 0.5 * (1 + torch.erf(s / math.sqrt(2)))
    i = torch.arange(1, m + 1, dtype=torch.float64, device=x.device)
    return float(torch.maximum(i / m - cdf, cdf - (i - 1) / m).max())


def test_in_kernel_eta_moments_and_independence(torch):
    """65 536 envs x 100 steps of in-kernel noise as the stepping kernel keys it (random actions, a
    crash pattern, auto-resets): eta sqrt(dt) has mean 0 and variance 1 within 4 sigma of their
    sampling error, kurtosis 3 within 4 sigma, Kolmogorov-Smirnov distance from N(0,1) below the
    1 % critical value, and no correlation (|r| within 4 / sqrt(M)) between components, between
    consecutive steps of an env, between neighbouring envs, and between the same step of two
    consecutive episodes."""
    n, T, dt = 65536, 100, 0.01
    env = _env(torch, n)
    env.reset()
    act = torch.empty((n, 4), dtype=torch.float32, device=env.device)
    etas = torch.empty((T, n, 3), dtype=torch.float32, device=env.device)
    for k in range(T):
        env.debug_eta(etas[k])
        env.random_actions(act, seed=5, step=k)
        act[::3, 0] = -1.0
        env.step(act)
    _, ctr = env.get_state()
    assert int(ctr[:, 2].max()) > 0, "no episode ended in the window"
    z = etas.double() * math.sqrt(dt)
    M = z.numel()
    mean, var = float(z.mean()), float(z.var())
    kurt = float(((z - mean) ** 4).mean()) / var ** 2
    print(f"\n[eta moments] M={M} mean {mean:.2e} var {var:.5f} kurtosis {kurt:.4f}")
    assert abs(mean) <= 4 / math.sqrt(M)
    assert abs(var - 1) <= 4 * math.sqrt(2 / M)
    assert abs(kurt - 3) <= 4 * math.sqrt(24 / M)
    for c in range(3):
        d = _ks_normal(z[:, :, c].flatten())
        print(f"[eta KS] component {c}: D = {d:.2e} (1 % critical {1.63 / math.sqrt(M / 3):.2e})")
        assert d <= 1.63 / math.sqrt(M / 3)

    def corr(a, b):
        a, b = a.flatten() - a.mean(), b.flatten() - b.mean()
        return float((a * b).sum() / torch.sqrt((a * a).sum() * (b * b).sum())), a.numel()

    pairs = {"components 0-1": (z[..., 0], z[..., 1]), "components 0-2": (z[..., 0], z[..., 2]),
             "components 1-2": (z[..., 1], z[..., 2]),
             "lag-1 steps": (z[1:], z[:-1]), "neighbour envs": (z[:, 1:], z[:, :-1])}
    # the same (step, env) in consecutive episodes: counters set explicitly
    ctr = np.zeros((n, 3), np.int32)
    ctr[:, 0] = np.arange(n) % 4000
    ctr[:, 2] = 7
    env.set_state(counters=ctr)
    e7 = env.debug_eta().double()
    ctr[:, 2] = 8
    env.set_state(counters=ctr)
    e8 = env.debug_eta().double()
    pairs["episode e vs e+1"] = (e7, e8)
    for name, (a, b) in pairs.items():
        r, m = corr(a, b)
        print(f"[eta corr] {name}: r = {r:+.2e} (4/sqrt(M) = {4 / math.sqrt(m):.2e})")
        assert abs(r) <= 4 / math.sqrt(m), name
    env.close()


def _launch_kind(n, cus):
    if n <= 64 * 4 * cus // 2:
        return "helper"
    return "lone-wave" if n <= 2 * 64 * 4 * cus else "bulk"


@pytest.mark.parametrize("n,task", [(4096, "hover"), (65536, "hover"), (262144, "hover"),
                                    (262144, "forward_flight")])
def test_in_kernel_noise_step_bitwise_equals_injected(torch, n, task):
    """The population stepped by the kernel the benchmark times at this size (in-kernel noise:
    helper kernel at 4 096 envs, lone-wave at 65 536, bulk at 262 144; BASELINE config 4 is the
    262 144-env HeliForwardFlight population, helicopter_with_tasks.py:78-115) and a twin stepped by
    the injected-noise kernel (the instantiation every oracle / golden parity test runs) fed the
    exported eta of the same step: observations, rewards, flags and info bits bitwise equal at every
    one of 400 steps (crashes, auto-resets, new episode keys), and the final state."""
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    kind = _launch_kind(n, cus)
    print(f"\n[{n} {task} envs] in-kernel launch: {kind}")
    a, b = _env(torch, n, task), _env(torch, n, task)
    a.reset()
    b.reset()
    act = torch.empty((n, 4), dtype=torch.float32, device=a.device)
    eta = torch.empty((n, 3), dtype=torch.float32, device=a.device)
    ends = 0
    for k in range(400):
        a.random_actions(act, seed=21, step=k)
        act[::3, 0] = -1.0
        a.debug_eta(eta)
        oa, ra, ta, ua, ia = a.step(act)
        ia_bits = a.info_u8.clone()
        ob, rb, tb, ub, ib = b.step(act, eta=eta)
        assert torch.equal(oa.view(torch.int32), ob.view(torch.int32)), k
        assert torch.equal(ra.view(torch.int32), rb.view(torch.int32)), k
        assert torch.equal(ta, tb) and torch.equal(ua, ub), k
        assert torch.equal(ia_bits, b.info_u8), k
        ends += int((ta | ua).sum())
    sa, ca = a.get_state()
    sb, cb = b.get_state()
    assert torch.equal(sa.view(torch.int32), sb.view(torch.int32))
    assert torch.equal(ca, cb)
    assert ends > 0 and int(ca[:, 2].max()) > 0
    print(f"[{n} envs] 400 steps bitwise, {ends} episode ends")
    a.close()
    b.close()
