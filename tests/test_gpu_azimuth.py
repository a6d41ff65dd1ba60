"""GPU: the rotor azimuths (state columns 2, 3) leave the stepped state (csrc/retrim.h AzRec) and
are reconstructed when the state is read.  These tests hold the reconstruction to the stepped
evolution: the parity tests compare the azimuths with the reference goldens, these check that
re-anchoring the records (set_state, a template change) anywhere in a run changes nothing, that
every reset starts from its template's azimuths and that each step adds dt * Omega and wraps
(helicopter_dynamics.py:74-75, :257-258, :288-289).  Run with -m gpu."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch():
    import torch as t
    if not t.cuda.is_available():
        pytest.skip("no HIP device")
    return t


def _env(n, **kw):
    from heligym_amd import HeliVecEnv
    return HeliVecEnv(n, task="hover", dt=0.01, device="cuda:0", seed=11, **kw)


def _wrap(x):   # float64 view of the fp32 floor-mod wrap to [-pi, pi)
    return (x + np.pi) % (2 * np.pi) - np.pi


def _same(a, b):   # bitwise (NaN-safe) tensor equality
    import torch as t
    if a.dtype == t.float32:
        a, b = a.view(t.int32), b.view(t.int32)
    return t.equal(a, b)


def _ang_close(a, b, tol=2e-5):
    d = np.abs(_wrap(np.asarray(a, np.float64) - np.asarray(b, np.float64)))
    return d <= tol


@pytest.mark.parametrize("mode", ["same_step", "next_step"])
def test_reanchored_twin_is_bitwise_identical(torch, mode):
    """Twin B re-anchors every env's azimuth record after every step (get_state -> set_state);
    twin A never does.  Outputs and full states stay bitwise equal, pending resets included."""
    N, K = 4100, 400   # ragged last wave
    A = _env(N, autoreset=True, autoreset_mode=mode)
    B = _env(N, autoreset=True, autoreset_mode=mode)
    A.reset()
    B.reset()
    act = torch.empty((N, 4), dtype=torch.float32, device=A.device)
    resets = 0
    for k in range(K):
        A.random_actions(act, seed=5, step=k)
        act[::2, 0] = -1.0   # low collective on every other env: crashes (~280 steps) and resets
        oa, ra, ta, ua, _ = A.step(act)
        ob, rb, tb, ub, _ = B.step(act)
        assert _same(oa, ob) and _same(ra, rb) and _same(ta, tb) and _same(ua, ub)
        resets += int((ta | ua).sum())
        s, c = B.get_state()
        B.set_state(s, c)
        if k % 13 == 0 or k == K - 1:
            sa, ca = A.get_state()
            sb, cb = B.get_state()
            assert _same(sa, sb) and _same(ca, cb)
    assert resets > 0
    A.close()
    B.close()


@pytest.mark.parametrize("reset_mode,mode", [("template", "same_step"), ("retrim", "same_step"),
                                             ("retrim", "next_step")])
def test_azimuths_advance_and_reset_to_template(torch, reset_mode, mode):
    """Each step adds f_dpsi = dt * Omega to both azimuths and wraps them; a reset puts the
    template's azimuths back; a changed trim condition re-anchors the running episodes (no jump)
    and later resets start from the new template.  In reset_mode "retrim" the reset state comes
    from the device trim (retrim_write writes the azimuth record), under both auto-reset modes
    (next_step: an env that ended at step k resets at step k + 1), with trim azimuths that are not
    the defaults."""
    N, K = 2048, 400
    env = _env(N, autoreset=True, reset_mode=reset_mode, autoreset_mode=mode,
               trim_cond={"psi_mr": 0.5, "psi_tr": 2.5})
    env.reset()
    om = np.array([env.cfg.af.mr_RPM, env.cfg.af.tr_RPM], np.float64) * 2 * np.pi / 60
    d = om * env.dt
    tmpl = env.template()["state"][2:4].astype(np.float32)
    act = torch.empty((N, 4), dtype=torch.float32, device=env.device)
    s, _ = env.get_state()
    prev = s[:, 2:4].cpu().numpy()
    np.testing.assert_array_equal(prev, np.tile(tmpl, (N, 1)))
    changed, resets = False, 0
    pending = np.zeros(N, bool)   # next_step: ended last step, resets this step
    for k in range(K):
        if k == K // 2:   # new template azimuths mid-run
            before = env.get_state()[0][:, 2:4].cpu().numpy()
            env.set_trim_cond({"psi_mr": 1.0, "psi_tr": -2.0})
            after = env.get_state()[0][:, 2:4].cpu().numpy()
            np.testing.assert_array_equal(before, after)
            tmpl = env.template()["state"][2:4].astype(np.float32)
            assert not np.array_equal(tmpl, np.zeros(2, np.float32))
            changed = True
        env.random_actions(act, seed=9, step=k)
        act[::2, 0] = -1.0   # crashes on every other env, after the template change
        _, _, term, trunc, _ = env.step(act)
        ended = (term | trunc).cpu().numpy()
        reset_now = ended if mode == "same_step" else pending
        cur = env.get_state()[0][:, 2:4].cpu().numpy()
        assert np.all(cur >= -np.float32(np.pi)) and np.all(cur < np.float32(np.pi))
        np.testing.assert_array_equal(cur[reset_now], np.tile(tmpl, (int(reset_now.sum()), 1)))
        live = ~reset_now
        ok = _ang_close(cur[live], prev[live] + d)
        assert ok.all(), (k, np.argwhere(~ok)[:3])
        prev = cur
        resets += int(reset_now.sum())
        pending = ended & ~reset_now if mode == "next_step" else pending
    assert changed and resets > N // 4, resets
    if reset_mode == "retrim":
        assert env.retrim_failures() == 0
    env.close()


def test_set_state_counters_only_keeps_azimuths(torch):
    """Setting only the counters re-anchors the records at the new counters: the azimuths read back
    unchanged, and stepping continues from them."""
    N = 1000
    env = _env(N, autoreset=False)
    env.reset()
    act = torch.zeros((N, 4), dtype=torch.float32, device=env.device)
    for k in range(37):
        env.step(act)
    s0, c0 = env.get_state()
    c1 = c0.clone()
    c1[:, 0] = torch.arange(N, device=env.device, dtype=torch.int32) % 7
    env.set_state(None, c1)
    s1, c2 = env.get_state()
    assert _same(s0, s1) and _same(c1, c2)
    env.step(act)
    s2, _ = env.get_state()
    d = (np.array([env.cfg.af.mr_RPM, env.cfg.af.tr_RPM]) * 2 * np.pi / 60) * env.dt
    assert _ang_close(s2[:, 2:4].cpu().numpy(), s1[:, 2:4].cpu().numpy() + d).all()
    env.close()
