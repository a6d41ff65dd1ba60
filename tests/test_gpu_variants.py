"""GPU: the step kernel's launch variants give bitwise the same results.  Which variant runs is a
function of N (the lone-wave NT variant, constant pairs pinned and non-temporal stores, up to two
waves per SIMD; the bulk variant past it), so the same envs are stepped once as one batch past the
NT range and once as shards inside it (env_offset keys the noise and the synthetic actions by
global env id).  Run with -m gpu."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch():
    import torch as t
    if not t.cuda.is_available():
        pytest.skip("no HIP device")
    return t


def _run(torch, n, offset, K):
    from heligym_amd import HeliVecEnv
    env = HeliVecEnv(n, task="hover", dt=0.01, seed=17, autoreset=True, env_offset=offset, device="cuda:0")
    env.reset()
    act = torch.empty((n, 4), dtype=torch.float32, device=env.device)
    outs = []
    for k in range(K):
        env.random_actions(act, seed=8, step=k)
        act[::3, 0] = -1.0   # low collective on every third env: crashes and resets
        obs, rew, term, trunc, _ = env.step(act)
        if k % 25 == 24:
            outs.append((obs.cpu().numpy().view(np.int32).copy(), rew.cpu().numpy().view(np.int32).copy(),
                         (term | trunc).cpu().numpy().copy()))
    s, c = env.get_state()
    outs.append((s.cpu().numpy().view(np.int32).copy(), c.cpu().numpy().copy(), None))
    env.close()
    return outs


def test_nt_variant_equals_bulk_variant(torch):
    """One batch of 2 H envs (bulk variant, past two waves per SIMD) against its two halves stepped
    as batches of H (NT variant, at most two waves per SIMD; ragged last wave): every observation,
    reward and done flag and the final state bitwise equal, resets included.  The NT range ends at
    2 waves x 64 lanes x 4 SIMDs x CUs envs (131 072 on MI355X's 256 CUs); H is sized from the
    device's CU count so that H is inside it and 2 H past it on any device."""
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    nt_max = 2 * 64 * 4 * cus
    H, K = (3 * nt_max) // 4 + 9, 350   # a multiple of 3 (the crash pattern below is act[::3]), ragged
    H -= H % 3
    assert H <= nt_max < 2 * H and H % 3 == 0 and H % 64
    full = _run(torch, 2 * H, 0, K)
    lo = _run(torch, H, 0, K)
    hi = _run(torch, H, H, K)
    resets = 0
    for f, a, b in zip(full, lo, hi):
        for j in range(3):
            if f[j] is None:
                continue
            np.testing.assert_array_equal(f[j][:H], a[j])
            np.testing.assert_array_equal(f[j][H:], b[j])
        if f[2] is not None:
            resets += int(f[2].sum())
    assert resets > 0


def test_small_batch_helper_kernel_equals_lone_wave(torch):
    """A batch of at most two tiles per CU runs the helper kernel (a second wave per block steps the
    tile's noise and wind, heligym_amd.hip step_help_kernel); a larger one the one-wave kernel.  The
    first H envs of a 3 H batch against a batch of H (ragged last tile): every observation, reward
    and done flag and the final state bitwise equal, resets included."""
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    H = 2 * 64 * cus - 61
    assert H % 64 and 3 * H > 2 * 64 * cus and 3 * H <= 2 * 64 * 4 * cus
    full = _run(torch, 3 * H, 0, 300)
    small = _run(torch, H, 0, 300)
    resets = 0
    for f, a in zip(full, small):
        for j in range(3):
            if f[j] is None:
                continue
            np.testing.assert_array_equal(f[j][:H], a[j])
        if f[2] is not None:
            resets += int(f[2][:H].sum())
    assert resets > 0


@pytest.mark.parametrize("variant", ["heavy", "wing"])
def test_runtime_specialised_kernel_bitwise_equals_generic(torch, variant, tmp_path, monkeypatch):
    """Another airframe (the heavier one with other rotor speeds; the winged one) stepped with its
    run-time specialised kernel (heligym_amd._rtc: its constants compiled in) and with the generic
    kernel: observations, rewards, flags and the final state bitwise equal over 300 steps with
    in-kernel noise and auto-resets, in the lone-wave and bulk launch variants, with and without
    the optional features (TimeLimit)."""
    import golden_cases as gc
    from heligym_amd import HeliVecEnv
    monkeypatch.setenv("HELIGYM_AMD_CACHE", str(tmp_path))
    doc = gc.load_variant(variant)[1]
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    for n, kw in ((4097, {}), (4097, dict(max_episode_steps=150)), (2 * 2 * 64 * 4 * cus + 65, {})):
        outs = []
        for spec in (False, True):
            env = HeliVecEnv(n, task="hover", dt=0.01, heli_name=doc, seed=3, autoreset=True, device="cuda:0", **kw)
            assert not env.specialized
            if spec:
                assert env.specialize() and env.specialized
            env.reset()
            act = torch.empty((n, 4), dtype=torch.float32, device=env.device)
            rec = []
            for k in range(300):
                env.random_actions(act, seed=4, step=k)
                act[::4, 0] = -1.0   # crashes and resets
                env.step_async(act, with_reset_info=False)
                if k % 50 == 49:
                    rec.append([b.clone() for b in (env.obs, env.reward, env.terminated_u8, env.truncated_u8)])
            st, ctr = env.get_state()
            torch.cuda.synchronize()
            outs.append(([[b.cpu().numpy() for b in r] for r in rec], st.cpu().numpy(), ctr.cpu().numpy()))
            env.close()
        done = sum(int(r[2].sum() + r[3].sum()) for r in outs[0][0])
        assert done > 0
        for ra, rb in zip(outs[0][0], outs[1][0]):
            for x, y in zip(ra, rb):
                np.testing.assert_array_equal(x.view(np.uint8), y.view(np.uint8))
        np.testing.assert_array_equal(outs[0][1].view(np.int32), outs[1][1].view(np.int32))
        np.testing.assert_array_equal(outs[0][2], outs[1][2])
