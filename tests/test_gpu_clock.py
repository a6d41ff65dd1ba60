"""GPU: hg_clock_stamp, the clock bench.py's windows are timed with (two stamps inside the window's
hipGraph around exactly K step launches).  Run with -m gpu."""
import ctypes

import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch():
    import torch as t
    if not t.cuda.is_available():
        pytest.skip("no HIP device")
    return t


def test_clock_stamps_bracket_steps_like_events(torch):
    """Stamps around 200 eager steps of 65 536 envs measure what HIP events around the same launches
    measure (the 100 MHz clock against the event timer: within 5 % and a few microseconds), and a
    stamp after more work reads a later time."""
    from heligym_amd import HeliVecEnv
    env = HeliVecEnv(65536, task="hover", dt=0.01, seed=5, autoreset=True, device="cuda:0")
    env.reset()
    act = torch.empty((65536, 4), dtype=torch.float32, device=env.device)
    env.random_actions(act, seed=1, step=0)
    st = torch.zeros((2,), dtype=torch.int64, device=env.device)
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    for k in range(50):
        env.step_async(act, with_reset_info=False)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    assert env.lib.hg_clock_stamp(ctypes.c_void_p(st[0:1].data_ptr()), stream) == 0
    for k in range(200):
        env.step_async(act, with_reset_info=False)
    assert env.lib.hg_clock_stamp(ctypes.c_void_p(st[1:2].data_ptr()), stream) == 0
    e1.record()
    torch.cuda.synchronize()
    t0, t1 = st.tolist()
    stamp_s = (t1 - t0) / 100e6
    event_s = e0.elapsed_time(e1) * 1e-3
    assert t1 > t0 > 0
    assert 200 * 3e-6 < stamp_s <= event_s * 1.05 + 5e-6, (stamp_s, event_s)
    assert stamp_s >= event_s * 0.95 - 20e-6, (stamp_s, event_s)
    # a misaligned destination is refused
    assert env.lib.hg_clock_stamp(ctypes.c_void_p(st.data_ptr() + 4), stream) != 0
    env.close()
