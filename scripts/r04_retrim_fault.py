"""Diagnostic: the bench's re-trim secondary (65 536 aged HeliHover envs, reset_mode="retrim", one
auto-reset mode per process), step by step with a synchronize after every graph replay, printing the
re-trim failures and the invalid job records the trim skipped (hg_debug_retrim_invalid).  Mirrors
bench.py's sequence: age 3 000 steps, warm-up, B eager steps on a side stream, one captured graph of B
steps, then timed windows of a preroll replay, get_state, K/B replays and get_state."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "heli-gym_amd")]
import torch  # noqa: E402
from heligym_amd import HeliVecEnv  # noqa: E402

mode = sys.argv[1] if len(sys.argv) > 1 else "same_step"
N, B, K = int(os.environ.get("N", "65536")), 100, 500
dev = torch.device("cuda:0")
env = HeliVecEnv(N, task="hover", dt=0.01, seed=1234, autoreset=True, device=dev, reset_mode="retrim",
                 autoreset_mode=mode)
env.reset()
bank = torch.empty((B, N, 4), dtype=torch.float32, device=dev)
for k in range(B):
    env.random_actions(bank[k], seed=0x5EED, step=k)


RINGS = os.environ.get("RINGS", "0") == "1"
DBG = hasattr(env.lib, "hg_debug_rt_log_ov") if os.environ.get("HELIGYM_AMD_LIB") else False
if DBG:
    import ctypes
    import numpy as np
    for nm in ("hg_debug_rt_log_ov", "hg_debug_rt_log_serial"):
        getattr(env.lib, nm).restype = ctypes.c_int
        getattr(env.lib, nm).argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32]
    ptrs = (ctypes.c_int64 * 3)()
    env.lib.hg_debug_ptrs.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    env.lib.hg_debug_ptrs(env._h, ptrs)
    names = {ptrs[0] + 4 * k: f"ring{k}" for k in range(3)}
    names.update({ptrs[2] + 4 * k: f"ov{k}" for k in range(3)})
    names[ptrs[1]] = "reset_count"
    print("pointers", [hex(p) for p in ptrs], flush=True)


def dbg_log(tag):
    for nm in ("hg_debug_rt_log_serial", "hg_debug_rt_log_ov"):
        buf = np.zeros((4096, 4), dtype=np.int64)
        n = getattr(env.lib, nm)(buf.ctypes.data, buf.nbytes, 1)
        n = min(n, 4096)
        rows = buf[:n]
        big = rows[rows[:, 1] > 1000]
        if len(big):
            print(f"  {tag} {nm}: {n} launches, {len(big)} with > 1000 jobs:",
                  [(names.get(int(r[0]), hex(int(r[0]))), int(r[1]), int(r[2]), int(r[3])) for r in big[:6]], flush=True)


def report(tag):
    import ctypes
    torch.cuda.synchronize()
    rings = ""
    if RINGS:
        q = (ctypes.c_int32 * 9)()
        env.lib.hg_debug_queues(env._h, q)
        rings = f" rings {list(q)}"
    print(f"[{mode}] {tag}: failures {env.retrim_failures()} invalid {env.retrim_invalid_jobs()}{rings}", flush=True)
    if DBG:
        dbg_log(tag)


t0 = time.time()
for k in range(3000):
    env.step_async(bank[k % B], with_reset_info=False)
    if k % 500 == 499:
        report(f"aged {k + 1}")
for k in range(5):
    env.step_async(bank[k % B], with_reset_info=False)
report("warmup")
s = torch.cuda.Stream(device=dev)
s.wait_stream(torch.cuda.current_stream(dev))
with torch.cuda.stream(s):
    for k in range(B):
        env.step_async(bank[k % B], with_reset_info=False)
torch.cuda.current_stream(dev).wait_stream(s)
report("side-stream steps")
full = torch.cuda.CUDAGraph()
with torch.cuda.graph(full):
    for k in range(B):
        env.step_async(bank[k % B], with_reset_info=False)
report("captured")
for r in range(K // B):
    full.replay()
    report(f"replay {r}")
for w in range(3):
    full.replay()
    report(f"window {w} preroll")
    _, c = env.get_state()
    report(f"window {w} get_state")
    for r in range(K // B):
        full.replay()
        report(f"window {w} replay {r}")
    _, c = env.get_state()
    report(f"window {w} end, episodes {int(c[:, 2].long().sum())}")
# a graph of G steps (G = 1, 2, 3, 4) replayed back to back, a report after each replay
for G in (1, 2, 3, 4):
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for k in range(G):
            env.step_async(bank[k % B], with_reset_info=False)
    for r in range(4):
        g.replay()
        report(f"G={G} replay {r}")
    del g
print(f"[{mode}] done in {time.time() - t0:.1f} s", flush=True)
env.close()
