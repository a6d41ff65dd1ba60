"""A/B of a re-trim library variant (HELIGYM_AMD_LIB): the device trims of 1 024 turbulent winds
(hg_trim_batch, saved to gpurun_out/gj_<tag>.npz for a bitwise comparison between variants), the
batch latency, and the re-trim step at 65 536 aged envs in three modes (graph replayed).  usage:
python scripts/r04_gj_ab.py TAG"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "heli-gym_amd")]
import torch  # noqa: E402
from heligym_amd import HeliVecEnv  # noqa: E402

tag = sys.argv[1]
env = HeliVecEnv(64, task="hover", dt=0.01)
rng = np.random.RandomState(0)
w = (np.array([14.14, 14.14, 0.0]) + rng.normal(0, 6, size=(1024, 3))).astype(np.float32)
out = env.trim_batch(w)
torch.cuda.synchronize()
np.savez(os.path.join(ROOT, "gpurun_out", f"gj_{tag}.npz"), **{k: v.cpu().numpy() for k, v in out.items()})
for K in (64, 1024):
    wk = w[:K]
    env.trim_batch(wk)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        env.trim_batch(wk)
    e1.record()
    torch.cuda.synchronize()
    print(f"[{tag}] trim_batch K={K}: {e0.elapsed_time(e1) / 10 * 1e3:.1f} us", flush=True)
env.close()
N, B = 65536, 100
for mode, ov in (("same_step", False), ("next_step", True)):
    env = HeliVecEnv(N, task="hover", dt=0.01, seed=1234, autoreset=True, device="cuda:0", reset_mode="retrim",
                     autoreset_mode=mode)
    if mode == "next_step":
        env.set_retrim_overlap(ov)
    env.reset()
    bank = torch.empty((B, N, 4), dtype=torch.float32, device=env.device)
    for k in range(B):
        env.random_actions(bank[k], seed=0x5EED, step=k)
    for k in range(2500):
        env.step_async(bank[k % B], with_reset_info=False)
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for k in range(B):
            env.step_async(bank[k], with_reset_info=False)
    g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for r in range(5):
        g.replay()
    torch.cuda.synchronize()
    us = (time.perf_counter() - t0) / (5 * B) * 1e6
    print(f"[{tag}] {mode:9s} overlap {int(ov)}: {us:7.2f} us/step  failures {env.retrim_failures()} "
          f"invalid {env.retrim_invalid_jobs()}", flush=True)
    env.close()
