"""Probe: HIP timing events recorded inside a captured hipGraph (torch.cuda.Event(external=True)),
bracketing exactly K steps after a pre-roll of P steps in the same graph, against events around
whole-graph launches.  65 536 aged HeliHover envs."""
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "heli-gym_amd")]
import torch  # noqa: E402
from heligym_amd import HeliVecEnv  # noqa: E402

N, P = 65536, 100
env = HeliVecEnv(N, task="hover", dt=0.01, seed=1234, autoreset=True, device="cuda:0")
env.reset()
bank = torch.empty((P, N, 4), dtype=torch.float32, device=env.device)
for k in range(P):
    env.random_actions(bank[k], seed=0x5EED, step=k)
for k in range(3000):
    env.step_async(bank[k % P], with_reset_info=False)
torch.cuda.synchronize()
for K in (20, 100, 1000):
    e0 = torch.cuda.Event(enable_timing=True, external=True)
    e1 = torch.cuda.Event(enable_timing=True, external=True)
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.graph(g, stream=s):
        for k in range(P):
            env.step_async(bank[k], with_reset_info=False)
        e0.record()
        for k in range(K):
            env.step_async(bank[k % P], with_reset_info=False)
        e1.record()
    g.replay()
    torch.cuda.synchronize()
    inner, outer = [], []
    for r in range(5):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        g.replay()
        b.record()
        torch.cuda.synchronize()
        inner.append(e0.elapsed_time(e1) * 1e3 / K)
        outer.append(a.elapsed_time(b) * 1e3 / (P + K))
    print(f"K={K:5d}: inner {statistics.median(inner):7.3f} us/step {[round(x, 3) for x in inner]}  "
          f"outer {statistics.median(outer):7.3f} us/step", flush=True)
    del g
env.close()
