"""Eager HeliVecEnv.step() at 65 536 aged envs against graph replay of the same steps, in one process
(the HIP runtime settings of the environment apply to both): median of 5 windows of 200 steps.
Diagnostic only."""
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "heli-gym_amd")]
import torch  # noqa: E402
from heligym_amd import HeliVecEnv  # noqa: E402

N, B, K = 65536, 100, 200
env = HeliVecEnv(N, task="hover", dt=0.01, seed=1234, autoreset=True, device="cuda:0")
env.reset()
bank = torch.empty((B, N, 4), dtype=torch.float32, device=env.device)
for k in range(B):
    env.random_actions(bank[k], seed=0x5EED, step=k)
for k in range(6000):
    env.step_async(bank[k % B], with_reset_info=False)
torch.cuda.synchronize()


def window(fn):
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / K


def eager():
    for k in range(K):
        env.step(bank[k % B])


g = torch.cuda.CUDAGraph()
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.graph(g, stream=s):
    for k in range(K):
        env.step_async(bank[k % B], with_reset_info=False)
eager()
g.replay()
ea = statistics.median(window(eager) for _ in range(5))
gr = statistics.median(window(g.replay) for _ in range(5))
t0 = time.perf_counter()
for k in range(K):
    env.step(bank[k % B])
host = (time.perf_counter() - t0) / K * 1e6
torch.cuda.synchronize()
print(f"{os.environ.get('TAG', 'default'):24s} eager {ea:6.3f} us/step  graph {gr:6.3f} us/step  ratio {ea / gr:.4f}  host {host:5.2f} us/call", flush=True)
