"""Kernel timeline of the overlapped next-step re-trim (run under rocprofv3 --kernel-trace): 65 536
aged HeliHover envs, reset_mode="retrim", next-step auto-reset, one hipGraph of 50 steps replayed
twice (overlap on), then the same eager.  Prints the per-step times; trace_ov.py reads the trace."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "heli-gym_amd")]
import torch  # noqa: E402
from heligym_amd import HeliVecEnv  # noqa: E402

ov = int(os.environ.get("OV", "1"))
N, B = int(os.environ.get("N", "65536")), 50
env = HeliVecEnv(N, task="hover", dt=0.01, seed=1234, autoreset=True, device="cuda:0", reset_mode="retrim",
                 autoreset_mode="next_step")
env.set_retrim_overlap(bool(ov))
env.reset()
bank = torch.empty((B, N, 4), dtype=torch.float32, device=env.device)
for k in range(B):
    env.random_actions(bank[k], seed=0x5EED, step=k)
for k in range(3000):
    env.step_async(bank[k % B], with_reset_info=False)
torch.cuda.synchronize()
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g, stream=s):
    for k in range(B):
        env.step_async(bank[k], with_reset_info=False)
torch.cuda.synchronize()
for r in range(3):
    t0 = time.perf_counter()
    g.replay()
    torch.cuda.synchronize()
    print(f"graph replay {r}: {(time.perf_counter() - t0) / B * 1e6:.2f} us/step", flush=True)
for r in range(2):
    t0 = time.perf_counter()
    for k in range(B):
        env.step_async(bank[k], with_reset_info=False)
    torch.cuda.synchronize()
    print(f"eager {r}: {(time.perf_counter() - t0) / B * 1e6:.2f} us/step", flush=True)
env.close()
