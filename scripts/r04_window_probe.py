"""Where a short timed window loses time: 65 536 aged HeliHover envs, windows of K steps timed with
HIP events in several ways (graph per window with / without the bench's episode count around it,
eager launches, one graph holding several windows).  Prints one line per variant; run under
rocprofv3 --kernel-trace to see the gaps between kernels."""
import argparse
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "heli-gym_amd")]
import torch  # noqa: E402
from heligym_amd import HeliVecEnv  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--envs", type=int, default=65536)
ap.add_argument("--K", type=int, default=20)
ap.add_argument("--reps", type=int, default=7)
args = ap.parse_args()
dev = torch.device("cuda:0")
N, K, B = args.envs, args.K, 100
env = HeliVecEnv(N, task="hover", dt=0.01, seed=1234, autoreset=True, device=dev)
env.reset()
bank = torch.empty((B, N, 4), dtype=torch.float32, device=dev)
for k in range(B):
    env.random_actions(bank[k], seed=0x5EED, step=k)
for k in range(3000):
    env.step_async(bank[k % B], with_reset_info=False)
torch.cuda.synchronize()
s = torch.cuda.Stream(device=dev)


def capture(steps):
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for k in range(steps):
            env.step_async(bank[k % B], with_reset_info=False)
    return g


with torch.cuda.stream(s):
    for k in range(K):
        env.step_async(bank[k % B], with_reset_info=False)
torch.cuda.synchronize()
gK = capture(K)
g100 = capture(100)


def episodes():
    _, c = env.get_state()
    return c[:, 2].long().sum()


def window(body, preroll, count):
    torch.cuda.synchronize()
    cur = torch.cuda.current_stream(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if preroll:
        preroll()
    if count:
        episodes()
    e0.record(cur)
    body()
    e1.record(cur)
    if count:
        episodes()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / K


def eager():
    for k in range(K):
        env.step_async(bank[k % B], with_reset_info=False)


def rep(name, fn):
    v = [fn() for _ in range(args.reps)]
    print(f"{name:55s} median {statistics.median(v):7.3f} us/step  all {[round(x, 2) for x in v]}", flush=True)


rep("graph(K), preroll graph(K), episode count", lambda: window(gK.replay, gK.replay, True))
rep("graph(K), preroll graph(K), no count", lambda: window(gK.replay, gK.replay, False))
rep("graph(K), preroll graph(100), no count", lambda: window(gK.replay, g100.replay, False))
rep("graph(K), preroll graph(100), episode count", lambda: window(gK.replay, g100.replay, True))
rep("graph(K), no preroll", lambda: window(gK.replay, None, False))
rep("eager(K), preroll graph(100)", lambda: window(eager, g100.replay, False))
rep("graph(K) x2 back to back, per K", lambda: window(lambda: (gK.replay(), gK.replay()), g100.replay, False) / 2)
rep("graph(100), preroll graph(100) [per 100/K]", lambda: window(g100.replay, g100.replay, False) * K / 100)
t0 = time.perf_counter()
for _ in range(50):
    gK.replay()
t1 = time.perf_counter()
torch.cuda.synchronize()
print(f"host time per graph(K) replay: {(t1 - t0) / 50 * 1e6:.1f} us")
