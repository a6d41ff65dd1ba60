"""Experiment: N envs stepped as G independent env groups, each with its own HIP stream and
hipGraph of B steps (EnvPool-style async groups), against the single-launch step.  Reports
env-steps/s per G.  Diagnostic only."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "heli-gym_amd"))


def run(N, G, steps, B=100):
    import torch
    from heligym_amd import HeliVecEnv
    dev = torch.device("cuda:0")
    n = N // G
    envs, banks, graphs, streams = [], [], [], []
    for g in range(G):
        s = torch.cuda.Stream(device=dev)
        with torch.cuda.stream(s):
            e = HeliVecEnv(n, task="hover", dt=0.01, seed=1234, autoreset=True, env_offset=g * n, device=dev)
            e.reset()
            bank = torch.empty((B, n, 4), dtype=torch.float32, device=dev)
            for k in range(B):
                e.random_actions(bank[k], seed=0x5EED, step=k)
            for k in range(B):
                e.step_async(bank[k], with_reset_info=False)
        torch.cuda.synchronize()
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr, stream=s):
            for k in range(B):
                e.step_async(bank[k], with_reset_info=False)
        envs.append(e); banks.append(bank); graphs.append(gr); streams.append(s)
    torch.cuda.synchronize()
    for g in range(G):
        with torch.cuda.stream(streams[g]):
            graphs[g].replay()
    torch.cuda.synchronize()
    reps = max(1, steps // B)
    main = torch.cuda.current_stream(dev)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record(main)
    for s in streams:
        s.wait_stream(main)
    for r in range(reps):
        for g in range(G):
            with torch.cuda.stream(streams[g]):
                graphs[g].replay()
    for s in streams:
        main.wait_stream(s)
    ev1.record(main)
    torch.cuda.synchronize()
    ms = ev0.elapsed_time(ev1)
    K = reps * B
    rate = N * K / (ms * 1e-3)
    print(f"N={N:8d} G={G} {ms / K * 1e3:7.2f} us/step {rate:.3e} env-steps/s", flush=True)
    for e in envs:
        e.close()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, nargs="+", default=[65536, 262144])
    ap.add_argument("--groups", type=int, nargs="+", default=[1, 2, 4])
    ap.add_argument("--steps", type=int, default=2000)
    a = ap.parse_args()
    for N in a.envs:
        for G in a.groups:
            run(N, G, a.steps)


if __name__ == "__main__":
    main()
