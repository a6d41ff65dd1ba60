"""Re-trim step cost by auto-reset mode (same step, next step with and without the overlapped trims),
graph replayed and eager, at one env count, on an aged population (3 000 steps).  The eager and graph windows are consecutive, so they see different reset rates.  Diagnostic
only."""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "heli-gym_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--steps", type=int, default=200)
    args = ap.parse_args()
    import torch
    from heligym_amd import HeliVecEnv
    N, K = args.envs, args.steps
    for mode, ov in (("same_step", False), ("next_step", False), ("next_step", True)):
        env = HeliVecEnv(N, task="hover", dt=0.01, seed=1234, autoreset=True, device="cuda:0", reset_mode="retrim",
                         autoreset_mode=mode)
        if mode == "next_step":
            env.set_retrim_overlap(ov)
        env.reset()
        bank = torch.empty((100, N, 4), dtype=torch.float32, device=env.device)
        for k in range(100):
            env.random_actions(bank[k], seed=0x5EED, step=k)
        for k in range(3000):   # into the steady state of resets
            env.step_async(bank[k % 100], with_reset_info=False)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(K):
            env.step_async(bank[k % 100], with_reset_info=False)
        torch.cuda.synchronize()
        eager = (time.perf_counter() - t0) / K * 1e6
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for k in range(100):
                env.step_async(bank[k], with_reset_info=False)
        g.replay()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for r in range(K // 100):
            g.replay()
        torch.cuda.synchronize()
        graph = (time.perf_counter() - t0) / (K // 100 * 100) * 1e6
        n_ep = int(env.get_state()[1][:, 2].long().sum())
        print(f"{mode:9s} overlap {int(ov)}  episodes {n_ep:7d}  eager {eager:7.2f} us/step  graph {graph:7.2f} us/step  failures {env.retrim_failures()}")
        env.close()


if __name__ == "__main__":
    main()
