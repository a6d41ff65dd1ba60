"""Host cost of the eager HeliVecEnv.step() / step_async() calls (diagnostic): wall time per call at
a tiny N (the GPU work is negligible, so the rate is the Python + launch path) and at 65 536 envs,
plus a cProfile of the tiny-N loop."""
import cProfile
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "heli-gym_amd"))


def main():
    import torch
    from heligym_amd import HeliVecEnv
    for n in (64, 65536):
        env = HeliVecEnv(n, task="hover", dt=0.01, autoreset=True)
        env.reset()
        act = torch.empty((n, 4), device=env.device)
        env.random_actions(act, seed=1, step=0)
        for fn_name in ("step", "step_async"):
            fn = getattr(env, fn_name)
            for _ in range(200):
                fn(act)
            torch.cuda.synchronize()
            K = 3000
            t0 = time.perf_counter()
            for _ in range(K):
                fn(act)
            t1 = time.perf_counter()
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            print(f"N={n:6d} {fn_name:10s}: issue {(t1 - t0) / K * 1e6:6.2f} us/call, "
                  f"complete {(t2 - t0) / K * 1e6:6.2f} us/step")
        if n == 64:
            pr = cProfile.Profile()
            pr.enable()
            for _ in range(3000):
                env.step(act)
            pr.disable()
            torch.cuda.synchronize()
            pstats.Stats(pr).sort_stats("tottime").print_stats(14)
        env.close()


if __name__ == "__main__":
    main()
