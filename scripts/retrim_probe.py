"""Latency of the device batched trim (hg_trim_batch) for K winds, and of a step in reset_mode
"retrim" vs "template" at 65536 envs (diagnostic)."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "heli-gym_amd"))


def main():
    import torch
    from heligym_amd import HeliVecEnv
    env = HeliVecEnv(64, task="hover", dt=0.01)
    rng = np.random.RandomState(0)
    for K in (1, 16, 130, 1024):
        w = (np.array([14.14, 14.14, 0.0]) + rng.normal(0, 3, size=(K, 3))).astype(np.float32)
        env.trim_batch(w)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            env.trim_batch(w)
        e1.record()
        torch.cuda.synchronize()
        print(f"trim_batch K={K:5d}: {e0.elapsed_time(e1) / 5 * 1e3:9.1f} us per call")
    env.close()
    for mode in ("template", "retrim"):
        env = HeliVecEnv(65536, task="hover", dt=0.01, reset_mode=mode)
        env.reset()
        act = torch.empty((65536, 4), device=env.device)
        cnt = torch.zeros(1, dtype=torch.int32, device=env.device)
        for k in range(300):
            env.random_actions(act, seed=1, step=k)
            env.step_async(act, with_reset_info=False)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(300, 500):
            env.random_actions(act, seed=1, step=k)
            env.step_async(act, with_reset_info=False)
            cnt += env.truncated_u8.sum(dtype=torch.int32) + env.terminated_u8.sum(dtype=torch.int32)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / 200
        print(f"{mode:9s}: {dt * 1e6:8.1f} us per step (eager, incl. actions + flag sums), "
              f"resets/step {int(cnt.item()) / 200:.1f}, retrim failures {env.retrim_failures()}")
        env.close()


if __name__ == "__main__":
    main()
