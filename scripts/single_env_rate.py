"""BASELINE config 1 through the single-env drop-in: one HeliHover env, 10 000 steps of zero action
with resets on termination (the reference runs 1 367 steps/s on one CPU core).  Each
step is one kernel launch plus a device->host copy of obs/reward/flags (numpy results, like the
reference)."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "heli-gym_amd"))


def main():
    from heligym_amd import HeliHover
    env = HeliHover(dt=0.02)
    env.reset()
    a = np.zeros(4, np.float32)
    for _ in range(200):
        env.step(a)
    steps, resets = 10000, 0
    env.reset()
    t0 = time.perf_counter()
    for _ in range(steps):
        _, _, term, trunc, _ = env.step(a)
        if term or trunc:
            env.reset()
            resets += 1
    el = time.perf_counter() - t0
    print(f"single env (HeliHover drop-in, dt 0.02, zero action): {steps / el:.0f} steps/s, {resets} resets, "
          f"{el / steps * 1e6:.1f} us/step")
    env.close()


if __name__ == "__main__":
    main()
