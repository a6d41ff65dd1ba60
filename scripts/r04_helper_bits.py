"""Bitwise check of a library variant against the in-tree one: N envs (aged, with resets), K steps
of random actions, a digest of the states, counters, observations, rewards and flags after each
phase.  usage: HELIGYM_AMD_LIB=... python scripts/r04_helper_bits.py N K [task] [reset_mode]"""
import hashlib
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "heli-gym_amd"))
from heligym_amd.vector import HeliVecEnv  # noqa: E402


def main():
    n, k = int(sys.argv[1]), int(sys.argv[2])
    task = sys.argv[3] if len(sys.argv) > 3 else "hover"
    mode = sys.argv[4] if len(sys.argv) > 4 else "template"
    env = HeliVecEnv(n, task=task, seed=7, device="cuda:0", reset_mode=mode, max_episode_steps=300)
    env.reset()
    g = torch.Generator(device="cuda:0").manual_seed(3)
    h = hashlib.sha256()
    resets = 0
    for s in range(k):
        act = torch.rand((n, 4), device="cuda:0", generator=g) * 2 - 1
        obs, rew, term, trunc, info = env.step(act)
        resets += int((term | trunc).sum())
        if s % 50 == 49 or s == k - 1:
            for t in (obs, rew, term, trunc):
                h.update(t.cpu().numpy().tobytes())
    st, cn = env.get_state()
    h.update(st.cpu().numpy().tobytes())
    h.update(cn.cpu().numpy().tobytes())
    torch.cuda.synchronize()
    print(f"{os.path.basename(os.environ.get('HELIGYM_AMD_LIB', 'in-tree'))} n={n} k={k} {task} {mode} "
          f"resets={resets} digest={h.hexdigest()[:16]}", flush=True)


if __name__ == "__main__":
    main()
