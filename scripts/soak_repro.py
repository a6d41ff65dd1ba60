"""Replays the GPU soak test's loop (1 M hover envs, eager step() with the reset info read every 41st
step) and reports any non-finite observation: step, env ids, columns, values (diagnostic)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "heli-gym_amd"))


def main():
    import torch
    from heligym_amd import HeliVecEnv
    N, K = 1 << 20, int(sys.argv[1]) if len(sys.argv) > 1 else 200
    read_info = "--no-info" not in sys.argv
    env = HeliVecEnv(N, task="hover", dt=0.01, autoreset=True, seed=3, device="cuda:0")
    env.reset()
    act = torch.empty((N, 4), dtype=torch.float32, device=env.device)
    np.set_printoptions(linewidth=200, precision=6)
    for k in range(K):
        env.random_actions(act, seed=6, step=k)
        obs, rew, term, trunc, info = env.step(act)
        if read_info and k % 41 == 40:
            _ = info["reset_index"], info["final_obs"]
        if k % 41 == 40 or k == K - 1:
            bad = ~torch.isfinite(obs)
            if bool(bad.any()):
                rows = torch.nonzero(bad.any(dim=1)).flatten()
                print(f"step {k}: {len(rows)} rows non-finite; ids {rows[:10].tolist()}")
                done = (term | trunc)
                for r in rows[:5].tolist():
                    print("  env", r, "cols", torch.nonzero(bad[r]).flatten().tolist(), "done", bool(done[r]),
                          "\n   obs", obs[r].cpu().numpy(), "\n   rew", float(rew[r]))
                st, ctr = env.get_state()
                for r in rows[:5].tolist():
                    print("  env", r, "counters", ctr[r].tolist(), "\n   state", st[r].cpu().numpy())
                return
    print(f"all finite over {K} steps (info reads: {read_info})")


if __name__ == "__main__":
    main()
