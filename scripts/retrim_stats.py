"""Diagnostic: the device trims' Newton solves in the bench's re-trim population (65 536 HeliHover envs,
random actions, re-trim per reset): solves tried with the host trim's pivot order and those the residual
test sent to the pivot search, per trim.  usage: python scripts/retrim_stats.py [same_step|next_step]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "heli-gym_amd"))


def main():
    import torch
    from heligym_amd import HeliVecEnv
    mode = sys.argv[1] if len(sys.argv) > 1 else "next_step"
    n = 65536
    env = HeliVecEnv(n, task="hover", dt=0.01, autoreset=True, reset_mode="retrim", autoreset_mode=mode,
                     seed=1234, device="cuda:0")
    env.reset()
    act = torch.empty((n, 4), dtype=torch.float32, device="cuda:0")
    for k in range(2000):
        env.random_actions(act, seed=0x5EED, step=k)
        env.step_async(act)
        if k in (999, 1999):
            torch.cuda.synchronize()
            t, r = env.retrim_solve_stats()
            _, ctr = env.get_state()
            trims = int(ctr[:, 2].long().sum())
            print(f"after {k + 1} steps: {trims} trims, {t} Newton solves ({t / max(trims, 1):.2f} per trim), "
                  f"{r} re-solved with the pivot search ({100.0 * r / max(t, 1):.1f} %), failures {env.retrim_failures()}")
    env.close()


if __name__ == "__main__":
    main()
