"""Rollout (hg_rollout) of the specialised vs the generic kernel from the same state: first
(step, env) where they disagree (diagnostic)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "heli-gym_amd"))


def main():
    import torch
    from heligym_amd import HeliVecEnv
    N, K, R = 4096, 300, 50
    res = []
    for spec in (True, False):
        env = HeliVecEnv(N, task="hover", dt=0.01, autoreset=True, seed=3, device="cuda:0")
        assert env.set_specialized(spec) == spec
        env.reset()
        act = torch.empty((N, 4), dtype=torch.float32, device=env.device)
        for k in range(K):
            env.random_actions(act, seed=9, step=k)
            act[: N // 2, 0] = -1.0
            env.step_async(act, with_reset_info=False)
        s0, c0 = env.get_state()
        s0 = s0.cpu().numpy().copy()
        bank = torch.empty((R, N, 4), dtype=torch.float32, device=env.device)
        for k in range(R):
            env.random_actions(bank[k], seed=10, step=k)
        ro = env.rollout(bank)
        s, c = env.get_state()
        res.append((s0, [x.cpu().numpy().copy() for x in ro], s.cpu().numpy(), c.cpu().numpy()))
        env.close()
    eq = lambda a, b: (a == b) | (np.isnan(a) & np.isnan(b))  # noqa: E731
    (a0, ra, sa, ca), (b0, rb, sb, cb) = res
    print("state before rollout equal:", bool(eq(a0, b0).all()))
    o_a, o_b = ra[0], rb[0]
    bad = ~eq(o_a, o_b).all(2)
    if bad.any():
        k = int(np.nonzero(bad.any(1))[0][0])
        idx = np.nonzero(bad[k])[0][:4]
        print(f"rollout obs first differ at step {k}, envs {idx} (of {bad[k].sum()})")
        for i in idx:
            print(" state before rollout", a0[i])
            print(" spec obs", o_a[k, i]); print(" gen  obs", o_b[k, i])
            if k:
                print(" prev obs spec", o_a[k - 1, i]); print(" prev obs gen ", o_b[k - 1, i])
    else:
        print("rollout obs equal; final state equal:", bool(eq(sa, sb).all()))


if __name__ == "__main__":
    main()
