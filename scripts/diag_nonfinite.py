"""First step at which an env's observation or reward is not finite (diagnostic).  Runs N hover envs
with U(-1,1) Philox actions and injected normal turbulence noise (torch generator, so the step can be
replayed through the oracle), keeps the state before each step, and on the first non-finite output
saves the offending envs' inputs and outputs to gpurun_out/nonfinite.npz.
With --philox the in-kernel noise is used instead (not replayable through the oracle, but the env
id, counters and state reproduce the step bitwise on the device).
usage: python scripts/diag_nonfinite.py [N] [K] [--philox]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "heli-gym_amd"))


def main():
    import torch
    from heligym_amd import HeliVecEnv
    argv = [a for a in sys.argv[1:] if not a.startswith("--")]
    philox = "--philox" in sys.argv
    N = int(argv[0]) if len(argv) > 0 else 1 << 20
    K = int(argv[1]) if len(argv) > 1 else 400
    dt = 0.01
    env = HeliVecEnv(N, task="hover", dt=dt, autoreset=True, seed=3)
    env.reset()
    act = torch.empty((N, 4), dtype=torch.float32, device=env.device)
    gen = torch.Generator(device=env.device)
    gen.manual_seed(11)
    for k in range(K):
        env.random_actions(act, seed=6, step=k)
        eta = None if philox else torch.randn((N, 3), generator=gen, device=env.device) / np.sqrt(dt)
        st, ctr = env.get_state()
        obs, rew, term, trunc, info = env.step(act, eta=eta)
        bad = ~(torch.isfinite(obs).all(dim=1) & torch.isfinite(rew))
        nb = int(bad.sum())
        if nb:
            ids = torch.nonzero(bad).flatten()[:64]
            out = {"step": k, "n_bad": nb, "ids": ids.cpu().numpy(), "dt": dt,
                   "state": st[ids].cpu().numpy(), "counters": ctr[ids].cpu().numpy(),
                   "actions": act[ids].cpu().numpy(), "philox": philox,
                   "eta": np.zeros((len(ids), 3), np.float32) if eta is None else eta[ids].cpu().numpy(),
                   "obs": obs[ids].cpu().numpy(), "reward": rew[ids].cpu().numpy(),
                   "term": term[ids].cpu().numpy(), "trunc": trunc[ids].cpu().numpy()}
            st2, ctr2 = env.get_state()
            out["state_after"] = st2[ids].cpu().numpy()
            os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
            np.savez(os.path.join(ROOT, "gpurun_out", "nonfinite.npz"), **out)
            print(f"step {k}: {nb} envs with non-finite output; first ids {out['ids'][:8]}")
            np.set_printoptions(linewidth=200, precision=6)
            for j in range(min(3, len(ids))):
                print("env", int(ids[j]), "counters", out["counters"][j], "term/trunc", out["term"][j], out["trunc"][j])
                print("  obs   ", out["obs"][j], "reward", out["reward"][j])
                print("  action", out["actions"][j], "eta", out["eta"][j])
                print("  state before", out["state"][j])
                print("  state after ", out["state_after"][j])
            return
    print(f"no non-finite output in {K} steps of {N} envs")


if __name__ == "__main__":
    main()
