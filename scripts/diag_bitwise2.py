"""Final observations after the bitwise test's exact step sequence (no per-step copies), for the
specialised and the generic kernel of the library in HELIGYM_AMD_LIB; saved to gpurun_out/<tag>.npz."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "heli-gym_amd"))


def run(spec, N=4096, K=300):
    import torch
    from heligym_amd import HeliVecEnv
    env = HeliVecEnv(N, task="hover", dt=0.01, autoreset=True, seed=3, device="cuda:0")
    assert env.set_specialized(spec) == spec
    env.reset()
    act = torch.empty((N, 4), dtype=torch.float32, device=env.device)
    rew_sum = torch.zeros((N,), dtype=torch.float32, device=env.device)
    flags = torch.zeros((N,), dtype=torch.int32, device=env.device)
    for k in range(K):
        env.random_actions(act, seed=9, step=k)
        act[: N // 2, 0] = -1.0
        env.step_async(act, with_reset_info=False)
        rew_sum += torch.nan_to_num(env.reward, nan=0.0)
        flags += env.terminated_u8.int() + 2 * env.truncated_u8.int()
    s, c = env.get_state()
    out = dict(obs=env.obs.cpu().numpy(), rew=rew_sum.cpu().numpy(), flags=flags.cpu().numpy(),
               state=s.cpu().numpy(), ctr=c.cpu().numpy())
    env.close()
    return out


def main():
    tag = sys.argv[1]
    res = {}
    for spec in (True, False):
        for rep in range(2):
            o = run(spec)
            for k, v in o.items():
                res[f"{'spec' if spec else 'gen'}{rep}/{k}"] = v
    np.savez(os.path.join(ROOT, "gpurun_out", f"{tag}.npz"), **res)
    eq = lambda a, b: bool(((a == b) | (np.isnan(a) & np.isnan(b))).all())  # noqa: E731
    for a, b in (("spec0", "spec1"), ("gen0", "gen1"), ("spec0", "gen0")):
        print(tag, a, b, {k: eq(res[f"{a}/{k}"], res[f"{b}/{k}"]) for k in ("obs", "state", "ctr", "flags")})


if __name__ == "__main__":
    main()
