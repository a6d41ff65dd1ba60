"""Host cost per call of the eager step path, split: a no-op ctypes call, the raw hg_step_rows call
with fixed arguments (ctypes + HIP launch), and HeliVecEnv.step() (+ Python).  Tiny N, so the GPU
work does not throttle the loop.  Diagnostic only."""
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "heli-gym_amd"))


def per_call(fn, k=5000):
    import torch
    for _ in range(200):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(k):
        fn()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    return (t1 - t0) / k * 1e6


def main():
    import torch
    from heligym_amd import HeliVecEnv
    env = HeliVecEnv(64, task="hover", dt=0.01)
    env.reset()
    act = torch.zeros((64, 4), device=env.device)
    bank = torch.zeros((100, 64, 4), device=env.device)
    lib = env.lib
    b = env._sets[0]
    p = b["p"]
    s = env._stream()
    args = (env._h, act.data_ptr(), env._p_obs, env._p_rew, env._p_term, env._p_trunc, p[0], None, p[2], s)
    print(f"ctypes no-op (hg_abi_version)   {per_call(lambda: lib.hg_abi_version()):6.2f} us")
    print(f"raw hg_step_rows, fixed args    {per_call(lambda: lib.hg_step_rows(*args)):6.2f} us")
    print(f"env.step(act)                   {per_call(lambda: env.step(act)):6.2f} us")
    k = [0]

    def bank_step():
        env.step(bank[k[0] % 100])
        k[0] += 1
    print(f"env.step(bank[k % 100])         {per_call(bank_step):6.2f} us")
    print(f"bank[k % 100] alone             {per_call(lambda: bank[7]):6.2f} us")
    env.close()


if __name__ == "__main__":
    main()
