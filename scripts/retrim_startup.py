"""Start-up of the device re-trim in env mode (the bench's same-step path) from an HG_TIMING=1 build
(HELIGYM_AMD_LIB=<that .so>): the aged 65 536-env re-trim population stepped a few times, then per
launch the first job's stamps -- kernel entry [62], job count + first record arrived [60], trim setup
arrived [59], first round start [0], then the rounds -- in s_memtime ticks and in us at the given
clock.  Diagnostic only."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "heli-gym_amd"))


def main():
    import torch
    sys.argv = ["bench.py", "--reset-mode", "retrim", "--autoreset-mode", "same_step", "--age-seconds", "20"]
    import bench
    args = bench.parse()
    dev = torch.device("cuda:0")
    N, B = args.envs, 64
    env = bench.make_env(args, torch, N, 0, dev)
    bank = bench.action_bank(args, torch, env, N, dev, B)
    bench.age(args, torch, env, bank, B)
    fn = env.lib.hg_debug_retrim_timing
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int64]
    ghz = 1.87   # s_memtime ticks per ns on MI355X (scripts/ubench, against the event clock)
    for k in range(5):
        buf = np.zeros(64, dtype=np.uint64)
        fn(buf.ctypes.data, buf.nbytes)   # clear nothing: read before and after, keep the new launch's
        env.step_async(bank[k % B], with_reset_info=False)
        torch.cuda.synchronize()
        t = np.zeros(64, dtype=np.uint64)
        assert fn(t.ctypes.data, t.nbytes) == 0
        t = t.astype(np.int64)
        e = t[62]
        us = lambda x: (x - e) / ghz / 1e3
        rounds = []
        r = 0
        while 4 + 4 * r < 59 and t[1 + 4 * r] > e:
            rounds.append(f"r{r} {us(t[1 + 4 * r]):.2f}/{us(t[2 + 4 * r]):.2f}/{us(t[3 + 4 * r]):.2f}/{us(t[4 + 4 * r]):.2f}")
            r += 1
        print(f"launch {k}: count+record {us(t[60]):.2f} us, setup {us(t[59]):.2f}, first round {us(t[0]):.2f}, "
              f"end {us(t[63]):.2f}, written {us(t[61]):.2f}; rounds (start/eval/accept/solve) " + "  ".join(rounds))
    env.close()


if __name__ == "__main__":
    main()
