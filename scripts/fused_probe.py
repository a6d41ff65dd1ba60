"""Where the time of a fused same-step re-trim launch goes (step_fused_kernel), from an HG_TIMING=1 build
(HELIGYM_AMD_LIB=<that .so>): the bench's aged 65 536-env same-step re-trim population, a few probed
launches; per launch the step waves' start / end spread and, per trim job, the claim, the record's
arrival and the write-out (s_memrealtime, 100 MHz), all relative to the first step wave's start.
Diagnostic only."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "heli-gym_amd"))


def main():
    import torch
    serial = "serial" in sys.argv[1:]   # the serial path instead (step kernel, then retrim_kernel)
    sys.argv = ["bench.py", "--reset-mode", "retrim", "--autoreset-mode", "same_step"]
    import bench
    args = bench.parse()
    dev = torch.device("cuda:0")
    N, B = args.envs, 64
    env = bench.make_env(args, torch, N, 0, dev)
    bank = bench.action_bank(args, torch, env, N, dev, B)
    if serial:
        env.set_retrim_overlap(False)
    bench.age(args, torch, env, bank, B)
    lib = env.lib
    for fn in (lib.hg_debug_timing, lib.hg_debug_fused_probe):
        fn.argtypes = [ctypes.c_void_p, ctypes.c_int64]
    waves = (N + 63) // 64
    tim = np.zeros((2048, 17), dtype=np.uint64)
    probe = np.zeros((1024, 4), dtype=np.uint64)
    for k in range(6):
        probe[:] = 0
        env.step_async(bank[k % B], with_reset_info=False)
        torch.cuda.synchronize()
        assert lib.hg_debug_timing(tim.ctypes.data, tim.nbytes) == 0
        assert lib.hg_debug_fused_probe(probe.ctypes.data, probe.nbytes) == 0
        t = tim[:waves].astype(np.int64)
        p = probe.astype(np.int64)
        t0 = t[:, 15].min()
        st, en = (t[:, 15] - t0) / 100.0, (t[:, 14] - t0) / 100.0   # us
        q = lambda x: " ".join(f"{v:6.2f}" for v in np.percentile(x, [0, 50, 90, 99, 100]))
        print(f"launch {k}: step waves start [min p50 p90 p99 max] {q(st)} us; end {q(en)} us")
        # (the probe buffer keeps earlier launches' jobs: this launch's are those claimed within 1 ms)
        jobs = np.nonzero((p[:, 1] > 0) & (np.abs(p[:, 0] - t0) < 100000) & (p[:, 1] >= p[:, 0]))[0]
        seen = p[jobs]
        if len(jobs):
            cl, ar, wr = [(seen[:, c] - t0) / 100.0 for c in range(3)]
            print(f"  {len(jobs)} trims: claim {q(cl)}; record {q(ar)}; written {q(wr)}; "
                  f"trim time {q(wr - ar)}")
    env.close()


if __name__ == "__main__":
    main()
