"""Phase timing of the device re-trim on the bench's own workload (diagnostic; an HG_TIMING=1 build
via HELIGYM_AMD_LIB): 65 536 envs, reset_mode="retrim", U(-1, 1) actions, aged; after each of S
steps, the stamps of that step's first trim (job 0 of block 0: entry, rounds, write-out), averaged.
Complements scripts/retrim_timing.py (one trim condition under a constant wind, no concurrency).
usage: python scripts/retrim_live_timing.py [envs] [autoreset_mode] [samples]"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "heli-gym_amd"))


def main():
    import torch
    from heligym_amd import HeliVecEnv
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    mode = sys.argv[2] if len(sys.argv) > 2 else "same_step"
    S = int(sys.argv[3]) if len(sys.argv) > 3 else 40
    env = HeliVecEnv(n, task="hover", dt=0.01, seed=1234, autoreset=True, reset_mode="retrim", autoreset_mode=mode)
    env.reset()
    bank = torch.empty((16, n, 4), dtype=torch.float32, device=env.device)
    for k in range(16):
        env.random_actions(bank[k], seed=0x5EED, step=k)
    for k in range(3000):   # 30 simulated seconds
        env.step_async(bank[k % 16], with_reset_info=False)
    torch.cuda.synchronize()
    fn = env.lib.hg_debug_retrim_timing
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int64]
    buf = np.zeros(64, dtype=np.uint64)
    ghz, rows, prev = 2.2, [], None
    for k in range(S):
        env.step_async(bank[k % 16], with_reset_info=False)
        torch.cuda.synchronize()
        assert fn(buf.ctypes.data, buf.nbytes) == 0
        t = buf.astype(np.int64)
        if t[63] <= t[0] or t[0] == 0 or t[0] == prev:   # no trim this step (the stamps are the last one's)
            continue
        prev = t[0]
        r, rounds = 0, []
        while 4 + 4 * r < 62 and t[1 + 4 * r] > t[0] and t[4 + 4 * r] > t[1 + 4 * r]:
            rounds.append(((t[2 + 4 * r] - t[1 + 4 * r]), (t[3 + 4 * r] - t[2 + 4 * r]), (t[4 + 4 * r] - t[3 + 4 * r])))
            r += 1
        rows.append(((t[63] - t[0]), (t[0] - t[62]) if t[62] > 0 and t[62] < t[0] else 0, rounds,
                     (t[61] - t[63]) if t[61] > t[63] else 0))
    env.close()
    if not rows:
        print("no trims stamped")
        return
    tot = np.array([r[0] for r in rows]) / ghz / 1e3
    st = np.array([r[1] for r in rows]) / ghz / 1e3
    wr = np.array([r[3] for r in rows]) / ghz / 1e3
    print(f"{len(rows)} stamped trims ({mode}): total median {np.median(tot):.2f} us (p90 {np.percentile(tot, 90):.2f}), "
          f"start-up median {np.median(st):.2f} us, write-out issue median {np.median(wr):.2f} us")
    for r in range(max(len(x[2]) for x in rows)):
        v = np.array([x[2][r] for x in rows if len(x[2]) > r]) / ghz / 1e3
        print(f"round {r}: n={len(v)}  eval {np.median(v[:, 0]):.2f}  accept+columns {np.median(v[:, 1]):.2f}  "
              f"gauss-jordan {np.median(v[:, 2]):.2f} us")


if __name__ == "__main__":
    main()
