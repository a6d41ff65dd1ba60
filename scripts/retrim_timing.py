"""Phase timing of the device re-trim (retrim_kernel) from an HG_TIMING=1 build
(HELIGYM_AMD_LIB=<that .so>): per Newton round, the trim_fcn evaluation, the trial acceptance and
the Gauss-Jordan solve of the first job.  Diagnostic only."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "heli-gym_amd"))


def main():
    import torch
    from heligym_amd import HeliVecEnv
    env = HeliVecEnv(64, task="hover", dt=0.01)
    w = np.array([[16.0, 12.0, 0.5]] * 130, dtype=np.float32)
    for _ in range(3):
        env.trim_batch(w)
    torch.cuda.synchronize()
    buf = np.zeros(64, dtype=np.uint64)
    fn = env.lib.hg_debug_retrim_timing
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int64]
    assert fn(buf.ctypes.data, buf.nbytes) == 0
    t = buf.astype(np.int64)
    ghz = 2.2
    print(f"total {(t[63] - t[0]) / ghz / 1e3:.2f} us (at {ghz} GHz)")
    if t[62] > 0:   # kernel entry -> the first job's start (job count, record, trim setup)
        print(f"start-up {(t[0] - t[62]) / ghz / 1e3:.2f} us")
    r = 0
    while 4 + 4 * r < 63 and t[1 + 4 * r] > 0 and t[4 + 4 * r] > 0:
        e = (t[2 + 4 * r] - t[1 + 4 * r]) / ghz / 1e3
        acc = (t[3 + 4 * r] - t[2 + 4 * r]) / ghz / 1e3
        gj = (t[4 + 4 * r] - t[3 + 4 * r]) / ghz / 1e3
        print(f"round {r}: eval {e:6.2f} us  accept+columns {acc:6.2f} us  gauss-jordan {gj:6.2f} us")
        r += 1
    names = ["multiplier read + pivot search (DPP reduction) + readlanes", "pivot row read + scaling",
             "elimination"]
    for c in range(2):
        s = t[40 + 6 * c: 44 + 6 * c]
        if np.all(s > 0):
            print(f"pivot step {c}: " + ", ".join(f"{n} {(s[k + 1] - s[k]) / ghz:.0f} cyc" for k, n in enumerate(names)))
    env.close()


if __name__ == "__main__":
    main()
