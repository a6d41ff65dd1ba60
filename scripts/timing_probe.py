"""Latency attribution of one step launch with a HG_TIMING=1 diagnostic build of the library
(HELIGYM_AMD_LIB=<that .so>): per-wave s_memtime stamps at phase boundaries -> median / p90 of each
phase over the recorded waves, plus the spread of wave start / end times.  Diagnostic only."""
import argparse
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "heli-gym_amd"))

PHASES = ["state loads", "philox", "wind step", "ground h_c", "RK stage 1", "RK stage 2", "RK stage 3",
          "RK stage 4 + update", "wraps + template fetch", "reward/flags/post-ground",
          "flag stores + reset + obs stores", "state stores", "store drain"]
ORDER = [0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 13, 11, 12]   # stamp slots in program order
# the small-batch helper kernel's stepping waves (step_help_kernel: slots 2-4 mark the hand-off)
PHASES_HELP = ["state loads", "context + stage-1 wind-free part", "wait at the hand-off barrier",
               "wind read from LDS", "RK stage 1", "RK stage 2", "RK stage 3", "RK stage 4 + update",
               "wraps + template fetch", "reward/flags/post-ground", "flag stores + reset + obs stores",
               "state stores", "store drain"]
HELPER = ["helper: state loads (counters, carry, wind state)", "helper: noise + wind step",
          "helper: LDS hand-off + barrier"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--warm", type=int, default=3000, help="steps before the recorded launch (aged population)")
    ap.add_argument("--dt", type=float, default=0.01)
    args = ap.parse_args()
    import torch
    from heligym_amd import HeliVecEnv
    env = HeliVecEnv(args.envs, task="hover", dt=args.dt, seed=0)
    env.reset()
    act = torch.empty((args.envs, 4), dtype=torch.float32, device=env.device)
    for k in range(args.warm):
        env.random_actions(act, seed=1, step=k)
        env.step_async(act, with_reset_info=False)
    torch.cuda.synchronize()
    buf = np.zeros((2048, 17), dtype=np.uint64)
    fn = env.lib.hg_debug_timing
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int64]
    assert fn(buf.ctypes.data, buf.nbytes) == 0
    nw = min(2048, args.envs // 64)
    t = buf[:nw, ORDER].astype(np.int64)
    rt = buf[:nw, 14:16].astype(np.int64)        # [end, start] s_memrealtime (100 MHz)
    span_cyc = (t[:, -1] - t[:, 0]).astype(np.float64)
    span_ns = (rt[:, 0] - rt[:, 1]) * 10.0
    ghz = np.median(span_cyc / np.maximum(span_ns, 1))
    print(f"waves {nw}; memtime clock ~{ghz:.2f} GHz (from realtime); wave life median "
          f"{np.median(span_ns)/1e3:.2f} us p90 {np.percentile(span_ns, 90)/1e3:.2f} us")
    starts = (rt[:, 1] - rt[:, 1].min()) * 10.0
    ends = (rt[:, 0] - rt[:, 1].min()) * 10.0
    print(f"wave start spread: p50 {np.median(starts)/1e3:.2f} us p90 {np.percentile(starts, 90)/1e3:.2f} "
          f"max {starts.max()/1e3:.2f} us; last wave end {ends.max()/1e3:.2f} us")
    d = np.diff(t, axis=1).astype(np.float64) / ghz / 1e3   # us
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    helper = args.envs <= 64 * 4 * cus // 2   # heligym_amd.hip launch_step: HG_HELPER_DIV = 2
    if helper:
        hb = np.zeros((2048, 5), dtype=np.uint64)
        fh = env.lib.hg_debug_timing_help
        fh.argtypes = [ctypes.c_void_p, ctypes.c_int64]
        assert fh(hb.ctypes.data, hb.nbytes) == 0
        h = hb[:nw].astype(np.int64)
        hd = np.diff(h[:, 1:5], axis=1).astype(np.float64) / ghz / 1e3
        hstart = (h[:, 0] - rt[:, 1].min()) * 10.0
        print(f"helper waves: start p50 {np.median(hstart)/1e3:.2f} us (stepping waves {np.median(starts)/1e3:.2f}); "
              f"life to the barrier median {np.median((h[:, 4] - h[:, 1]) / ghz) / 1e3:.2f} us")
        for j, name in enumerate(HELPER):
            print(f"  {name:48s} median {np.median(hd[:, j]):6.3f} us   p90 {np.percentile(hd[:, j], 90):6.3f} us")
        print("stepping waves:")
    for j, name in enumerate(PHASES_HELP if helper else PHASES):
        print(f"  {name:24s} median {np.median(d[:, j]):6.3f} us   p90 {np.percentile(d[:, j], 90):6.3f} us   "
              f"max {d[:, j].max():6.3f} us")
    # which wave-uniform branches the waves took, and how long those waves lived
    fl = buf[:nw, 16].astype(np.int64)
    names = {1: "reset", 2: "gear contact", 4: "full sincos"}
    print(f"branch flags: " + ", ".join(f"{v} {int(((fl & b) != 0).sum())} waves" for b, v in names.items()))
    for cls, sel in (("no branch", fl == 0), ("reset only", fl == 1), ("gear", (fl & 2) != 0),
                     ("full sincos", (fl & 4) != 0)):
        if sel.any():
            print(f"  {cls:12s} {int(sel.sum()):5d} waves: life median {np.median(span_ns[sel])/1e3:.2f} us, "
                  f"max {span_ns[sel].max()/1e3:.2f} us; end median {np.median(ends[sel])/1e3:.2f} max {ends[sel].max()/1e3:.2f} us")
    last = np.argsort(ends)[-20:]
    print("the 20 last-ending waves: flags", fl[last].tolist(), "start", np.round(starts[last] / 1e3, 2).tolist())
    env.close()


if __name__ == "__main__":
    main()
