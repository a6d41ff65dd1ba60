"""Diagnostic: attribute the fp32 step's error on one observation to (a) the formula that forms it
from the stage-4 input state and (b) the stage-4 input state itself, on the CPU.

scripts/f32_probe.cpp compiles the kernel's own fp32 step source (stage_f32.h) for the host with the
same multiply-add fusion; this script runs it on the cases of tests/test_gpu_parity.py's tumbling
test and compares, per case:
  total   = probe obs - oracle obs (the oracle's own fp64 stage-4 state)
  formula = probe obs - oracle dynamics evaluated at the PROBE's fp32 stage-4 state
  state   = the difference of the two (what the stage-4 input state's own error costs)
in units of contract (i).  Usage: python scripts/f32_probe.py [col] [lo hi]
"""
import ctypes
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "heli-gym_amd"), os.path.join(ROOT, "tests")]
SO = os.path.join(ROOT, "build", "f32_probe.so")


def build(extra=()):
    src = os.path.join(ROOT, "scripts", "f32_probe.cpp")
    subprocess.check_call(["/opt/rocm/bin/hipcc", "-x", "hip", "--offload-host-only", "-O2", "-std=c++17", "-fPIC",
                           "-shared", "-mfma", "-ffp-contract=on", *extra, "-o", SO, src])
    return ctypes.CDLL(SO)


def params_bytes(lib_hg, cfg, rows, cols, size):
    buf = ctypes.create_string_buffer(size)
    from heligym_amd import _abi
    _abi.check(lib_hg.hg_debug_params(ctypes.byref(cfg), rows, cols, 0, buf, size), lib_hg)
    return buf


def tumbling_cases(rates, seed=7):
    import golden_cases as gc
    b = gc.single_step_batch(gc.load("0.01"), "hover")
    rng = np.random.RandomState(seed)
    keep = np.nonzero(b["obs"][:, 16] > 50.0)[0][:400]
    b = {k: (v[keep] if isinstance(v, np.ndarray) and len(v) == len(b["state"]) else v) for k, v in b.items()}
    n = len(b["state"])
    mag = rng.uniform(rates[0], rates[1], size=(n, 3)) * rng.choice([-1.0, 1.0], size=(n, 3))
    b["state"] = b["state"].copy()
    b["state"][:, 9:12] = mag
    return b


def main():
    col = int(sys.argv[1]) if len(sys.argv) > 1 else 0
    rates = (float(sys.argv[2]), float(sys.argv[3])) if len(sys.argv) > 3 else (12.0, 40.0)
    from heligym_amd import _abi, config
    from oracle.oracle import Oracle
    lib_hg = _abi.load_library()
    pl = build()
    pl.probe_step.argtypes = [ctypes.c_void_p] * 11
    size = pl.probe_params_size()
    cfg, doc = config.make_config(task="hover", dt=0.01)
    u16 = config.load_terrain(doc)
    tft = config.terrain_ft(u16, cfg.af.env_MAX_GR_ALT)
    hi = tft.astype(np.float32)
    lo = (tft - hi.astype(np.float64)).astype(np.float32)
    hmap = np.ascontiguousarray(np.stack([hi, lo], -1))
    P = params_bytes(lib_hg, cfg, tft.shape[0], tft.shape[1], size)
    orc = Oracle(cfg, u16)
    b = tumbling_cases(rates)
    F = ctypes.POINTER(ctypes.c_float)
    D = ctypes.POINTER(ctypes.c_double)
    fp = lambda a: a.ctypes.data_as(F)  # noqa: E731
    dp = lambda a: a.ctypes.data_as(D)  # noqa: E731
    rows = []
    for i in range(len(b["state"])):
        s32 = b["state"][i].astype(np.float32)
        act = b["actions"][i].astype(np.float32)
        eta = b["eta"][i].astype(np.float32)
        obs, st4, W, hc = np.zeros(17, np.float32), np.zeros(18, np.float32), np.zeros(3, np.float32), np.zeros(1, np.float32)
        hs, k4 = np.zeros(18, np.float32), np.zeros(18, np.float32)
        pl.probe_step(ctypes.addressof(P), hmap.ctypes.data, fp(s32), fp(act), fp(eta), fp(obs), fp(st4), fp(W), fp(hc), fp(hs), fp(k4))
        s = s32.astype(np.float64)
        prev = np.zeros(17)
        prev[4:7], prev[16] = s[23:26], s[26]
        e = orc.env_from(s[:18], s[18:23], prev, np.zeros(18), 0.0, 0.0)
        o = orc.step(e, act, eta)
        ref = np.array(o.obs)
        # oracle dynamics at the probe's fp32 stage-4 state, wind and ground
        d = np.zeros(18)
        obs_at = np.zeros(17)
        orc.lib.or_dynamics(orc.m, dp(st4.astype(np.float64)), dp(act.astype(np.float64)),
                            dp(W.astype(np.float64)), float(hc[0]), dp(d), dp(obs_at))
        tol = 2e-4 + 2e-5 * abs(ref[col])
        rows.append(((obs[col] - ref[col]) / tol, (obs[col] - obs_at[col]) / tol, (obs_at[col] - ref[col]) / tol,
                     ref[col], i))
    r = np.array(rows)
    order = np.argsort(-np.abs(r[:, 0]))
    print(f"obs[{col}] rates {rates}: {len(r)} cases; |total|/tol max {np.abs(r[:, 0]).max():.3f}, "
          f"|formula| max {np.abs(r[:, 1]).max():.3f}, |state| max {np.abs(r[:, 2]).max():.3f}")
    for j in order[:12]:
        print(f"  case {int(r[j, 4]):4d} ref {r[j, 3]:12.4f} total {r[j, 0]:+.3f} formula {r[j, 1]:+.3f} state {r[j, 2]:+.3f}")


if __name__ == "__main__":
    main()
