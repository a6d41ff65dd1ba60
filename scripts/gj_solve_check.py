"""Diagnostic: the device trim's 16 x 16 Newton solve on its own (scripts/ubench/gj_solve.hip), the
blocked MFMA Gauss-Jordan (csrc/gj_mfma.h, which=0) and the unblocked split-row solve (which=1), against
numpy.linalg.solve on (a) the host trim's central-difference Jacobians of 300 turbulent winds (the
systems the device trim solves, cond ~3 000), (b) random Gaussian systems, (c) systems that need row
exchanges (zero diagonal), and (d) a singular one (must come out non-finite).  Prints the error in
units of cond(J) * eps * |x| and the cycles per solve (s_memtime)."""
import ctypes
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "heli-gym_amd")]
SO = os.path.join(ROOT, "build", "gj_solve.so")
# (name, extra flags): the stamped build, the same without stamps (true cycles), one Newton step after v_rcp_f64
VARIANTS = [("gj_solve", []), ("gj_solve_nostamp", ["-DGJ_NO_STAMPS"]), ("gj_solve_nr1", ["-DGJ_NO_STAMPS", "-DGJM_RCP_NR=1"]),
            ("gj_solve_steps", ["-DGJ_NO_STAMPS", "-DGJS_BLOCK_INV=0"])]   # (the static solve's pivot steps)


def build():
    src = os.path.join(ROOT, "scripts", "ubench", "gj_solve.hip")
    os.makedirs(os.path.dirname(SO), exist_ok=True)
    for name, fl in VARIANTS:
        subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
                               "-ffp-contract=on", "-mllvm", "-amdgpu-mfma-vgpr-form", *fl, "-o",
                               os.path.join(ROOT, "build", name + ".so"), src])


def pivot_order(J):
    """The rows partial pivoting (first largest |entry|, the host's solve16) takes for columns 0..15."""
    M = np.array(J, dtype=np.float64)
    idx = np.arange(16)
    for c in range(16):
        p = c + int(np.argmax(np.abs(M[c:, c])))
        M[[c, p]] = M[[p, c]]
        idx[[c, p]] = idx[[p, c]]
        M[c] /= M[c, c]
        for i in range(16):
            if i != c:
                M[i] -= M[i, c] * M[c]
    return idx


def jacobians(n, with_steps=False):
    from heligym_amd import _abi, config
    lib = _abi.load_library()
    f = lib.hg_debug_trim_jacobians
    f.restype = ctypes.c_int32
    f.argtypes = [ctypes.POINTER(_abi.hg_config), ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p,
                  ctypes.c_void_p, ctypes.c_int32]
    cfg, doc = config.make_config(task="hover", dt=0.01)
    tft = np.ascontiguousarray(config.terrain_ft(config.load_terrain(doc), cfg.af.env_MAX_GR_ALT))
    rng = np.random.RandomState(7)
    wm = np.array([20 * np.cos(np.pi / 4), 20 * np.sin(np.pi / 4), 0.0])
    def run(W):
        J = np.zeros((20, 16, 16))
        k = f(ctypes.byref(cfg), tft.ctypes.data, 1024, 1024, np.asarray(W, np.float64).ctypes.data, J.ctypes.data, 20)
        return J[:max(k, 0)]
    out, steps = [], []
    while len(out) < n:
        Js = run(wm + rng.normal(0, 6, 3) * np.array([1, 1, 0.5]))
        out.extend(Js)
        steps.extend(range(len(Js)))
    if not with_steps:
        return np.array(out[:n])
    # the pivot order of the mean-wind trim's own Newton steps (hg::TrimSetup::piv), step k >= 3 uses 3
    mean = [pivot_order(J) for J in run(wm)]
    perms = np.array([mean[min(k, len(mean) - 1)] for k in steps[:n]], dtype=np.int8)
    return np.array(out[:n]), perms


def main():
    if "--build" in sys.argv or not os.path.exists(SO):
        build()
    lib = ctypes.CDLL(SO)
    lib.gj_solve_run.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_int] * 2 + [ctypes.c_void_p] * 3 + [ctypes.c_int]
    lib.gj_solve_stamps.argtypes = [ctypes.c_void_p]
    rng = np.random.RandomState(3)
    tj, tperm = jacobians(300, with_steps=True)
    sets = {"trim jacobians": tj, "gaussian": rng.normal(size=(200, 16, 16))}
    perms = {"trim jacobians": tperm, "gaussian": np.array([pivot_order(J) for J in sets["gaussian"]], np.int8)}
    zd = rng.normal(size=(100, 16, 16))
    for k in range(100):
        np.fill_diagonal(zd[k], 0.0)
        zd[k][:, rng.permutation(16)[:4]] *= 1e-3   # a few small columns
    sets["zero diagonal"] = zd
    perms["zero diagonal"] = np.tile(np.arange(16, dtype=np.int8), (100, 1))   # identity: zero pivots, must fall back
    sing = rng.normal(size=(4, 16, 16))
    for k in range(4):
        sing[k][:, 5] = sing[k][:, 3] * 2.0
    eps = np.finfo(np.float64).eps
    for name, J in sets.items():
        J = np.ascontiguousarray(J)
        b = np.ascontiguousarray(rng.normal(size=(len(J), 16)) * 10)
        ref = np.linalg.solve(J, b[..., None])[..., 0]
        cond = np.linalg.cond(J)
        pm = np.ascontiguousarray(perms[name])
        for which, label in ((0, "blocked mfma"), (1, "split rows"), (2, "static pivots")):
            x = np.zeros_like(b)
            cyc = np.zeros(len(J), np.uint64)
            fb = np.zeros(len(J), np.int32)
            assert lib.gj_solve_run(J.ctypes.data, b.ctypes.data, pm.ctypes.data, len(J), which, x.ctypes.data,
                                    cyc.ctypes.data, fb.ctypes.data, 256) == 0
            err = np.abs(x - ref).max(1) / (cond * eps * (np.abs(ref).max(1) + 1))
            res = np.abs(np.einsum("nij,nj->ni", J, x) - b).max(1) / (eps * (np.abs(J).max((1, 2)) * np.abs(x).max(1) * 16 + np.abs(b).max(1)))
            print(f"{name:15s} {label:13s} n={len(J)} err/(cond eps |x|) max {np.nanmax(err):.3g} median {np.nanmedian(err):.3g}"
                  f"  backward err/eps max {np.nanmax(res):.3g}  finite {np.isfinite(x).all()}  cycles median {np.median(cyc):.0f}"
                  + (f"  fell back {int(fb.sum())} (cycles median of those {np.median(cyc[fb == 1]) if fb.any() else 0:.0f})"
                     if which == 2 else ""))
    # phase stamps of the blocked solve (job 0, one wave alone on the GPU)
    J = np.ascontiguousarray(sets["trim jacobians"][:1])
    b = np.ascontiguousarray(rng.normal(size=(1, 16)))
    x = np.zeros((1, 16))
    cyc = np.zeros(1, np.uint64)
    fb = np.zeros(1, np.int32)
    pm = np.ascontiguousarray(perms["trim jacobians"][:1])
    for which, label in ((0, "blocked"), (2, "static pivots")):
        for _ in range(3):
            assert lib.gj_solve_run(J.ctypes.data, b.ctypes.data, pm.ctypes.data, 1, which, x.ctypes.data,
                                    cyc.ctypes.data, fb.ctypes.data, 1) == 0
        t = np.zeros(40, np.uint64)
        assert lib.gj_solve_stamps(t.ctypes.data) == 0
        t = t.astype(np.int64)
        print(f"{label} solve, one wave, cycles: {int(cyc[0])} (fell back: {int(fb[0])})")
        for pn in range(4):
            b0 = t[8 * pn]
            if which == 0:
                seg = [t[8 * pn + 1] - b0] + [t[8 * pn + 2 + k] - t[8 * pn + 1 + k] for k in range(4)]
            else:
                seg = [0] + [t[8 * pn + 2] - b0] + [t[8 * pn + 3 + k] - t[8 * pn + 2 + k] for k in range(3)]
            seg.append(t[8 * pn + 6] - t[8 * pn + 5])
            nxt = t[8 * pn + 8] if pn < 3 else t[32]
            print(f"  panel {pn}: gather {seg[0]}, steps {seg[1:5]}, operands {seg[5]}, mfma->next {nxt - t[8 * pn + 6]}")
        if which == 2:
            print(f"  residual check {t[33] - t[32]}")
    # cycles without the phase stamps, and with one Newton step after v_rcp_f64
    J = np.ascontiguousarray(sets["trim jacobians"])
    pm = np.ascontiguousarray(perms["trim jacobians"])
    b = np.ascontiguousarray(rng.normal(size=(len(J), 16)) * 10)
    ref = np.linalg.solve(J, b[..., None])[..., 0]
    cond = np.linalg.cond(J)
    for name, _ in VARIANTS[1:]:
        lv = ctypes.CDLL(os.path.join(ROOT, "build", name + ".so"))
        lv.gj_solve_run.argtypes = lib.gj_solve_run.argtypes
        for which, label in ((0, "blocked mfma"), (1, "split rows"), (2, "static pivots")):
            x = np.zeros_like(b)
            cyc = np.zeros(len(J), np.uint64)
            fb = np.zeros(len(J), np.int32)
            assert lv.gj_solve_run(J.ctypes.data, b.ctypes.data, pm.ctypes.data, len(J), which, x.ctypes.data,
                                   cyc.ctypes.data, fb.ctypes.data, 256) == 0
            err = np.abs(x - ref).max(1) / (cond * eps * (np.abs(ref).max(1) + 1))
            print(f"[{name}] trim jacobians {label:13s} cycles median {np.median(cyc):.0f}  err/(cond eps |x|) max "
                  f"{err.max():.3g}  fell back {int(fb.sum())}")
    lib.gj_dpp_check.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    vin = np.ascontiguousarray(np.arange(64, dtype=np.float64) + 1.5)
    dout = np.zeros((64, 3))
    assert lib.gj_dpp_check(vin.ctypes.data, dout.ctypes.data) == 0
    src = vin.reshape(4, 16)[:, 3].repeat(16)
    print("DPP row_newbcast:3 -- v_mov_b64 ok:", np.array_equal(dout[:, 0], src),
          " v_rcp_f64 ok:", np.allclose(dout[:, 1], 1 / src, rtol=1e-7), "(own-lane rcp:", np.allclose(dout[:, 1], 1 / vin, rtol=1e-7), ")",
          " v_fmac_f64 ok:", np.array_equal(dout[:, 2], vin + 2 * src))
    lib.gj_rcp_check.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
    xs = np.ascontiguousarray(np.concatenate([rng.uniform(-50, 50, 100000), 10.0 ** rng.uniform(-6, 6, 100000)]))
    er = np.zeros((len(xs), 3))
    assert lib.gj_rcp_check(xs.ctypes.data, er.ctypes.data, len(xs)) == 0
    print("v_rcp_f64 |r x - 1| max: raw %.3g, 1 Newton step %.3g, 2 steps %.3g (eps %.3g)" % (*er.max(0), eps))
    for which, label in ((0, "blocked mfma"), (1, "split rows"), (2, "static pivots")):
        x = np.zeros((4, 16))
        cyc = np.zeros(4, np.uint64)
        b = rng.normal(size=(4, 16))
        fb = np.zeros(4, np.int32)
        pm = np.tile(np.arange(16, dtype=np.int8), (4, 1))
        assert lib.gj_solve_run(sing.ctypes.data, b.ctypes.data, pm.ctypes.data, 4, which, x.ctypes.data,
                                cyc.ctypes.data, fb.ctypes.data, 4) == 0
        print(f"singular        {label:13s} every solution non-finite: {(~np.isfinite(x).all(1)).all()}  |x| max {np.abs(x).max():.3g}")


if __name__ == "__main__":
    main()
