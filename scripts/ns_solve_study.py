"""Round 5 study (host only): could the device trim's 16 x 16 Gauss-Jordan solve (2.9 us of each
Newton step, retrim_body.h) become a few fp64 MFMA Newton-Schulz iterations X <- X (2I - J X) started
from a shared inverse?  The host trim records the central-difference Jacobian of every Newton step
(hg_debug_trim_jacobians); for 200 turbulent winds around the mean wind this prints how far the
inverse at the mean wind's first step (X0) and at its trim point (X*) -- or the previous Newton step's
exact inverse -- is from each J (max |I - J X|), and how many Newton-Schulz iterations reach 1e-14.
Result (profiles/r05_ns_solve_study.txt): the Jacobians are ill-conditioned (cond ~3 000) and a gust
of a few ft/s moves them far from any shared inverse (median max|I - J X| ~ 6), so the iteration
needs 5-11 steps or diverges: not a reliable replacement for the pivoted solve.  Not built."""
import sys, ctypes, numpy as np
sys.path[:0]=['/root/repo','/root/repo/heli-gym_amd']
from heligym_amd import _abi, config
lib=_abi.load_library()
f=lib.hg_debug_trim_jacobians
f.restype=ctypes.c_int32
f.argtypes=[ctypes.POINTER(_abi.hg_config), ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32]
cfg,doc=config.make_config(task="hover", dt=0.01)
tft=np.ascontiguousarray(config.terrain_ft(config.load_terrain(doc), cfg.af.env_MAX_GR_ALT))
def jacs(w):
    J=np.zeros((20,16,16)); W=np.array(w,dtype=np.float64)
    n=f(ctypes.byref(cfg), tft.ctypes.data, 1024, 1024, W.ctypes.data, J.ctypes.data, 20)
    assert n>0, n
    return J[:n]
wm=np.array([20*np.cos(np.pi/4), 20*np.sin(np.pi/4), 0.0])
Jm=jacs(wm)
print("mean wind: Newton steps", len(Jm), "cond", [f"{np.linalg.cond(j):.0f}" for j in Jm])
X0=np.linalg.inv(Jm[0]); Xs=np.linalg.inv(Jm[-1])
rng=np.random.RandomState(1)
def ns(J, X, maxit=12):
    I=np.eye(16)
    hist=[]
    for it in range(maxit):
        E=I-J@X; e=np.abs(E).max(); hist.append(e)
        if e<1e-14: break
        X=X@(2*I-J@X)
    return it, hist
stats=[]
for t in range(200):
    w=wm+rng.normal(0,6,3)*np.array([1,1,0.5])
    Js=jacs(w)
    row=[]
    for k,J in enumerate(Js):
        Xi = X0 if k==0 else Xs
        it,h=ns(J,Xi)
        row.append((k, np.abs(np.eye(16)-J@Xi).max(), it))
    stats.append(row)
for k in range(4):
    e=[r[k][1] for r in stats if len(r)>k]; it=[r[k][2] for r in stats if len(r)>k]
    if e: print(f"step {k}: n={len(e)}  ||I-J X_init||max  median {np.median(e):.3g} max {np.max(e):.3g};  NS iterations median {np.median(it)} max {np.max(it)}")
# previous-step inverse as init
st2=[]
for t in range(100):
    w=wm+rng.normal(0,6,3)*np.array([1,1,0.5])
    Js=jacs(w)
    X=None
    for k,J in enumerate(Js):
        Xi = X0 if k==0 else Xprev
        it,h=ns(J,Xi)
        st2.append((k, h[0], it))
        Xprev=np.linalg.inv(J)
for k in range(4):
    e=[r[1] for r in st2 if r[0]==k]; it=[r[2] for r in st2 if r[0]==k]
    if e: print(f"prev-inv init step {k}: ||E0|| median {np.median(e):.3g} max {np.max(e):.3g}; iters median {np.median(it)} max {np.max(it)}")
