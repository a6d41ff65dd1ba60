"""Probe: HIP timing events recorded inside a captured hipGraph (torch.cuda.Event(external=True)),
bracketing exactly K steps after a pre-roll of P steps in the same graph, against events around
whole-graph launches.  65 536 aged HeliHover envs."""
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "heli-gym_amd")]
import ctypes  # noqa: E402

import torch  # noqa: E402
from heligym_amd import HeliVecEnv  # noqa: E402

# torch refuses external events on ROCm; the HIP runtime records them as graph event-record nodes
hip = ctypes.CDLL("libamdhip64.so")


class HipEvent:
    def __init__(self):
        self.h = ctypes.c_void_p()
        assert hip.hipEventCreate(ctypes.byref(self.h)) == 0

    def elapsed_time(self, other):
        ms = ctypes.c_float()
        rc = hip.hipEventElapsedTime(ctypes.byref(ms), self.h, other.h)
        assert rc == 0, rc
        return ms.value


def chk(rc, what):
    assert rc == 0, f"{what}: {rc}"


class TimedGraph:
    """child(pre-roll graph) -> event e0 -> child(timed graph) -> event e1, one hipGraph (explicit API)."""

    def __init__(self, g_pre, g_timed):
        self.e0, self.e1 = HipEvent(), HipEvent()
        self.graph = ctypes.c_void_p()
        chk(hip.hipGraphCreate(ctypes.byref(self.graph), ctypes.c_uint(0)), "hipGraphCreate")
        prev = None
        for kind, obj in (("child", g_pre), ("event", self.e0), ("child", g_timed), ("event", self.e1)):
            node = ctypes.c_void_p()
            deps = (ctypes.c_void_p * 1)(prev) if prev is not None else None
            nd = ctypes.c_size_t(1 if prev is not None else 0)
            if kind == "child":
                chk(hip.hipGraphAddChildGraphNode(ctypes.byref(node), self.graph, deps, nd,
                                                  ctypes.c_void_p(obj.raw_cuda_graph())), "child node")
            else:
                chk(hip.hipGraphAddEventRecordNode(ctypes.byref(node), self.graph, deps, nd, obj.h), "event node")
            prev = node
        self.exec = ctypes.c_void_p()
        chk(hip.hipGraphInstantiate(ctypes.byref(self.exec), self.graph, None, None, ctypes.c_size_t(0)),
            "instantiate")

    def replay(self):
        chk(hip.hipGraphLaunch(self.exec, ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)), "launch")

    def inner_ms(self):
        return self.e0.elapsed_time(self.e1)


N, P = 65536, 100
env = HeliVecEnv(N, task="hover", dt=0.01, seed=1234, autoreset=True, device="cuda:0")
env.reset()
bank = torch.empty((P, N, 4), dtype=torch.float32, device=env.device)
for k in range(P):
    env.random_actions(bank[k], seed=0x5EED, step=k)
for k in range(3000):
    env.step_async(bank[k % P], with_reset_info=False)
torch.cuda.synchronize()
for K in (20, 100, 1000):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    gp, gk = torch.cuda.CUDAGraph(keep_graph=True), torch.cuda.CUDAGraph(keep_graph=True)
    with torch.cuda.graph(gp, stream=s):
        for k in range(P):
            env.step_async(bank[k], with_reset_info=False)
    with torch.cuda.graph(gk, stream=s):
        for k in range(K):
            env.step_async(bank[k % P], with_reset_info=False)
    tg = TimedGraph(gp, gk)
    tg.replay()
    torch.cuda.synchronize()
    inner, outer = [], []
    for r in range(5):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        tg.replay()
        b.record()
        torch.cuda.synchronize()
        inner.append(tg.inner_ms() * 1e3 / K)
        outer.append(a.elapsed_time(b) * 1e3 / (P + K))
    print(f"K={K:5d}: inner {statistics.median(inner):7.3f} us/step {[round(x, 3) for x in inner]}  "
          f"outer {statistics.median(outer):7.3f} us/step", flush=True)
    del tg, gp, gk
env.close()
