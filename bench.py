#!/usr/bin/env python3
"""Throughput of the vectorised heli-gym step on MI355X (BASELINE.json metric).

One "step" = one hg_step launch advancing every env of every rank by one env-step (wind RK,
helicopter RK4, reward, flags, auto-reset) with actions read from HBM.  Workload (BASELINE.json
configs[2]): 65 536 HeliHover-v0 envs per GPU, Dryden turbulence on (level 1), dt = 0.01 s, fp32,
U(-1,1) random actions (a Philox-generated bank resident in HBM before timing), auto-reset on.

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...   (one rank per GPU)

`--gpus N` without a torch.distributed launcher starts one itself (a child process; this parent
never touches the GPU).  Prints ONE JSON line on rank 0.  Envs shard with no data-path collective
(weak scaling).  With N > 1 the line also carries BASELINE config 5 (1 048 576 envs sharded over
the ranks, observations gathered to rank 0 over RCCL every step) with and without the gather;
`--gather-obs` makes that the headline instead.
"""
import argparse
import json
import os
import socket
import statistics
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for p in (ROOT, os.path.join(ROOT, "heli-gym_amd"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)

# Algorithmic HBM bytes per env-step, SURVEY 8(d): read 132 B (heli + wind state 23 fp32, carry 4,
# counters 2, action 4) + write 186 B.  Implementation extras (the episode-index counter that keys
# the noise, 4 + 4 B; the info byte, 1 B) are not algorithmic and are not counted.  (SURVEY's write
# total itself is 4 B short of its own item list, 29 x 4 + 68 + 4 + 1 + 1 = 190: keeping 318 B makes
# `achieved` conservative.)
BYTES_PER_ENV_STEP = 318
# what the kernel actually moves (bytes the PMC traffic is compared with): reads 128 (state tile
# 112: heli 16 + wind 5 + carry 4 + counters 3 words, the rotor azimuths are not stepped; action 16),
# writes 187 (state tile 112, obs 68, reward 4, terminated / truncated / info 3)
IMPL_BYTES_PER_ENV_STEP = 128 + 187
# hg_rollout: per step action 16 + obs 68 + reward 4 + flags 2; state + counters once per launch
ROLLOUT_BYTES_PER_ENV_STEP = 16 + 68 + 4 + 2
BYTES_STATE_RW = 2 * 112
HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md (spec; 6.3 TB/s measured copy)
REFERENCE_NUMPY_PER_CORE = 1367.0   # env-steps/s/core, reference on config 1
CONFIG5_TOTAL = 1048576             # BASELINE configs[4]
OUT_OF_CACHE_ENVS = 4194304         # 1.32 GB moved per launch: past the 256 MB Infinity Cache


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1000, help="steps per timed window (exactly)")
    ap.add_argument("--warmup", type=int, default=100)
    ap.add_argument("--repeats", type=int, default=5, help="timed windows; the median is reported")
    ap.add_argument("--age-seconds", type=float, default=60.0,
                    help="simulated seconds every env population is stepped (untimed, after reset) before its "
                         "graphs are captured, so that timed windows see steady-state episode phases and resets")
    ap.add_argument("--envs", type=int, default=65536, help="envs per GPU")
    ap.add_argument("--dt", type=float, default=0.01)
    ap.add_argument("--task", default="hover", choices=["hover", "forward_flight", "heli"])
    ap.add_argument("--rollout-steps", type=int, default=100,
                    help="also time hg_rollout (this many steps per launch, same action bank); 0 = off")
    ap.add_argument("--reset-mode", default="template", choices=["template", "retrim"],
                    help="auto-reset state: mean-wind trim template (default) or per-reset device re-trim (F8)")
    ap.add_argument("--autoreset-mode", default="same_step", choices=["same_step", "next_step"],
                    help="auto-reset in the step that ends the episode (default) or in the next one (gymnasium)")
    ap.add_argument("--max-episode-steps", type=int, default=None, help="TimeLimit (gymnasium registry: 5000)")
    ap.add_argument("--graph-steps", type=int, default=100, help="steps captured per hipGraph")
    ap.add_argument("--gather-obs", action="store_true",
                    help="headline = BASELINE config 5: obs gathered to rank 0 every step (needs N > 1)")
    ap.add_argument("--no-config5", action="store_true", help="N > 1: skip the config-5 secondary figure")
    ap.add_argument("--config5-timeout", type=float, default=float(os.environ.get("HG_BENCH_CONFIG5_TIMEOUT", 240)),
                    help="wall-clock limit (s) of the config-5 child run; past it the child is killed and the line "
                         "carries config5.error")
    ap.add_argument("--config5-only", action="store_true",
                    help="(internal) the config-5 child: measure BASELINE config 5 only, print {'config5': ...}")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline sample budget")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-parity", action="store_true")
    ap.add_argument("--no-secondary", action="store_true", help="headline only (profiling runs)")
    ap.add_argument("--generic-kernel", action="store_true",
                    help="step with the generic kernel instead of the default airframe's constant-specialised one")
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher / rank / timing plumbing only, no kernel (CPU tests); value is null")
    return ap.parse_args()


# ------------------------------------------------------------------------------------ launcher
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch(args):
    """--gpus N > 1 without WORLD_SIZE: run N ranks under torch.distributed.run as a child process
    (this process imports no GPU code) and exit with its status."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__), *sys.argv[1:]]
    return subprocess.call(cmd)


def run_config5_child(args, world):
    """BASELINE config 5 (1 048 576 envs over the ranks, RCCL gather to rank 0) in a child run of its
    own, started by rank 0 BEFORE this process touches the GPU or joins the process group (the other
    ranks wait in the rendezvous), under a wall-clock limit: an RCCL error, a crash or a hang in the
    child costs only its own block of the line ({"error": ...}), never the headline.  The child is
    `torch.distributed.run` over the same N GPUs (or, for the one-rank rehearsal, one process), each
    of its ranks also bounded by a watchdog (os._exit) a little inside the limit."""
    import signal
    import tempfile
    limit = max(10.0, args.config5_timeout)
    argv = [a for a in sys.argv[1:] if a != "--config5-only"] + ["--config5-only"]
    me = os.path.abspath(__file__)
    if world > 1:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
               "--master-addr=127.0.0.1", f"--master-port={_free_port()}", me, *argv]
    else:
        cmd = [sys.executable, me, *argv]
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "GROUP_RANK", "ROLE_RANK",
                        "ROLE_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT", "TORCHELASTIC_RUN_ID",
                        "TORCHELASTIC_RESTART_COUNT", "TORCHELASTIC_MAX_RESTARTS", "TORCHELASTIC_USE_AGENT_STORE",
                        "TORCH_NCCL_ASYNC_ERROR_HANDLING")}
    if os.environ.get("HG_BENCH_CONFIG5_NO_WATCHDOG") != "1":   # (CPU test of the parent's kill path)
        env["HG_BENCH_CONFIG5_WATCHDOG"] = str(limit - 5.0)
    progress(f"config5: child run ({world} ranks, limit {limit:.0f} s)")
    t0 = time.perf_counter()
    with tempfile.TemporaryFile(mode="w+") as out, tempfile.TemporaryFile(mode="w+") as err:
        p = subprocess.Popen(cmd, stdout=out, stderr=err, env=env, cwd=ROOT, start_new_session=True)
        try:
            rc = p.wait(timeout=limit)
        except subprocess.TimeoutExpired:
            rc = None
            for sig, grace in ((signal.SIGTERM, 15), (signal.SIGKILL, 15)):   # the launcher stops its workers
                try:
                    os.killpg(p.pid, sig)
                except ProcessLookupError:
                    break
                try:
                    p.wait(timeout=grace)
                    break
                except subprocess.TimeoutExpired:
                    continue
        out.seek(0)
        err.seek(0)
        lines = [ln for ln in out.read().splitlines() if ln.startswith("{")]
        errtext = err.read()
        # the exceptions the ranks raised (the launcher's own summary fills the tail)
        raised = [ln.strip() for ln in errtext.splitlines() if "Error:" in ln or "Exception:" in ln][:6]
        tail = {"raised": raised, "tail": errtext[-1500:]}
    wall = time.perf_counter() - t0
    if rc is None:
        return {"error": f"config-5 child run killed at its {limit:.0f} s limit", "stderr": tail}
    if rc != 0 or not lines:
        return {"error": f"config-5 child run failed (exit status {rc})", "stderr": tail}
    try:
        c5 = json.loads(lines[-1])["config5"]
    except (ValueError, KeyError) as exc:
        return {"error": f"config-5 child run printed no config5 block ({exc!r})", "stderr": tail}
    c5["child_wall_s"] = wall
    return c5


def config5_watchdog():
    """Config-5 child ranks: leave at the limit the parent set, whatever the process is doing (a hang
    in a collective included), so that the child run ends by itself."""
    import threading
    lim = os.environ.get("HG_BENCH_CONFIG5_WATCHDOG")
    if lim:
        t = threading.Timer(float(lim), lambda: os._exit(124))
        t.daemon = True
        t.start()


def cpu_share():
    """CPUs this process may use: its affinity mask, capped by a cgroup CPU quota if one is set."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = float(q) / float(period)
    except (OSError, ValueError):
        try:
            q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            period = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            if q > 0:
                quota = q / period
        except (OSError, ValueError):
            pass
    n = aff if quota is None else max(1, min(aff, int(quota)))
    return n, aff, quota


# ------------------------------------------------------------------------------------ references
def summary_mode(d):
    """The reset path a PMC summary profiled, from the bench options it was run with (its
    `bench_args`): ("template", "same_step") for the step kernel's own profiles, ("retrim", amode) for
    the re-trim ones (retrim_kernel / step_ov_kernel).  The auto-reset mode only matters with re-trim."""
    tok = (d.get("bench_args") or "").split()
    opt = lambda k, dflt: tok[tok.index(k) + 1] if k in tok and tok.index(k) + 1 < len(tok) else dflt
    rm = opt("--reset-mode", "template")
    return (rm, opt("--autoreset-mode", "same_step") if rm == "retrim" else "same_step")


def pmc_summary(envs, dt, task, need="hbm_bytes_per_launch", tags=None, mode=("template", "same_step")):
    """The newest committed PMC summary for this workload (profiles/<tag>_pmc_summary.json, written
    by scripts/summarize_prof.py from rocprofv3 --pmc passes) that has `need`, as (dict, path), or
    None.  Newest = last in tag order; `tags` restricts the search to those tags.  The summary must
    be of the same reset path (`mode` = (reset_mode, autoreset_mode), summary_mode), so a re-trim
    line never carries the template step kernel's counters or the other way round."""
    import glob
    if mode[0] != "retrim":
        mode = ("template", "same_step")
    best = None
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc_summary.json"))):
        try:
            d = json.load(open(f))
        except Exception:
            continue
        if tags is not None and d.get("tag") not in tags:
            continue
        have = need in d or need in d.get("counters_per_launch", {})
        if (d.get("envs") == envs and abs(d.get("dt", -1) - dt) < 1e-12 and d.get("task", "hover") == task and have
                and summary_mode(d) == tuple(mode)):
            best = (d, os.path.relpath(f, ROOT))
    return best


def pattern_ceiling():
    """The committed measurement of the step kernel's own 4 M-env memory pattern (scripts/ubench/mover.hip:
    the fastest launch period over its sweeps of occupancy and independent VALU load,
    profiles/r05_mover_4m_pmc_summary.json, scripts/summarize_mover.py), or None."""
    path = os.path.join(ROOT, "profiles", "r05_mover_4m_pmc_summary.json")
    try:
        d = json.load(open(path))
        return d if "period_us_event_timed" in d else None
    except (OSError, ValueError):
        return None


def pmc_traffic(envs, dt, task, mode=("template", "same_step")):
    """HBM bytes per launch of the reset path's profiled kernel (FETCH_SIZE / WRITE_SIZE passes), or None."""
    r = pmc_summary(envs, dt, task, mode=mode)
    return None if r is None else (r[0]["hbm_bytes_per_launch"], r[1])


def shader_clock_ghz(dt, task, fallback_ghz):
    """The shader clock under this kernel's load: GRBM_GUI_ACTIVE / 8 XCDs / kernel time of the
    committed PMC summary of the out-of-cache workload (its ~0.27 ms dispatches are long enough for
    that quotient, MI355X_MICROARCH.md DVFS note); else the device's maximum clock."""
    r = pmc_summary(OUT_OF_CACHE_ENVS, dt, task, need="GRBM_GUI_ACTIVE")
    if r is not None and r[0].get("kernel_avg_ns_trace"):
        return r[0]["counters_per_launch"]["GRBM_GUI_ACTIVE"] / 8 / r[0]["kernel_avg_ns_trace"], r[1] + " (GRBM_GUI_ACTIVE / 8 / trace time)"
    return fallback_ghz, "device maximum clock"


def valu_issue(envs, dt, task, kern_s, simds, clock_ghz, mode=("template", "same_step")):
    """The VALU issue ceiling beside the HBM one: VALU wave-instructions per
    launch (SQ_INSTS_VALU of the committed PMC summary of this workload) x 4 cycles (a wave issues at
    most one VALU instruction per ~4 cycles) / (SIMDs x clock x the live per-launch time)."""
    r = pmc_summary(envs, dt, task, need="SQ_INSTS_VALU", mode=mode)
    if r is None:
        return None
    c = r[0]["counters_per_launch"]
    waves = c.get("SQ_WAVES") or 1.0
    valu = c["SQ_INSTS_VALU"]
    out = {"valu_issue_frac": valu * 4 / (simds * clock_ghz * 1e9 * kern_s),
           "valu_per_wave": valu / waves, "salu_per_wave": c.get("SQ_INSTS_SALU", 0.0) / waves,
           "valu_issue_source": f"{r[1]} (SQ_INSTS_VALU per launch) x 4 cycles / ({simds} SIMDs x "
                                f"{clock_ghz:.3f} GHz x live kernel time)"}
    return out


def cpu_baseline(dt, task, seconds):
    """Oracle (C restatement) on a bounded sample of the same workload: one host core, then the
    process's CPU share (one thread per CPU, each stepping its own envs; ctypes releases the GIL)."""
    import threading
    from heligym_amd import config
    from oracle.oracle import Oracle
    cfg, doc = config.make_config(task=task, dt=dt)
    orc = Oracle(cfg, config.load_terrain(doc))
    tr = orc.trim()
    t0 = time.perf_counter()
    n0, _ = orc.rollout(tr, 1, 2000, seed=1)
    rate0 = n0 / (time.perf_counter() - t0)
    single_s = seconds * 0.6
    steps = max(1000, int(rate0 * single_s / 64))
    t0 = time.perf_counter()
    n, _ = orc.rollout(tr, 64, steps, seed=2)
    el = time.perf_counter() - t0
    single = n / el
    threads, aff, quota = cpu_share()
    wall = seconds * 0.4 / max(1, threads // 4)   # bounded CPU work: ~0.4 x seconds x 4 core-seconds
    per = max(500, int(rate0 * wall / 16))        # steps per thread (16 envs each) for ~`wall` s
    done = [0] * threads

    def work(k):
        done[k] = orc.rollout(tr, 16, per, seed=100 + k)[0]

    ts = [threading.Thread(target=work, args=(k,)) for k in range(threads)]
    t0 = time.perf_counter()
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    elm = time.perf_counter() - t0
    return {"value": sum(done) / elm, "unit": "env-steps/s", "cores": threads, "kind": "port",
            "cores_source": f"sched_getaffinity {aff} CPUs, cgroup quota {quota}",
            "single_core_value": single,
            "reference_numpy_per_core": REFERENCE_NUMPY_PER_CORE,
            "reference_numpy_note": "the reference's own NumPy step, config 1 (1 env, zero action), measured "
                                    "in the build container (SURVEY 8(d)); the reference cannot run on the box",
            "sample": f"oracle/heli_oracle.c (dt={dt}, U(-1,1) actions, turbulence on, auto-reset): "
                      f"{threads} threads x 16 envs x {per} steps in {elm:.1f} s; single core 64 envs x "
                      f"{steps} steps in {el:.1f} s"}


def parity_error(dt, task):
    """max-abs step() error vs the reference's recorded steps (tests/golden) at this dt, and the
    error / tolerance of the parity test's contract (i) (measured input-rounding and altitude-ulp
    terms from tests/golden/rounding_terms.npz, data; see tests/test_gpu_parity.py)."""
    import numpy as np
    import torch
    import golden_cases as gc
    import rounding_terms
    from heligym_amd import HeliVecEnv
    tag = {0.01: "0.01", 0.02: "0.02"}.get(round(dt, 6))
    if tag is None or task not in ("hover", "forward_flight"):
        return None
    b = gc.single_step_batch(gc.load(tag), task)
    env = HeliVecEnv(len(b["state"]), task=task, dt=dt, autoreset=False,
                     target={"vel": 100.0} if task == "forward_flight" else None)
    env.set_state(b["state"].astype(np.float32), b["counters"].astype(np.int32))
    obs, rew, term, trunc, info = env.step(torch.as_tensor(b["actions"].astype(np.float32), device=env.device),
                                           eta=torch.as_tensor(b["eta"].astype(np.float32), device=env.device))
    st, _ = env.get_state()
    obs, st, rew = obs.cpu().numpy(), st.cpu().numpy(), rew.cpu().numpy()
    term, trunc = term.cpu().numpy(), trunc.cpu().numpy()
    env.close()
    e_obs = gc.step_errors(obs, b["obs"], gc.OBS_ANGLE_COLS)
    e_st = gc.step_errors(st[:, :18], b["heli"], gc.HELI_ANGLE_COLS)
    r_obs, r_heli, _ = rounding_terms.load(f"{tag}/{task}")
    u_obs, u_heli, _ = rounding_terms.load_ulp(f"{tag}/{task}")
    tol_o = 2e-4 + 2e-5 * np.abs(b["obs"]) + r_obs + 2 * u_obs
    tol_s = 2e-4 + 2e-5 * np.abs(b["heli"]) + r_heli + 2 * u_heli
    worst = np.maximum((e_obs / tol_o).max(axis=1), (e_st / tol_s).max(axis=1))
    contact = b["obs"][:, 16] < gc.CONTACT_GR_ALT
    flags_ok = bool(np.all(term == b["terminated"]) and np.all(trunc == b["truncated"]))
    return {"cases": int(len(b["obs"])), "obs_max_abs": float(e_obs.max()), "state_max_abs": float(e_st.max()),
            "reward_max_abs": float(np.abs(rew - b["reward"]).max()),
            "max_err_over_tol": float(worst.max()),
            "contact_cases": int(contact.sum()),
            "contact_max_err_over_tol": float(worst[contact].max()) if contact.any() else None,
            "flags_identical": flags_ok,
            "tolerance": "|d| <= 2e-4 + 2e-5|x_ref| (SURVEY 8a-i) + the step's measured fp64->fp32 "
                         "input-rounding term + 2 x its altitude-ulp sensitivity (nonzero in gear contact)"}


# ------------------------------------------------------------------------------------ timing
class Timer:
    """`repeats` windows of exactly K steps, each bracketed by barrier + synchronize with HIP events on
    the stream the work is launched on; per window the max over ranks; the median window reported.

    Each window is preceded (after the barrier and synchronize) by one untimed run of the same body,
    so that the GPU is busy when the timed region starts: the host's launch latency of the first
    graph replay (about 16 us) stays out of the window, as it does in a loop that replays graphs back
    to back (a 20-step window measured 8.6 us per step without this against 7.8 at 1 000 steps).
    With an env, the episodes begun are summed on the device right before and right after the timed
    region (queued, no host sync inside): the resets of the timed steps alone."""

    def __init__(self, torch, dist, world, dev):
        self.torch, self.dist, self.world, self.dev = torch, dist, world, dev
        self.per_rank = None   # the last run's median window of every rank (before the max)
        self.event_s = None

    def run(self, body, repeats, stream=None, env=None, preroll=True):
        t = self.torch
        s = stream if stream is not None else t.cuda.current_stream(self.dev)
        secs, walls, resets, events = [], [], 0, []
        inner = isinstance(body, TimedGraph)   # the window's clock stamps are inside the body's graph
        for _ in range(repeats):
            if self.world > 1:
                self.dist.barrier()
            t.cuda.synchronize()
            e0, e1 = t.cuda.Event(enable_timing=True), t.cuda.Event(enable_timing=True)
            if preroll and not inner:
                getattr(body, "preroll", body)()
            n0 = episodes(env, sync=False) if env is not None and not inner else None
            w0 = time.perf_counter()
            e0.record(s)
            body()
            e1.record(s)
            w1 = time.perf_counter()
            n1 = episodes(env, sync=False) if env is not None and not inner else None
            t.cuda.synchronize()
            if self.world > 1:
                self.dist.barrier()
            walls.append(max(time.perf_counter(), w1) - w0)
            secs.append(body.inner_s() if inner else e0.elapsed_time(e1) * 1e-3)
            if inner:
                events.append(e0.elapsed_time(e1) * 1e-3)
            if env is not None:
                resets += body.resets() if inner else int(n1) - int(n0)
        v = t.tensor(secs + walls, dtype=t.float64, device=self.dev)
        self.per_rank = [statistics.median(secs)]
        if self.world > 1:
            mine = t.tensor([statistics.median(secs)], dtype=t.float64, device=self.dev)
            every = [t.zeros_like(mine) for _ in range(self.world)]
            self.dist.all_gather(every, mine)
            self.per_rank = [float(x.item()) for x in every]
            self.dist.all_reduce(v, op=self.dist.ReduceOp.MAX)
        v = v.cpu().tolist()
        secs, walls = v[:repeats], v[repeats:]
        self.resets = resets
        # (TimedGraph) HIP events around each whole graph: pre-roll + counts + the K steps
        self.event_s = statistics.median(events) if events else None
        return statistics.median(secs), secs, statistics.median(walls)

    def run_counted(self, env, body, repeats, stream=None):
        """run(), plus the resets inside the timed windows (summed over ranks, per window)."""
        r = self.run(body, repeats, stream, env=env)
        n = self.resets
        if self.world > 1:
            v = self.torch.tensor([n], dtype=self.torch.int64, device=self.dev)
            self.dist.all_reduce(v)
            n = int(v.item())
        return r + (n / repeats,)


def progress(msg):
    """One line per bench phase on stderr (the JSON line stays the last line of stdout): a run that
    fails names the phase it failed in."""
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


class TimedGraph:
    """One hipGraph per window: a pre-roll of P = max(B, 1 000) steps (HG_TG_PREROLL), the episode count, a GPU clock stamp, exactly K
    steps, a second stamp, the episode count again.  The stamps (hg_clock_stamp: the constant 100 MHz
    clock, written by a one-lane kernel) bracket the K timed steps, so a window of any K measures them
    in steady state: the GPU is already stepping when the first stamp is taken, and the window holds K
    step kernels with their dependent-launch gaps plus the gap after the first stamp (about 1.6 us).
    HIP events around a short window add about 15 us of event and launch latency to it (20 steps:
    8.4-8.5 us per step against 7.6-7.7 at 1 000 steps, profiles/r04_inner_events.txt), which is why they are
    not the window's clock here; they still bracket the whole graph (`event_s`, reported beside it).
    `inner_s()` is the K steps' time, `resets()` the episodes begun in them and the W = 8 untimed
    steps right before them (the first count sits W steps before the first stamp)."""

    CLOCK_HZ = 100e6

    def __init__(self, torch, dev, one_step, K, B, env):
        import ctypes
        self.torch, self.K = torch, K
        lib = env.lib
        self.stamps = torch.zeros((2,), dtype=torch.int64, device=dev)
        s = torch.cuda.Stream(device=dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(s):
            for k in range(B):   # warm the capture stream
                one_step(k)
        torch.cuda.current_stream(dev).wait_stream(s)
        torch.cuda.synchronize()
        self.n = [None, None]

        def count(j):
            _, c = env.get_state()
            self.n[j] = c[:, 2].long().sum()

        def stamp(j):
            st = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
            if lib.hg_clock_stamp(ctypes.c_void_p(self.stamps[j:j + 1].data_ptr()), st) != 0:
                raise RuntimeError("hg_clock_stamp failed")
        # layout (A/B, profiles/r04_window_ab.txt): 0 the first episode count right before the first stamp;
        # 1 no counts; 2 (default) W = 8 plain steps between that count and the first stamp -- the
        # steps right after the count kernels run slower (20-step windows: 8.11 / 8.01 / 7.96 us);
        # a pre-roll of 1 000 steps instead of 100: 8.17 -> 7.89 us (the GPU's clock and caches settle)
        layout = int(os.environ.get("HG_TG_LAYOUT", "2"))
        W = self.W = 8 if layout == 2 else 0
        P = self.P = int(os.environ.get("HG_TG_PREROLL", str(max(B, 1000))))
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph, stream=s):
            for k in range(P - W):
                one_step(k % B)
            if layout != 1:
                count(0)
            for k in range(P - W, P):
                one_step(k % B)
            stamp(0)
            for k in range(K):
                one_step(k % B)
            stamp(1)
            if layout != 1:
                count(1)
            else:
                self.n = [self.stamps[0] * 0, self.stamps[0] * 0]
        self()
        torch.cuda.synchronize()

    def __call__(self):
        self.graph.replay()

    def inner_s(self):
        t = self.stamps.tolist()
        return (t[1] - t[0]) / self.CLOCK_HZ

    def resets(self):
        return int(self.n[1].item()) - int(self.n[0].item())


def windows(torch, dev, one_step, K, B, env=None):
    """The timed body for exactly K steps: a TimedGraph (events inside the graph around the K steps),
    or -- where the explicit graph API is unavailable -- graphs_for's replays.  Returns (body, keep,
    mode)."""
    if os.environ.get("HG_BENCH_OUTER_WINDOWS") != "1" and env is not None and hasattr(env, "lib"):
        try:
            tg = TimedGraph(torch, dev, one_step, K, B, env)
            return tg, (tg,), (f"one hipGraph per window: {tg.P} pre-roll steps (the last {tg.W} after the first "
                               f"episode count), then the {K} timed steps between two GPU clock stamps")
        except Exception as exc:   # (reported in the mode string)
            torch.cuda.synchronize()
            progress(f"TimedGraph unavailable ({exc}); graph replays")
            err = f" (TimedGraph unavailable: {exc})"
    else:
        err = ""
    rep, keep = graphs_for(torch, dev, one_step, K, B)
    return rep, keep, (f"hipGraphs of {B} steps" + (f" + {K % B} eager launches" if K % B else "") if K >= B
                       else f"{K} eager launches behind a queued {B}-step hipGraph") + err


def graphs_for(torch, dev, one_step, K, B):
    """Exactly K steps: K // B replays of a hipGraph of B steps, then the K mod B remaining steps
    launched eagerly.  A graph launch costs the GPU about 8 us more than the same steps launched
    eagerly behind queued work (scripts/r04_window_probe.py: 20 steps 8.2 us per step as one graph,
    7.85 eager, 7.83 in graphs of 100), so a remainder -- the whole window when K < B -- goes out
    eagerly.  `replay.preroll` is one graph of B steps: the timer queues it before each window, so
    the GPU is busy when the window starts and the host has queued the window's launches by the time
    the GPU reaches them."""
    s = torch.cuda.Stream(device=dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(s):
        for k in range(B):   # warm the capture stream
            one_step(k)
    torch.cuda.current_stream(dev).wait_stream(s)
    torch.cuda.synchronize()
    full = torch.cuda.CUDAGraph()
    with torch.cuda.graph(full):
        for k in range(B):
            one_step(k)

    def replay():
        for _ in range(K // B):
            full.replay()
        for k in range(K % B):
            one_step(k)
    replay.preroll = full.replay
    replay()
    torch.cuda.synchronize()
    return replay, (full,)


class _DryEnv:
    """--dry-run stand-in: buffers only, no kernel (exercises launcher, ranks, gather, timing)."""

    def __init__(self, torch, n, dev):
        self.num_envs, self.specialized = n, False
        self.obs = torch.zeros((n, 17), dtype=torch.float32, device=dev)

    def step_async(self, actions, with_reset_info=True, obs_out=None):
        pass

    def close(self):
        pass


def make_env(args, torch, n, offset, dev):
    if args.dry_run:
        return _DryEnv(torch, n, dev)
    from heligym_amd import HeliVecEnv
    env = HeliVecEnv(n, task=args.task, dt=args.dt, seed=1234, autoreset=True, env_offset=offset,
                     device=dev, reset_mode=args.reset_mode, autoreset_mode=args.autoreset_mode,
                     max_episode_steps=args.max_episode_steps)
    if args.generic_kernel:
        env.set_specialized(False)
    env.reset()
    return env


def action_bank(args, torch, env, n, dev, B):
    bank = torch.empty((B, n, 4), dtype=torch.float32, device=dev)
    if not args.dry_run:
        for k in range(B):
            env.random_actions(bank[k], seed=0x5EED, step=k)
    return bank


def age(args, torch, env, bank, B, dt=None):
    """Step a freshly reset population for --age-seconds of simulated time (untimed), so that its
    episodes are spread over their phases -- crashes, gear contact, resets -- as in a long run.
    Every env starts its first episode together; random-action episodes end after about 10 s
    (SURVEY a27), so without this a short timed window right after reset holds no episode end.  The
    envs that never crash (about 5 %, most of them resting on the ground) reach the 40 s time limit
    together; the default 60 s ages the population past that cohort (scripts/r04_population.py)."""
    if args.dry_run:
        return 0
    steps = int(round(args.age_seconds / (dt or args.dt)))
    t_last = time.time()
    for k in range(steps):
        env.step_async(bank[k % B], with_reset_info=False)
        if (k + 1) % 500 == 0:   # under a profiler each dispatch is slow: a line now and then shows progress
            torch.cuda.synchronize()
            if time.time() - t_last > 20:
                progress(f"ageing: {k + 1} / {steps} steps")
                t_last = time.time()
    torch.cuda.synchronize()
    return steps


def episodes(env, sync=True):
    """Episodes begun so far, summed over the envs (the episode-index counters): the difference
    around a timed region is the number of resets inside it.  sync=False: a device scalar, queued
    on the current stream (read it after a synchronize)."""
    if not hasattr(env, "get_state"):
        return 0
    _, c = env.get_state()
    n = c[:, 2].long().sum()
    return int(n.item()) if sync else n


def gather_loop(torch, dist, env, bank, B, K, rank, world, dev, backend, overlap=True):
    """K steps, each followed by a gather of its observations to rank 0 (dist.gather over RCCL).
    Observations alternate between two buffers so that the gather of step k runs on the
    communicator's stream while step k+1 computes (random actions do not wait for them); step k+2
    waits for gather k before it overwrites that buffer."""
    n = env.num_envs
    bufs = [torch.empty((n, 17), dtype=torch.float32, device=dev) for _ in range(2)]
    on_gpu = backend == "nccl"
    # rank 0's destination rows, double-buffered like the observations (step k+1's gather is queued
    # while a consumer may still read step k's)
    gls = [[torch.empty((n, 17), dtype=torch.float32, device=dev if on_gpu else "cpu") for _ in range(world)]
           if rank == 0 else None for _ in range(2)]

    def body(steps=K):
        works = [None, None]
        for k in range(steps):
            b = k & 1
            if works[b] is not None:
                works[b].wait()
            env.step_async(bank[k % B], with_reset_info=False, obs_out=bufs[b])
            x = bufs[b] if on_gpu else bufs[b].cpu()   # gloo rehearsal: host staging
            works[b] = dist.gather(x, gather_list=gls[b], dst=0, async_op=True)
            if not overlap or not on_gpu:
                works[b].wait()
                works[b] = None
        for w in works:
            if w is not None:
                w.wait()
    return body


def gather_graphs(torch, dist, env, bank, B, K, rank, world, dev):
    """The gather loop captured in hipGraphs (RCCL collectives captured with the steps): each graph
    holds G steps, the observations alternating between two buffers; step k's gather runs on a side
    stream concurrent with step k+1, and step k+2 waits (event) for gather k before it overwrites that
    buffer.  A graph's side stream joins the main stream at its end, so the last gather of a graph
    is not overlapped.  Returns (replay of exactly K steps, what the graphs keep alive)."""
    n = env.num_envs
    bufs = [torch.empty((n, 17), dtype=torch.float32, device=dev) for _ in range(2)]
    gls = [[torch.empty((n, 17), dtype=torch.float32, device=dev) for _ in range(world)] if rank == 0 else None
           for _ in range(2)]
    G = max(2, min(B, K))
    cap = torch.cuda.Stream(device=dev)
    side = torch.cuda.Stream(device=dev)

    def steps(count):
        main = torch.cuda.current_stream(dev)
        done = [None, None]
        for k in range(count):
            b = k & 1
            if done[b] is not None:
                main.wait_event(done[b])
            env.step_async(bank[k % B], with_reset_info=False, obs_out=bufs[b])
            side.wait_stream(main)
            with torch.cuda.stream(side):
                dist.gather(bufs[b], gather_list=gls[b], dst=0)
                done[b] = torch.cuda.Event()
                done[b].record(side)
        main.wait_stream(side)

    cap.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(cap):   # warm-up outside capture (communicator, streams)
        steps(min(G, K))
    torch.cuda.current_stream(dev).wait_stream(cap)
    torch.cuda.synchronize()
    full = torch.cuda.CUDAGraph()
    with torch.cuda.graph(full, stream=cap):
        steps(G)
    rest = None
    if K % G:
        rest = torch.cuda.CUDAGraph()
        with torch.cuda.graph(rest, stream=cap):
            steps(K % G)

    def replay():
        for _ in range(K // G):
            full.replay()
        if rest is not None:
            rest.replay()
    replay()
    torch.cuda.synchronize()
    return replay, (full, rest, bufs, gls, cap, side), G


def airframes(args, torch, timer, N, dev, B, K, R, head_s):
    """Row f4's other airframes at headline speed: the heavier airframe with other rotor speeds and
    the winged one (tests/golden traj_var_* documents), stepped with the generic kernel and then with
    the kernel specialised for their constants at run time (HeliVecEnv.specialize, heligym_amd._rtc),
    against the default airframe's compiled-in kernel (the headline)."""
    import golden_cases as gc
    from heligym_amd import HeliVecEnv
    out = {}
    for name in ("heavy", "wing"):
        doc = gc.load_variant(name)[1]
        env = HeliVecEnv(N, task=args.task, dt=args.dt, seed=1234, autoreset=True, heli_name=doc, device=dev)
        env.reset()
        bank = action_bank(args, torch, env, N, dev, B)
        age(args, torch, env, bank, B)

        def one(k):
            env.step_async(bank[k % B], with_reset_info=False)
        rep, keep, _m = windows(torch, dev, one, K, B, env)
        s_g, _, _, rs_g = timer.run_counted(env, rep, R)
        del keep
        t0 = time.perf_counter()
        spec = env.specialize()
        t_build = time.perf_counter() - t0
        rep, keep, _m = windows(torch, dev, one, K, B, env)
        s_s, _, _, rs_s = timer.run_counted(env, rep, R)
        del keep
        out[name] = {"generic_ms_per_step": s_g / K * 1e3, "specialised_ms_per_step": s_s / K * 1e3,
                     "specialised": spec, "specialise_s": t_build,
                     "specialised_over_default_airframe": (s_s / K) / head_s,
                     "resets_in_window": [rs_g, rs_s]}
        env.close()
    out["note"] = ("specialise_s: hipcc --genco of csrc/step_rtc.hip with the airframe's constants (0 when "
                   "cached); specialised_over_default_airframe: against the headline's compiled-in AW109 kernel")
    return out


def config5(args, torch, dist, timer, env5, bank5, n5, B, K, R, rank, world, dev, backend):
    """BASELINE config 5 on this rank's shard: the gather loop (hipGraphs of steps + RCCL gathers, or
    eager where capture is unavailable) and the plain (graph) steps."""
    K5 = min(K, 500)
    mode5, body = None, None
    if backend == "nccl" and not args.dry_run and os.environ.get("HG_BENCH_CONFIG5_EAGER") != "1":
        try:
            body, _keep5, G5 = gather_graphs(torch, dist, env5, bank5, B, K5, rank, world, dev)
            mode5 = (f"hipGraph: graphs of {G5} steps, each step's dist.gather of obs to rank 0 captured with it "
                     "(side stream, double-buffered)")
        except Exception as exc:   # capture unsupported here: measure the eager loop instead, and say so
            torch.cuda.synchronize()
            body, mode5 = None, f"eager (graph capture of the gather failed: {type(exc).__name__}: {exc})"
    if body is None:
        body = gather_loop(torch, dist, env5, bank5, B, K5, rank, world, dev, backend)
        body(min(args.warmup, K5))
        mode5 = mode5 or "eager, dist.gather of obs to rank 0 every step, double-buffered"
    s_g5, _, _, rs_g5 = timer.run_counted(env5, body, R)
    ranks_g5 = timer.per_rank

    def step5(k):
        env5.step_async(bank5[k % B], with_reset_info=False)
    if args.dry_run:
        def rep5():
            for k in range(K5):
                step5(k)
        mode_n5 = f"{K5} eager launches (dry run)"
    else:
        rep5, _k5, mode_n5 = windows(torch, dev, step5, K5, B, env5)
    s_n5, _, _, rs_n5 = timer.run_counted(env5, rep5, R)
    ranks_n5 = timer.per_rank
    return {"workload": f"HeliHover-v0 x {CONFIG5_TOTAL} envs sharded over {world} ranks ({n5} on rank {rank})",
            "with_gather": {"value": CONFIG5_TOTAL * K5 / s_g5, "unit": "env-steps/s",
                            "ms_per_step": s_g5 / K5 * 1e3,
                            "per_rank_ms_per_step": [x / K5 * 1e3 for x in ranks_g5],
                            "resets_in_window": rs_g5, "mode": mode5},
            "without_gather": {"value": CONFIG5_TOTAL * K5 / s_n5, "unit": "env-steps/s",
                               "ms_per_step": s_n5 / K5 * 1e3,
                               "per_rank_ms_per_step": [x / K5 * 1e3 for x in ranks_n5],
                               "resets_in_window": rs_n5, "mode": mode_n5},
            "gather_bytes_per_step_to_rank0": (world - 1) * n5 * 17 * 4, "steps": K5}


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch(args))
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    backend = None
    # HG_BENCH_FORCE_DIST=1: a process group (RCCL) even for one rank, so that the config-5 gather
    # loop runs on hardware with one GPU (gather to itself) -- a rehearsal of the API usage only
    forced = os.environ.get("HG_BENCH_FORCE_DIST") == "1" and world == 1 and not args.dry_run
    from datetime import timedelta
    if args.config5_only:
        config5_watchdog()
        if os.environ.get("HG_BENCH_CONFIG5_INJECT") == "hang":   # (CPU test hook)
            time.sleep(3600)
        if os.environ.get("HG_BENCH_CONFIG5_INJECT") == "fail" and rank == world - 1:
            raise RuntimeError("injected config-5 failure")
    want5 = (world > 1 or forced) and not args.no_config5 and not args.no_secondary and not args.gather_obs
    c5_child = None
    if want5 and not args.config5_only and rank == 0:
        c5_child = run_config5_child(args, world)   # before this process touches the GPU
    # the other ranks wait for rank 0 in the rendezvous while its config-5 child runs; past that, a
    # collective that does not complete errors out instead of hanging the run
    pg_timeout = timedelta(seconds=120 + (args.config5_timeout + 60 if want5 and not args.config5_only else 0))
    if forced:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(_free_port()))
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
    if args.dry_run:
        dev = torch.device("cpu")
        torch.cuda.synchronize = lambda *a, **k: None   # noqa: E731  (no device in a dry run)
        if world > 1:
            backend = "gloo"
            dist.init_process_group("gloo", timeout=pg_timeout)
    elif world > 1 or forced:
        # HG_BENCH_BACKEND=gloo: rehearsal of the N>1 path with several ranks on one GPU (RCCL
        # refuses two ranks on one device); timings from such a run are not a measurement
        backend = os.environ.get("HG_BENCH_BACKEND", "nccl")
        if backend == "nccl":
            # the device is selected after the rendezvous: while rank 0's config-5 child measures, the
            # ranks waiting here hold no HIP context on the GPUs the child's ranks use (the
            # communicators are created lazily, at the first collective, on the device set here)
            dist.init_process_group("nccl", timeout=pg_timeout)
            torch.cuda.set_device(local)
        else:
            torch.cuda.set_device(local % torch.cuda.device_count())
            dist.init_process_group(backend, timeout=pg_timeout)
        dev = torch.device(f"cuda:{torch.cuda.current_device()}")
    else:
        torch.cuda.set_device(0)
        dev = torch.device("cuda:0")
    dist_on = world > 1 or forced
    seen_world = dist.get_world_size() if dist_on else 1
    if seen_world != world:
        sys.exit(f"bench.py: process group has {seen_world} ranks, expected {world}")
    if args.gather_obs and world < 2:
        sys.exit("bench.py: --gather-obs needs N > 1 ranks")
    if args.dry_run:
        from contextlib import nullcontext
        torch.cuda.Event = _HostEvent
        torch.cuda.current_stream = lambda *a, **k: None   # noqa: E731
        torch.cuda.stream = lambda *a, **k: nullcontext()  # noqa: E731
    timer = Timer(torch, dist, world, dev)
    B = max(1, args.graph_steps)
    K = max(1, args.steps)
    R = max(1, args.repeats)

    if args.config5_only:   # the config-5 child's ranks (run_config5_child)
        from heligym_amd.distributed import shard_bounds
        off5, n5 = shard_bounds(CONFIG5_TOTAL, rank, world)
        env5 = make_env(args, torch, n5, off5, dev)
        bank5 = action_bank(args, torch, env5, n5, dev, B)
        age(args, torch, env5, bank5, B)
        c5 = config5(args, torch, dist, timer, env5, bank5, n5, B, K, R, rank, world, dev, backend)
        if rank == 0:
            print(json.dumps({"config5": c5}), flush=True)
        env5.close()
        dist.destroy_process_group()
        return

    secondary = {}
    head_event_s = None
    if args.gather_obs:
        # headline = BASELINE config 5: CONFIG5_TOTAL envs sharded over the ranks, gather to rank 0
        from heligym_amd.distributed import shard_bounds
        off, N = shard_bounds(CONFIG5_TOTAL, rank, world)
        env = make_env(args, torch, N, off, dev)
        bank = action_bank(args, torch, env, N, dev, B)
        aged = age(args, torch, env, bank, B)
        body = None
        if backend == "nccl" and os.environ.get("HG_BENCH_CONFIG5_EAGER") != "1":
            try:
                body, _keep, G = gather_graphs(torch, dist, env, bank, B, K, rank, world, dev)
                mode = f"hipGraph (graphs of {G} steps with their dist.gather of obs to rank 0 captured, double-buffered)"
            except Exception as exc:
                torch.cuda.synchronize()
                mode = f"eager (graph capture of the gather failed: {type(exc).__name__}: {exc})"
        if body is None:
            body = gather_loop(torch, dist, env, bank, B, K, rank, world, dev, backend)
            body(min(args.warmup, K))
            if backend != "nccl" or os.environ.get("HG_BENCH_CONFIG5_EAGER") == "1":
                mode = "eager (per-step launch + dist.gather to rank 0, double-buffered)"
        sec, secs, wall, resets = timer.run_counted(env, body, R)
        per_rank = timer.per_rank
        total_envs = CONFIG5_TOTAL
    else:
        N = args.envs
        progress(f"headline: {N} envs")
        env = make_env(args, torch, N, rank * N, dev)
        bank = action_bank(args, torch, env, N, dev, B)
        aged = age(args, torch, env, bank, B)

        def one_step(k):
            env.step_async(bank[k % B], with_reset_info=False)

        for k in range(args.warmup):
            one_step(k)
        torch.cuda.synchronize()
        if args.dry_run:
            def replay():
                for k in range(K):
                    one_step(k)
        else:
            replay, _keep, mode = windows(torch, dev, one_step, K, B, env)
        sec, secs, wall, resets = timer.run_counted(env, replay, R)
        per_rank = timer.per_rank
        head_event_s = timer.event_s
        if args.dry_run:
            mode = f"{K} eager launches (dry run)"
        total_envs = N * world

        if not args.no_secondary and not args.dry_run:
            # the same step with the compacted reset info (same-step auto-reset: reset indices and
            # terminal observations compacted in-kernel; each step's kernel zeroes a later step's count)
            if args.reset_mode == "template" and args.autoreset_mode == "same_step":
                progress("step_with_reset_info / step_api_eager")

                def one_step_ri(k):
                    env.step_async(bank[k % B], with_reset_info=True)
                rep_ri, _k2, _m = windows(torch, dev, one_step_ri, K, B, env)
                s_ri, _, _, rs_ri = timer.run_counted(env, rep_ri, R)
                del _k2
                secondary["step_with_reset_info"] = {
                    "value": total_envs * K / s_ri, "unit": "env-steps/s", "ms_per_step": s_ri / K * 1e3,
                    "resets_in_window": rs_ri,
                    "note": "step_async(with_reset_info=True): reset_index + final_obs compaction "
                            "(hg_step_chained: the counts rotate over three slots, each step's kernel zeroing a later one's; "
                            "no zeroing launch), hipGraph"}
                # HeliVecEnv.step() as an RL loop calls it: eager, lazy info
                Ke = 200   # (its own window length: 20 eager launches would carry the HIP events' latency)

                def eager_api():
                    for k in range(Ke):
                        env.step(bank[k % B])
                eager_api()
                s_api, s_api_all, _, rs_api = timer.run_counted(env, eager_api, 5)   # median of 5 windows (host jitter)
                # the same step() calls graph-replayed: what the eager launches cost beyond the
                # step's own work (step() also writes its auto-resets' terminal observations)
                rep_sg, _k4, _m = windows(torch, dev, lambda k: env.step(bank[k % B]), Ke, B, env)
                s_sg, _, _, _ = timer.run_counted(env, rep_sg, 3)
                del _k4
                secondary["step_api_eager"] = {
                    "value": total_envs * Ke / s_api, "unit": "env-steps/s", "ms_per_step": s_api / Ke * 1e3,
                    "graph_replayed_ms_per_step": s_sg / Ke * 1e3,
                    "steps": Ke, "windows_s": s_api_all, "resets_in_window": rs_api,
                    "note": "HeliVecEnv.step() as an RL loop calls it: eager launch of the plain "
                                         "kernel (hg_step_rows: reset envs flagged in the info bytes, their "
                                         "terminal observations at their own rows); its info dict is lazy "
                                         "(fields not read here; the reset info costs one nonzero when read)"}
            if env.specialized and not args.generic_kernel:
                # the generic kernel (model constants loaded, any airframe); bitwise-identical results
                progress("generic_kernel")
                env.set_specialized(False)
                rep_g, _k3, _m = windows(torch, dev, one_step, K, B, env)
                s_g, _, _, rs_g = timer.run_counted(env, rep_g, R)
                del _k3
                env.set_specialized(True)
                secondary["generic_kernel"] = {"kernel": "generic (constants loaded, any airframe)",
                                               "value": total_envs * K / s_g, "unit": "env-steps/s",
                                               "ms_per_step": s_g / K * 1e3, "resets_in_window": rs_g}
            if world == 1 and args.task != "heli" and args.reset_mode == "template" and N <= 262144:
                progress("airframes")
                try:
                    secondary["airframes"] = airframes(args, torch, timer, N, dev, B, K, R, sec / K)
                except Exception as exc:   # (hipcc missing, ...): report, never lose the line
                    secondary["airframes"] = {"error": repr(exc)}
            if args.rollout_steps > 0 and args.reset_mode == "template":
                Rs = args.rollout_steps
                progress("rollout")
                rbank = bank if Rs == B else torch.stack([bank[k % B] for k in range(Rs)])
                rout = env.rollout(rbank)
                nroll = max(1, K // Rs)

                def rollouts():
                    for _ in range(nroll):
                        env.rollout(rbank, out=rout)
                s_r, _, _, rs_r = timer.run_counted(env, rollouts, R)
                secondary["rollout"] = {
                    "api": "hg_rollout", "steps_per_launch": Rs, "steps": nroll * Rs,
                    "value": total_envs * nroll * Rs / s_r, "unit": "env-steps/s",
                    "ms_per_step": s_r / (nroll * Rs) * 1e3, "resets_in_window": rs_r,
                    "bytes_per_env_step": ROLLOUT_BYTES_PER_ENV_STEP + BYTES_STATE_RW / Rs,
                    "note": "open-loop action sequences (planning / data generation); same results as "
                            "hg_step, state read and written once per launch"}

        if world == 1 and not args.no_secondary and not args.dry_run and args.reset_mode == "template":
            # the same workload with exact F8 resets: every auto-reset re-trimmed on the device against
            # the env's last wind (reset_mode="retrim", helicopter.py:208-212)
            Kr = min(K, 500)
            for name, amode in (("retrim", args.autoreset_mode), ("retrim_next_step", "next_step")):
                if name == "retrim_next_step" and args.autoreset_mode == "next_step":
                    continue
                progress(f"{name} ({amode})")
                envr = make_env(argparse.Namespace(**{**vars(args), "reset_mode": "retrim", "autoreset_mode": amode}),
                                torch, N, rank * N, dev)

                def stepr(k):
                    envr.step_async(bank[k % B], with_reset_info=False)
                aged_r = age(args, torch, envr, bank, B)
                for k in range(min(args.warmup, 50)):
                    stepr(k)
                repr_, _kr, _m = windows(torch, dev, stepr, Kr, B, envr)
                s_rt, _, _, rs_rt = timer.run_counted(envr, repr_, 3)
                del _kr
                ov = amode == "next_step" and envr.set_retrim_overlap(True)
                solves, searched = envr.retrim_solve_stats()
                _, ctr_r = envr.get_state()
                trims = int(ctr_r[:, 2].long().sum())
                # a window without a reset would time the plain step, not the re-trim: no value then
                secondary[name] = {
                    "envs": N, "value": N * Kr / s_rt if rs_rt > 0 else None, "unit": "env-steps/s",
                    "ms_per_step": s_rt / Kr * 1e3 if rs_rt > 0 else None, "window_ms_per_step": s_rt / Kr * 1e3,
                    "resets_in_window": rs_rt, "aged_steps": aged_r, "autoreset_mode": amode,
                    "steps": Kr, "retrim_failures": envr.retrim_failures(),
                    "retrim_invalid_jobs": envr.retrim_invalid_jobs(),
                    "trim_solves": {"trims": trims, "newton_solves": solves, "searched": searched,
                                    "solves_per_trim": solves / trims if trims else None,
                                    "note": "over the env's life (ageing + windows): Newton solves tried with the "
                                            "host trim's pivot order, and those the residual test sent to the "
                                            "pivot search (csrc/gj_mfma.h)"},
                    "note": "reset_mode='retrim': each auto-reset re-trimmed on the device (Newton trim against the "
                            "env's last wind, the reference's reset from episode 2 on), hipGraph"
                            + ("; next-step auto-reset (make_vec's configuration): the episodes a step ends are "
                               "trimmed in the first blocks of the next step's launch (step_ov_kernel)"
                               if ov else "")}
                envr.close()

        if world == 1 and not args.no_secondary and not args.dry_run and args.envs < OUT_OF_CACHE_ENVS:
            # the same step past the 256 MB Infinity Cache (1.32 GB moved per launch): HBM bytes, not
            # fabric bytes, with its own committed PMC summary
            Nx = OUT_OF_CACHE_ENVS
            progress(f"out_of_cache: {Nx} envs")
            envx = make_env(args, torch, Nx, 0, dev)
            bankx = action_bank(args, torch, envx, Nx, dev, B)
            Kx = min(K, 200)

            def stepx(k):
                envx.step_async(bankx[k % B], with_reset_info=False)
            aged_x = age(args, torch, envx, bankx, B)
            for k in range(min(args.warmup, 20)):
                stepx(k)
            repx, _kx, _m = windows(torch, dev, stepx, Kx, B, envx)
            s_x, _, _, rs_x = timer.run_counted(envx, repx, 3)
            del _kx
            ach = Nx * BYTES_PER_ENV_STEP / (s_x / Kx) / 1e9
            ceil = pattern_ceiling()
            secondary["out_of_cache"] = {
                "envs": Nx, "value": Nx * Kx / s_x, "unit": "env-steps/s", "ms_per_step": s_x / Kx * 1e3,
                "steps": Kx, "achieved_GBs": ach, "frac": ach / HBM_PEAK_GBS,
                # the step's own memory pattern with the arithmetic taken out (scripts/ubench/mover.hip):
                # the period this access pattern reaches on the chip, and the step's fraction of it
                "pattern_ceiling": ceil and {"ms_per_step": ceil["period_us_event_timed"] * 1e-3,
                                             "GBs_315": ceil["ceiling_GBs_315"],
                                             "frac_of_ceiling": ceil["period_us_event_timed"] * 1e-3 / (s_x / Kx * 1e3),
                                             "source": "profiles/r05_mover_4m_pmc_summary.json"},
                "resets_in_window": rs_x, "aged_steps": aged_x,
                "traffic": (pmc_traffic(Nx, args.dt, args.task) or (None,))[0],
                "traffic_source": (pmc_traffic(Nx, args.dt, args.task) or (None, None))[1],
                "note": "working set 1.32 GB per launch, past the 256 MB MALL: the traffic is HBM bytes"}
            envx.close()
            del bankx

        if c5_child is not None:   # BASELINE config 5, measured by rank 0's child run before the headline
            secondary["config5"] = c5_child

    if rank != 0:
        if dist_on:
            dist.destroy_process_group()
        return

    value = total_envs * K / sec
    # average step-kernel duration: the timed window holds exactly K step-kernel launches back to
    # back on the env's stream (graph mode) -- what rocprofv3's kernel-trace average measures
    kern_s = sec / K
    achieved = (total_envs / world) * BYTES_PER_ENV_STEP / kern_s / 1e9
    task_name = {"hover": "HeliHover-v0", "forward_flight": "HeliForwardFlight-v0", "heli": "Heli"}[args.task]
    out = {
        "metric": "env-steps/sec at 65536 envs, 1/2/4/8 MI355X; max-abs step() err vs ref",
        "value": None if args.dry_run else value,
        "unit": "env-steps/s",
        "n_gpus": world,
        "steps": K,
        "warmup": args.warmup,
        "ms_per_step": sec / K * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "fp32",
        "data": "synthetic: U(-1,1) Philox actions (HBM-resident bank of %d steps), Philox turbulence" % B,
        "config": {"workload": f"{task_name} x {total_envs // world} envs/GPU, Dryden turbulence level 1, "
                               f"dt={args.dt}, auto-reset"
                               f"{' (re-trim per reset, F8)' if args.reset_mode == 'retrim' else ''}"
                               f"{' in the next step' if args.autoreset_mode == 'next_step' else ''}"
                               f"{f', TimeLimit {args.max_episode_steps}' if args.max_episode_steps else ''}, {mode}"
                               + (", BASELINE config 5" if args.gather_obs else ""),
                   "envs_per_gpu": total_envs // world, "dt": args.dt, "task": args.task,
                   "reset_mode": args.reset_mode, "autoreset_mode": args.autoreset_mode,
                   "max_episode_steps": args.max_episode_steps,
                   "kernel": "specialised (default airframe constants compiled in)" if env.specialized else "generic",
                   "parallelism": f"env-shard x{world}", "world_size_seen": seen_world,
                   "backend": backend or "none (1 rank)"},
        "timing": {"repeats": R, "window_s": secs, "median_window_s": sec, "wall_median_s": wall,
                   "window_clock": ("GPU clock stamps (hg_clock_stamp, 100 MHz) around exactly the K step launches inside "
                                    "each window's hipGraph, after a pre-roll of the same graph" if head_event_s is not None
                                    else "HIP events around the window's launches"),
                   "event_window_s": head_event_s,
                   "event_note": "HIP events around the whole window graph (pre-roll, episode counts, K steps)",
                   "wall_note": "host time from submitting the timed body to its completion",
                   "steps_per_window": K, "aged_steps": aged,
                   "aged_note": f"each env population stepped {args.age_seconds:g} simulated s (untimed) after reset "
                                "before capture: windows see steady-state episode phases",
                   "resets_in_window": resets,
                   "resets_note": ("episodes begun in the K timed steps and the 8 steps before them"
                                   if head_event_s is not None else "episodes begun in the K timed steps"),
                   "per_rank_ms_per_step": [x / K * 1e3 for x in per_rank]},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": None,
                     "kernel": (f"step_help_kernel<{args.task.upper()}>"   # (heligym_amd.hip launch_step: a helper
                                # wave per tile up to half a wave per SIMD, HG_HELPER_DIV)
                                if torch.cuda.is_available() and args.envs <= 2 * 64 * torch.cuda.get_device_properties(0).multi_processor_count
                                else f"step_kernel<{args.task.upper()}>"),
                     "kernel_avg_us": kern_s * 1e6,
                     "kernel_avg_source": "the median timed window (GPU clock stamps around its K launches) / K",
                     "bytes_per_env_step": BYTES_PER_ENV_STEP,
                     "impl_bytes_per_env_step": IMPL_BYTES_PER_ENV_STEP,
                     "algorithmic_bytes_per_launch": (total_envs // world) * BYTES_PER_ENV_STEP},
    }
    head_mode = (args.reset_mode, args.autoreset_mode)   # the reset path whose PMC summary applies
    if args.dry_run:
        out["dry_run"] = "plumbing check only: no kernel ran, nothing was measured"
        out["roofline"].update(achieved=None, frac=None)
    else:
        props = torch.cuda.get_device_properties(dev)
        simds = 4 * props.multi_processor_count
        ghz, ghz_src = shader_clock_ghz(args.dt, args.task, getattr(props, "clock_rate", 2400000) / 1e6)
        vi = valu_issue(total_envs // world, args.dt, args.task, kern_s, simds, ghz, mode=head_mode)
        if vi is not None:
            out["roofline"].update(vi, clock_ghz=ghz, clock_source=ghz_src)
        if "out_of_cache" in secondary:
            oc = secondary["out_of_cache"]
            vx = valu_issue(oc["envs"], args.dt, args.task, oc["ms_per_step"] * 1e-3, simds, ghz)
            if vx is not None:
                oc.update(vx)
    if args.gather_obs:
        out["roofline"]["kernel_avg_source"] = "timed window / steps (eager with gathers: an upper bound)"
    out.update(secondary)
    tr = None if args.dry_run else pmc_traffic(total_envs // world, args.dt, args.task, mode=head_mode)
    if tr is not None:
        out["roofline"]["traffic"] = tr[0]
        out["roofline"]["traffic_source"] = tr[1] + " (HBM bytes per launch, PMC)"
    if not args.no_parity and not args.dry_run:
        try:
            out["max_abs_step_err"] = parity_error(args.dt, args.task)
        except Exception as e:   # report, never hide
            out["max_abs_step_err"] = {"error": repr(e)}
    if world == 1 and not args.no_cpu_baseline and not args.dry_run:
        out["cpu_baseline"] = cpu_baseline(args.dt, args.task, args.cpu_seconds)
    print(json.dumps(out), flush=True)
    env.close()
    if dist_on:
        dist.destroy_process_group()


class _HostEvent:
    """--dry-run: torch.cuda.Event stand-in on the host clock."""

    def __init__(self, enable_timing=True):
        self.t = None

    def record(self, stream=None):
        self.t = time.perf_counter()

    def elapsed_time(self, other):
        return (other.t - self.t) * 1e3


if __name__ == "__main__":
    main()
