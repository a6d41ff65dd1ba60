#!/usr/bin/env python3
"""Throughput of the vectorised heli-gym step on MI355X (BASELINE.json metric).

One "step" = one hg_step launch advancing every env of every rank by one env-step (wind RK,
helicopter RK4, reward, flags, auto-reset) with actions read from HBM.  Workload (BASELINE.json
configs[2]): 65 536 HeliHover-v0 envs per GPU, Dryden turbulence on (level 1), dt = 0.01 s, fp32,
U(-1,1) random actions (a Philox-generated bank resident in HBM before timing), auto-reset on.

    python bench.py [--gpus N --steps K --warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...      (one process per GPU, RCCL)

Prints ONE JSON line on rank 0.  Envs shard with no data-path collective (weak scaling); the
optional --gather-obs adds an RCCL all-gather of the observations every step (BASELINE config 5).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for p in (ROOT, os.path.join(ROOT, "heli-gym_amd"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)

# Algorithmic HBM bytes per env-step (DESIGN.md "Roofline"): reads state 27x4 + counters 3x4 +
# action 16 = 136 B; writes state 108 + counters 12 + obs 68 + reward 4 + terminated/truncated/info 3
# = 195 B.
BYTES_PER_ENV_STEP = 136 + 195
# hg_rollout: per step action 16 + obs 68 + reward 4 + flags 3; state + counters (240 B) once per launch
ROLLOUT_BYTES_PER_ENV_STEP = 16 + 68 + 4 + 3
BYTES_STATE_RW = 2 * (108 + 12)
HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md (spec; 6.3 TB/s measured copy)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--warmup", type=int, default=200)
    ap.add_argument("--envs", type=int, default=65536, help="envs per GPU")
    ap.add_argument("--dt", type=float, default=0.01)
    ap.add_argument("--task", default="hover", choices=["hover", "forward_flight", "heli"])
    ap.add_argument("--rollout-steps", type=int, default=100,
                    help="also time hg_rollout (this many steps per launch, same action bank); 0 = off")
    ap.add_argument("--reset-mode", default="template", choices=["template", "retrim"],
                    help="auto-reset state: mean-wind trim template (default) or per-reset device re-trim (F8)")
    ap.add_argument("--graph-steps", type=int, default=100, help="steps captured per hipGraph")
    ap.add_argument("--gather-obs", action="store_true", help="RCCL all-gather of obs every step")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline sample budget")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-parity", action="store_true")
    ap.add_argument("--generic-kernel", action="store_true",
                    help="step with the generic kernel instead of the default airframe's constant-specialised one")
    return ap.parse_args()


def pmc_traffic(envs, dt, task):
    """HBM bytes per step-kernel launch from the newest committed PMC summary for this workload
    (profiles/<tag>_pmc_summary.json, written by scripts/summarize_prof.py from rocprofv3 --pmc
    FETCH_SIZE / WRITE_SIZE passes).  None if this workload was not profiled."""
    import glob
    best = None
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc_summary.json"))):
        try:
            d = json.load(open(f))
        except Exception:
            continue
        if d.get("envs") == envs and abs(d.get("dt", -1) - dt) < 1e-12 and task == "hover" \
                and "hbm_bytes_per_launch" in d:
            best = (d["hbm_bytes_per_launch"], os.path.relpath(f, ROOT))
    return best


def cpu_baseline(dt, task, seconds):
    """Oracle (C restatement) on a bounded sample of the same workload: one host core, then the
    box's CPU share (OMP_NUM_THREADS threads, each stepping its own envs; ctypes releases the GIL)."""
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
    threads = max(1, int(os.environ.get("OMP_NUM_THREADS", "16")))
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
            "single_core_value": single,
            "sample": f"oracle/heli_oracle.c (dt={dt}, U(-1,1) actions, turbulence on, auto-reset): "
                      f"{threads} threads x 16 envs x {per} steps in {elm:.1f} s; single core 64 envs x "
                      f"{steps} steps in {el:.1f} s"}


def parity_error(dt, task):
    """max-abs step() error vs the reference's recorded steps (tests/golden) at this dt."""
    import numpy as np
    import torch
    import golden_cases as gc
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
    e_obs = gc.step_errors(obs, b["obs"], gc.OBS_ANGLE_COLS)
    e_st = gc.step_errors(st[:, :18], b["heli"], gc.HELI_ANGLE_COLS)
    tol = lambda r: 2e-4 + 2e-5 * np.abs(r)  # noqa: E731
    flags_ok = bool(np.all(term == b["terminated"]) and np.all(trunc == b["truncated"]))
    env.close()
    # landing-gear contact (ground altitude < 10 ft): the stiff spring turns fp32 input rounding into
    # a visible force difference, so contact steps are reported on their own, as the parity test does
    contact = b["obs"][:, 16] < gc.CONTACT_GR_ALT
    r_obs, r_st = (e_obs / tol(b["obs"])).max(axis=1), (e_st / tol(b["heli"])).max(axis=1)
    worst = np.maximum(r_obs, r_st)
    return {"cases": int(len(b["obs"])), "obs_max_abs": float(e_obs.max()), "state_max_abs": float(e_st.max()),
            "reward_max_abs": float(np.abs(rew - b["reward"]).max()),
            "max_err_over_tol": float(worst[~contact].max()),
            "contact_cases": int(contact.sum()),
            "contact_max_err_over_tol": float(worst[contact].max()) if contact.any() else None,
            "flags_identical": flags_ok,
            "tolerance": "|d| <= 2e-4 + 2e-5|x_ref| (SURVEY 8a-i); gear-contact steps (ground altitude "
                         "< 10 ft) reported separately, tested at 4x"}


def main():
    args = parse()
    import torch
    import torch.distributed as dist
    from heligym_amd import HeliVecEnv

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        # HG_BENCH_BACKEND=gloo: rehearsal of the N>1 path with several ranks on one GPU (RCCL
        # refuses two ranks on one device); timings from such a run are not a measurement
        backend = os.environ.get("HG_BENCH_BACKEND", "nccl")
        if backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
        else:
            torch.cuda.set_device(local % torch.cuda.device_count())
            dist.init_process_group(backend)
    else:
        torch.cuda.set_device(0)
    dev = torch.device(f"cuda:{torch.cuda.current_device()}")
    N = args.envs
    env = HeliVecEnv(N, task=args.task, dt=args.dt, seed=1234, autoreset=True, env_offset=rank * N,
                     device=dev, reset_mode=args.reset_mode)
    if args.generic_kernel:
        env.set_specialized(False)
    env.reset()

    B = max(1, args.graph_steps)
    bank = torch.empty((B, N, 4), dtype=torch.float32, device=dev)
    for k in range(B):
        env.random_actions(bank[k], seed=0x5EED, step=k)
    gathered = None
    if args.gather_obs and world > 1:
        gathered = torch.empty((world * N, 17), dtype=torch.float32, device=dev)

    def one_step(k):
        env.step_async(bank[k % B], with_reset_info=False)
        if gathered is not None:
            dist.all_gather_into_tensor(gathered, env.obs)

    # eager warmup, then capture B steps into a hipGraph (launch-bound inner loop)
    for k in range(args.warmup):
        one_step(k)
    torch.cuda.synchronize()
    graph = None
    if gathered is None:
        s = torch.cuda.Stream(device=dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(s):
            for k in range(B):   # warm the capture stream
                one_step(k)
        torch.cuda.current_stream(dev).wait_stream(s)
        torch.cuda.synchronize()
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            for k in range(B):
                one_step(k)
        graph.replay()
        torch.cuda.synchronize()

    reps = max(1, args.steps // B) if graph is not None else args.steps
    K = reps * B if graph is not None else args.steps
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record()
    if graph is not None:
        for _ in range(reps):
            graph.replay()
    else:
        for k in range(K):
            one_step(k)
    ev1.record()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    wall = time.perf_counter() - t0
    elapsed = ev0.elapsed_time(ev1) * 1e-3
    el_t = torch.tensor([max(elapsed, 0.0), wall], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(el_t, op=dist.ReduceOp.MAX)
    elapsed = float(el_t[0])

    # Secondary figure (not `value`): the same step with the generic kernel (model constants loaded
    # from the device copy, as for any non-default airframe); bitwise-identical results.
    generic = None
    if env.specialized and gathered is None and not args.generic_kernel:
        env.set_specialized(False)
        gg = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gg):
            for k in range(B):
                one_step(k)
        gg.replay()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        g0, g1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        g0.record()
        for _ in range(reps):
            gg.replay()
        g1.record()
        torch.cuda.synchronize()
        gt = torch.tensor([g0.elapsed_time(g1) * 1e-3], dtype=torch.float64, device=dev)
        if world > 1:
            dist.all_reduce(gt, op=dist.ReduceOp.MAX)
        generic = {"kernel": "generic (constants loaded, any airframe)", "value": N * world * K / float(gt[0]),
                   "unit": "env-steps/s", "ms_per_step": float(gt[0]) / K * 1e3}
        env.set_specialized(True)
        del gg

    # Secondary figure (not `value`): the same workload as open-loop rollouts, hg_rollout over the
    # same action bank, `rollout_steps` steps per launch with the env state kept in registers.
    roll = None
    if args.rollout_steps > 0 and gathered is None and args.reset_mode == "template":
        R = args.rollout_steps
        rbank = bank if R == B else torch.stack([bank[k % B] for k in range(R)])
        rout = env.rollout(rbank)
        torch.cuda.synchronize()
        nroll = max(1, K // R)
        if world > 1:
            dist.barrier()
        r0, r1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        r0.record()
        for _ in range(nroll):
            env.rollout(rbank, out=rout)
        r1.record()
        torch.cuda.synchronize()
        rt = torch.tensor([r0.elapsed_time(r1) * 1e-3], dtype=torch.float64, device=dev)
        if world > 1:
            dist.all_reduce(rt, op=dist.ReduceOp.MAX)
        rsec = float(rt[0])
        roll = {"api": "hg_rollout", "steps_per_launch": R, "steps": nroll * R,
                "value": N * world * nroll * R / rsec, "unit": "env-steps/s",
                "ms_per_step": rsec / (nroll * R) * 1e3,
                "bytes_per_env_step": ROLLOUT_BYTES_PER_ENV_STEP + BYTES_STATE_RW / R,
                "note": "open-loop action sequences (planning / data generation); same results as "
                        "hg_step, state read and written once per launch"}

    # Average step-kernel duration = HIP-event time of the timed region / launches: in graph mode
    # the region holds exactly K step-kernel launches back to back on the env's stream (no other
    # work), which is what rocprofv3's kernel-trace average measures (profiles/*_kernel_stats.csv).
    kern_s = elapsed / K

    if rank != 0:
        if world > 1:
            dist.destroy_process_group()
        return
    total_steps = N * world * K
    value = total_steps / elapsed
    achieved = N * BYTES_PER_ENV_STEP / kern_s / 1e9
    out = {
        "metric": "env-steps/sec at 65536 envs, 1/2/4/8 MI355X; max-abs step() err vs ref",
        "value": value,
        "unit": "env-steps/s",
        "n_gpus": world,
        "steps": K,
        "warmup": args.warmup,
        "ms_per_step": elapsed / K * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "fp32",
        "data": "synthetic: U(-1,1) Philox actions (HBM-resident bank of %d steps), Philox turbulence" % B,
        "config": {"workload": f"{'HeliHover-v0' if args.task == 'hover' else args.task} x {N} envs/GPU, "
                               f"Dryden turbulence level 1, dt={args.dt}, auto-reset"
                               f"{' (re-trim per reset, F8)' if args.reset_mode == 'retrim' else ''}, "
                               f"{'hipGraph of %d steps' % B if graph is not None else 'eager'}"
                               + (", RCCL obs all-gather every step" if gathered is not None else ""),
                   "envs_per_gpu": N, "dt": args.dt, "task": args.task, "reset_mode": args.reset_mode,
                   "kernel": "specialised (default airframe constants compiled in)" if env.specialized else "generic",
                   "parallelism": f"env-shard x{world}"},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": None,
                     "kernel": f"step_kernel<{args.task.upper()}>", "kernel_avg_us": kern_s * 1e6,
                     "kernel_avg_source": "HIP events over the timed region / launches" if graph is not None
                     else "HIP events over the timed region / launches (eager: includes launch gaps)",
                     "bytes_per_env_step": BYTES_PER_ENV_STEP,
                     "algorithmic_bytes_per_launch": N * BYTES_PER_ENV_STEP},
        "wall_s": float(el_t[1]),
    }
    if generic is not None:
        out["generic_kernel"] = generic
    if roll is not None:
        out["rollout"] = roll
    tr = pmc_traffic(N, args.dt, args.task)
    if tr is not None:
        out["roofline"]["traffic"] = tr[0]
        out["roofline"]["traffic_source"] = tr[1] + " (bytes per launch)"
    if not args.no_parity:
        try:
            out["max_abs_step_err"] = parity_error(args.dt, args.task)
        except Exception as e:   # report, never hide
            out["max_abs_step_err"] = {"error": repr(e)}
    if world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(args.dt, args.task, args.cpu_seconds)
    print(json.dumps(out))
    env.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
