"""bench.py's launch and multi-rank plumbing on CPU (gloo, --dry-run: no kernel runs, value null):
`--gpus N` without a launcher starts N ranks itself, the world size is checked, the timed windows
are max-reduced over ranks, rank 0 prints one JSON line, and N > 1 adds BASELINE config 5 (obs
gathered to rank 0).  The GPU measurement itself is bench.py on the MI355X box."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run(*args, env=None):
    e = dict(os.environ)
    e.pop("WORLD_SIZE", None)
    e.update(env or {})
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--dry-run", "--steps", "12",
                        "--warmup", "2", "--repeats", "2", *args], capture_output=True, text=True, env=e,
                       timeout=300, cwd=ROOT)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    return p.returncode, lines, p.stderr


def test_gpus_2_spawns_two_ranks_and_reports_config5():
    rc, lines, err = run("--gpus", "2")
    assert rc == 0, err[-2000:]
    assert len(lines) == 1   # rank 0 only
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["world_size_seen"] == 2
    assert d["value"] is None and "dry_run" in d
    assert d["steps"] == 12 and d["timing"]["repeats"] == 2 and len(d["timing"]["window_s"]) == 2
    assert d["scaling"] == "weak" and d["config"]["parallelism"] == "env-shard x2"
    c5 = d["config5"]
    assert "1048576" in c5["workload"] and "with_gather" in c5 and "without_gather" in c5
    assert c5["gather_bytes_per_step_to_rank0"] == 524288 * 17 * 4


def test_gpus_8_dry_run():
    """The driver's scaling run at N = 8: eight ranks, config 5 sharded 131 072 envs per rank (the
    graph-captured gather needs RCCL; on gloo the eager loop stands in and says so)."""
    rc, lines, err = run("--gpus", "8")
    assert rc == 0, err[-2000:]
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert d["n_gpus"] == 8 and d["config"]["world_size_seen"] == 8
    assert d["config"]["parallelism"] == "env-shard x8"
    c5 = d["config5"]
    assert "131072 on rank 0" in c5["workload"]
    assert c5["gather_bytes_per_step_to_rank0"] == 7 * 131072 * 17 * 4
    assert c5["with_gather"]["mode"].startswith("eager")


def test_gather_obs_headline_is_config5():
    rc, lines, err = run("--gpus", "2", "--gather-obs")
    assert rc == 0, err[-2000:]
    d = json.loads(lines[0])
    assert "BASELINE config 5" in d["config"]["workload"] and d["config"]["envs_per_gpu"] == 524288


def test_config5_failure_keeps_the_headline():
    """A config-5 rank that raises (e.g. an RCCL error in its first gather): the config-5 child run
    fails, the headline line still prints, with config5.error and the child's stderr tail."""
    rc, lines, err = run("--gpus", "2", env={"HG_BENCH_CONFIG5_INJECT": "fail"})
    assert rc == 0, err[-2000:]
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and "window_s" in d["timing"]
    assert "failed" in d["config5"]["error"] and any("injected config-5 failure" in ln for ln in d["config5"]["stderr"]["raised"])


def test_config5_hang_keeps_the_headline():
    """A config-5 child that hangs (every rank stuck, e.g. in a captured multi-rank gather): its ranks'
    watchdog ends them at the limit, and with the watchdog off the parent kills the child run at the
    limit; either way the headline line prints with config5.error, well inside the driver's limit."""
    import time
    for extra, words in (({}, ("failed", "killed")), ({"HG_BENCH_CONFIG5_NO_WATCHDOG": "1"}, ("killed",))):
        t0 = time.time()
        rc, lines, err = run("--gpus", "2", "--config5-timeout", "25",
                             env={"HG_BENCH_CONFIG5_INJECT": "hang", **extra})
        assert rc == 0, err[-2000:]
        assert len(lines) == 1
        d = json.loads(lines[0])
        assert any(w in d["config5"]["error"] for w in words), d["config5"]
        assert "window_s" in d["timing"]
        assert time.time() - t0 < 150


def test_world_size_mismatch_fails():
    rc, lines, err = run("--gpus", "2", env={"WORLD_SIZE": "3"})
    assert rc != 0 and not lines and "WORLD_SIZE=3" in err


def test_gather_obs_needs_ranks():
    rc, lines, err = run("--gather-obs")
    assert rc != 0 and not lines


def test_pmc_summary_is_keyed_on_the_reset_path(tmp_path, monkeypatch):
    """pmc_summary() only returns a summary of the same reset path: a re-trim line (retrim_kernel or
    step_ov_kernel profiles) never carries the template step kernel's counters, nor the other way round
    (the sweep's re-trim lines showed the template kernel's VALU and traffic)."""
    sys.path.insert(0, ROOT)
    import bench
    prof = tmp_path / "profiles"
    prof.mkdir()
    base = {"envs": 65536, "dt": 0.01, "task": "hover", "hbm_bytes_per_launch": 1.0}
    for tag, args in (("a1", ""), ("a2", "--reset-mode retrim --autoreset-mode same_step"),
                      ("a3", "--reset-mode retrim --autoreset-mode next_step")):
        (prof / f"{tag}_pmc_summary.json").write_text(json.dumps({**base, "tag": tag, "bench_args": args}))
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    got = lambda mode: bench.pmc_summary(65536, 0.01, "hover", mode=mode)[0]["tag"]
    assert got(("template", "same_step")) == "a1"
    assert got(("template", "next_step")) == "a1"   # (the auto-reset mode only matters with re-trim)
    assert got(("retrim", "same_step")) == "a2"
    assert got(("retrim", "next_step")) == "a3"
    assert bench.pmc_summary(65536, 0.01, "hover", mode=("retrim", "same_step"), tags=["a1"]) is None
