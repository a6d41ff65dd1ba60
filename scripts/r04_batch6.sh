# Round-4: TimedGraph pre-roll length at K = 20 (clock ramp?), headline only.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for P in 100 1000 4000; do
  HG_TG_PREROLL=$P timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-secondary --no-cpu-baseline --no-parity > gpurun_out/b_p$P.log 2>&1 || { echo "P $P failed"; tail -4 gpurun_out/b_p$P.log; exit 4; }
  tail -1 gpurun_out/b_p$P.log > gpurun_out/b_p$P.json; echo -n "preroll $P: "; python scripts/bench_brief.py gpurun_out/b_p$P.json
done
HG_TG_PREROLL=1000 timeout -k 10 300 python bench.py --steps 1000 --no-secondary --no-cpu-baseline --no-parity > gpurun_out/b_p1k.log 2>&1 && tail -1 gpurun_out/b_p1k.log > gpurun_out/b_p1k.json && python scripts/bench_brief.py gpurun_out/b_p1k.json
python - <<'PY'
import json
for t in ("p100", "p1000", "p4000", "p1k"):
    d = json.load(open(f"gpurun_out/b_{t}.json"))
    print(t, [round(x / d["steps"] * 1e6, 3) for x in d["timing"]["window_s"]], "event", d["timing"].get("event_window_s"))
PY
