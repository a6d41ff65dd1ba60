# BASELINE.json configs on one GPU (each its own time limit; stop on the first crash)
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
out=gpurun_out/sweep.jsonl; : > $out
run() { timeout -k 10 240 python bench.py --no-cpu-baseline --no-secondary --repeats 3 "$@" >> $out 2> gpurun_out/sweep_err.log || { echo "FAILED: $*"; tail -5 gpurun_out/sweep_err.log; exit 3; }; }
run --envs 4096 --dt 0.01
run --envs 65536 --dt 0.01
run --envs 65536 --dt 0.02
run --envs 262144 --dt 0.01 --task forward_flight
run --envs 1048576 --dt 0.01 --steps 500
run --envs 4194304 --dt 0.01 --steps 200 --no-parity
run --envs 65536 --dt 0.01 --reset-mode retrim --steps 500 --no-parity
run --envs 65536 --dt 0.01 --reset-mode retrim --autoreset-mode next_step --steps 500 --no-parity
run --envs 262144 --dt 0.01 --task forward_flight --reset-mode retrim --steps 300 --no-parity
python - <<'PY'
import json
for l in open("gpurun_out/sweep.jsonl"):
    d = json.loads(l); r = d["roofline"]
    print(f'{d["config"]["workload"][:60]:60s} {d["value"]:.3e} steps/s  {d["ms_per_step"]*1e3:8.1f} us/step  kern {r["kernel_avg_us"]:8.1f} us  {r["achieved"]:7.0f} GB/s  frac {r["frac"]:.3f}')
PY
