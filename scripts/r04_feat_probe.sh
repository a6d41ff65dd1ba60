# Step-kernel cost by feature set (aged populations, kernel trace): plain, FEAT with a TimeLimit only,
# and reset_mode "retrim" (FEAT + wind records + the re-trim kernel).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # tag, bench args
  rm -rf gpurun_out/prof_$1
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$1 -o p -- python3 bench.py --no-secondary --steps 300 --no-cpu-baseline --no-parity $2 > gpurun_out/feat_$1.log 2>&1 || { echo "$1 failed"; tail -3 gpurun_out/feat_$1.log; exit 3; }
  python3 scripts/trace_brief.py gpurun_out/prof_$1 "$1: $(grep "^{" gpurun_out/feat_$1.log | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"]*1e3,3), "us/step resets/window", d["timing"]["resets_in_window"])')"
}
run plain ""
run tlimit "--max-episode-steps 1000000000"
run retrim "--reset-mode retrim"
run retrim_next "--reset-mode retrim --autoreset-mode next_step --max-episode-steps 5000"
