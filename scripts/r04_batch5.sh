# Round-4: the bench line at the driver's short window and at the default 1 000 steps (TimedGraph
# windows, 60 s ageing), and the kernel trace of the headline command.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
run() {  # tag, args...
  local tag=$1; shift
  timeout -k 10 500 python bench.py "$@" > gpurun_out/b_$tag.log 2>&1 || { echo "bench $tag failed"; grep -v "^frame" gpurun_out/b_$tag.log | tail -6; exit 4; }
  tail -1 gpurun_out/b_$tag.log > gpurun_out/b_$tag.json; python scripts/bench_brief.py gpurun_out/b_$tag.json
}
run k20 --steps 20 --warmup 5
run def
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof5 -o bench -- python3 bench.py --no-cpu-baseline --no-parity --no-secondary > gpurun_out/prof5.log 2>&1 || { echo "rocprof failed"; tail -5 gpurun_out/prof5.log; exit 5; }
tail -1 gpurun_out/prof5.log | cut -c1-200
find gpurun_out/prof5 -name "*kernel_stats.csv" | head -2
