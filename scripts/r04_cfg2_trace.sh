# Kernel trace of the config-2 bench (4 096 envs, the small-batch helper kernel)
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/cfg2_prof -o bench -- python3 bench.py --envs 4096 --no-cpu-baseline --no-parity --no-secondary > gpurun_out/cfg2_prof.log 2>&1 || { echo "rocprof failed"; tail -5 gpurun_out/cfg2_prof.log; exit 6; }
tail -1 gpurun_out/cfg2_prof.log > gpurun_out/cfg2_prof_line.json
find gpurun_out/cfg2_prof -name "*.csv" ! -name "*kernel_stats.csv" -delete
find gpurun_out/cfg2_prof -name "*kernel_stats.csv" -exec head -5 {} \;
