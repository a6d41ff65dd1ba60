#!/bin/bash
# Round 6 end, part 2: the headline's kernel-trace + PMC summary (profile_round.sh TAG=r06f), a
# rocprofv3 kernel trace of the default bench command, and the BASELINE config sweep.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=r06f bash scripts/profile_round.sh || exit 3
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06_final_prof -o bench -- python3 bench.py --no-cpu-baseline --no-parity > gpurun_out/r06_final_prof.log 2>&1 || { echo "rocprof failed"; tail -5 gpurun_out/r06_final_prof.log; exit 4; }
find gpurun_out/r06_final_prof -name "*.csv" ! -name "*kernel_stats.csv" -delete
bash scripts/bench_sweep.sh
