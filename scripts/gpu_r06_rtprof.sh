#!/bin/bash
# Round 6: kernel-trace duration distributions of the re-trim paths (next-step: step_ov_kernel; same-step:
# step kernel + retrim_kernel) at 65 536 aged envs, and the bench's re-trim lines with solve statistics.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
D=gpurun_out/rtprof
mkdir -p $D
for mode in next_step same_step; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $D/$mode -o run -- python3 bench.py --reset-mode retrim \
      --autoreset-mode $mode --steps 500 --repeats 2 --no-secondary --no-cpu-baseline --no-parity > $D/$mode.json 2> $D/$mode.log || exit 3
  f=$(find $D/$mode -name "*kernel_trace.csv" | head -1)
  python3 scripts/kernel_trace_dist.py $f > $D/${mode}_dist.txt
  find $D/$mode -name "*.csv" -delete
  cat $D/${mode}_dist.txt
done
