#!/bin/bash
# Round 6 end, with the block-inverse solve: pytest -m gpu, smoke, the default bench line, and the
# re-trim kernels' trace + PMC summaries (r06b_rt_same: retrim_kernel, r06b_rt_next: step_ov_kernel).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/gpu_r06_final.sh || exit 3
TAG=r06b_rt_same KERNEL_RE=retrim_kernel BENCH_ARGS="--reset-mode retrim --autoreset-mode same_step" bash scripts/profile_round.sh || exit 4
TAG=r06b_rt_next KERNEL_RE=step_ov_kernel BENCH_ARGS="--reset-mode retrim --autoreset-mode next_step" bash scripts/profile_round.sh || exit 5
