#!/bin/bash
# Round 6: rocprofv3 kernel-trace + PMC summaries of the re-trim kernels at 65 536 aged envs
# (retrim_kernel: same-step; step_ov_kernel: next-step) and of BASELINE config 4 (262 144
# HeliForwardFlight envs, the template step kernel).  Summaries -> gpurun_out/sum_<tag>/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=r06_rt_same KERNEL_RE=retrim_kernel BENCH_ARGS="--reset-mode retrim --autoreset-mode same_step" bash scripts/profile_round.sh || exit 3
TAG=r06_rt_next KERNEL_RE=step_ov_kernel BENCH_ARGS="--reset-mode retrim --autoreset-mode next_step" bash scripts/profile_round.sh || exit 4
TAG=r06_cfg4 N=262144 TASK=forward_flight bash scripts/profile_round.sh || exit 5
