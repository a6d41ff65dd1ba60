#!/bin/bash
# Round 6: the fused same-step re-trim -- its bitwise test against the serial path first (bounded, one
# process), then the trim tests and the bench's re-trim lines.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -v --timeout 240 --timeout-method thread -m gpu \
    -k "fused" > gpurun_out/fused_tests.txt 2>&1 || { tail -30 gpurun_out/fused_tests.txt; exit 3; }
tail -8 gpurun_out/fused_tests.txt
bash scripts/gpu_r06_rtbench.sh
