#!/bin/bash
# Round 6: the fused same-step launch -- its bitwise tests against the serial path, then the bench's
# same-step re-trim line (serial path, round 6 before fusing: 29.4 us per step).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -v --timeout 240 --timeout-method thread -m gpu \
    -k "fused" > gpurun_out/fused_tests.txt 2>&1 || { tail -30 gpurun_out/fused_tests.txt; exit 3; }
grep -E "PASS|FAIL|passed|failed" gpurun_out/fused_tests.txt
timeout -k 10 300 python3 bench.py --reset-mode retrim --autoreset-mode same_step --steps 300 \
    --no-secondary --no-cpu-baseline --no-parity > gpurun_out/fab.json 2> gpurun_out/fab.log || exit 3
python3 -c "import json; d=json.loads(open('gpurun_out/fab.json').read().strip().splitlines()[-1]); print('fused same-step', d['ms_per_step'])"
