#!/bin/bash
# Round 6: the trim solve on the GPU -- the standalone solve check (blocked, unblocked, static pivots),
# the re-trim phase timing with the static-pivot solve and without it, then the trim parity tests.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python3 scripts/gj_solve_check.py > gpurun_out/gj_check.txt 2>&1 &&
HELIGYM_AMD_LIB=build/variants/timing.so timeout -k 10 200 python3 scripts/retrim_timing.py > gpurun_out/rt_static.txt 2>&1 &&
HELIGYM_AMD_LIB=build/variants/timing_nostatic.so timeout -k 10 200 python3 scripts/retrim_timing.py > gpurun_out/rt_search.txt 2>&1 &&
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -m gpu \
    -k "trim" > gpurun_out/trim_tests.txt 2>&1
rc=$?
cat gpurun_out/gj_check.txt gpurun_out/rt_static.txt gpurun_out/rt_search.txt
tail -30 gpurun_out/trim_tests.txt
exit $rc
