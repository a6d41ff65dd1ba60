#!/bin/bash
# Round 6: trim parity tests, the re-trim phase timing (HG_TIMING build) and the default bench line
# (headline + every secondary, re-trim modes included) on the current library.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -m gpu \
    -k "trim" > gpurun_out/trim_tests.txt 2>&1 &&
HELIGYM_AMD_LIB=build/variants/timing.so timeout -k 10 200 python3 scripts/retrim_timing.py > gpurun_out/rt_static.txt 2>&1 &&
timeout -k 10 500 python3 bench.py > gpurun_out/bench_r06a.json 2> gpurun_out/bench_r06a.log
rc=$?
tail -5 gpurun_out/trim_tests.txt
cat gpurun_out/rt_static.txt
tail -3 gpurun_out/bench_r06a.log
exit $rc
