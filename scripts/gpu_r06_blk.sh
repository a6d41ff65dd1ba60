#!/bin/bash
# Round 6: the block-inverse panel -- solve check (accuracy, fallbacks, cycles against the pivot-step
# panel), trim tests + phase timing, then the interleaved A/B of the re-trim lines against it.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python3 scripts/gj_solve_check.py > gpurun_out/gj_check.txt 2>&1 || { tail -20 gpurun_out/gj_check.txt; exit 3; }
grep -E "static|nostamp|_steps|fell" gpurun_out/gj_check.txt | head -14
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -m gpu \
    -k "trim" > gpurun_out/trim_tests.txt 2>&1 || { tail -30 gpurun_out/trim_tests.txt; exit 4; }
tail -1 gpurun_out/trim_tests.txt
HELIGYM_AMD_LIB=build/variants/timing.so timeout -k 10 200 python3 scripts/retrim_timing.py > gpurun_out/rt_static.txt 2>&1 && cat gpurun_out/rt_static.txt
VARIANTS=build/variants/steps.so bash scripts/gpu_r06_ab.sh
