#!/bin/bash
# Round 6: trim tests, re-trim phase timing and the bench's re-trim lines only (fast A/B of trim changes).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -m gpu \
    -k "trim" > gpurun_out/trim_tests.txt 2>&1 &&
HELIGYM_AMD_LIB=build/variants/timing.so timeout -k 10 200 python3 scripts/retrim_timing.py > gpurun_out/rt_static.txt 2>&1 &&
for mode in same_step next_step; do
  timeout -k 10 300 python3 bench.py --reset-mode retrim --autoreset-mode $mode --steps 500 --no-secondary \
      --no-cpu-baseline --no-parity > gpurun_out/rtb_$mode.json 2> gpurun_out/rtb_$mode.log || exit 3
done
rc=$?
tail -2 gpurun_out/trim_tests.txt
cat gpurun_out/rt_static.txt
for mode in same_step next_step; do python3 -c "import json,sys; d=json.loads(open('gpurun_out/rtb_$mode.json').read().strip().splitlines()[-1]); print('$mode', d['ms_per_step'])"; done
exit $rc
