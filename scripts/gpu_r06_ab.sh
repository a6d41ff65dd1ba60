#!/bin/bash
# Round 6: interleaved A/B of library variants on the bench's re-trim lines (same-step and next-step),
# two rounds each: VARIANTS="a.so b.so ..." (the default library first).
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
  for lib in heli-gym_amd/heligym_amd/libheligym_amd.so ${VARIANTS:-}; do
    for mode in same_step next_step; do
      HELIGYM_AMD_LIB=$lib timeout -k 10 200 python3 bench.py --reset-mode retrim --autoreset-mode $mode --steps 500 \
          --no-secondary --no-cpu-baseline --no-parity > gpurun_out/ab.json 2> gpurun_out/ab.log || exit 3
      python3 -c "import json; d=json.loads(open('gpurun_out/ab.json').read().strip().splitlines()[-1]); print('$rep $lib $mode', round(d['ms_per_step']*1e3, 3))"
    done
  done
done
