#!/bin/bash
# Round 6: A/B of fused same-step launch variants (HELIGYM_AMD_LIB), the bench's same-step re-trim line.
set -o pipefail
mkdir -p gpurun_out
for lib in heli-gym_amd/heligym_amd/libheligym_amd.so ${VARIANTS:-}; do
  HELIGYM_AMD_LIB=$lib timeout -k 10 200 python3 bench.py --reset-mode retrim --autoreset-mode same_step --steps 300 \
      --no-secondary --no-cpu-baseline --no-parity > gpurun_out/fab.json 2> gpurun_out/fab.log || exit 3
  python3 -c "import json; d=json.loads(open('gpurun_out/fab.json').read().strip().splitlines()[-1]); print('$lib', d['ms_per_step'])"
done
