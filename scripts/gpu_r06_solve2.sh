#!/bin/bash
# Round 6: the static-pivot solve after a change -- the standalone solve check, the re-trim phase
# timing, the trim parity tests, then the bench's re-trim lines.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python3 scripts/gj_solve_check.py > gpurun_out/gj_check.txt 2>&1 || { tail -20 gpurun_out/gj_check.txt; exit 3; }
grep -E "static|nostamp|fell" gpurun_out/gj_check.txt | head -12
bash scripts/gpu_r06_rtbench.sh
