#!/bin/bash
# Round 6 end: pytest -m gpu (one process, per-test limit), smoke(), and the default bench line (headline
# + every secondary, CPU baseline and parity) -> gpurun_out/r06_final_*.  Stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
    > gpurun_out/r06_final_gpu_tests.txt 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/r06_final_gpu_tests.txt; exit 3; }
tail -2 gpurun_out/r06_final_gpu_tests.txt
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06_final_smoke.txt 2>&1 || { echo "smoke failed"; tail -5 gpurun_out/r06_final_smoke.txt; exit 4; }
tail -1 gpurun_out/r06_final_smoke.txt
timeout -k 10 600 python3 bench.py > gpurun_out/r06_final_bench.json 2> gpurun_out/r06_final_bench.log || { echo "bench failed"; tail -5 gpurun_out/r06_final_bench.log; exit 5; }
tail -1 gpurun_out/r06_final_bench.json | cut -c1-400
