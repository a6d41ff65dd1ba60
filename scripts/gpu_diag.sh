set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python scripts/diag_parity.py > gpurun_out/diag.log 2>&1; rc=$?
tail -c 20000 gpurun_out/diag.log | tail -150; exit $rc
