set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 60 ./build/ubench/issue > gpurun_out/issue.log 2>&1 || { echo issue failed; cat gpurun_out/issue.log; exit 3; }
cat gpurun_out/issue.log
timeout -k 10 60 ./build/ubench/floor > gpurun_out/floor.log 2>&1 || { echo floor failed; cat gpurun_out/floor.log; exit 3; }
cat gpurun_out/floor.log
