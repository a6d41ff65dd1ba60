# FETCH_SIZE / WRITE_SIZE calibration on known byte counts (scripts/ubench/pmc_calib.hip, built
# here into build/ubench/pmc_calib by: hipcc --offload-arch=gfx950 -O3 -o build/ubench/pmc_calib
# scripts/ubench/pmc_calib.hip).  One counter per rocprofv3 pass.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
D=gpurun_out/calib
mkdir -p $D
i=0
for c in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $D/p$i -o run -- ./build/ubench/pmc_calib > $D/p$i.log 2>&1 || { echo "calib pass $c failed"; tail -5 $D/p$i.log; exit 3; }
done
python3 scripts/summarize_calib.py $D
