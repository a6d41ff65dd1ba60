# Sweep the persistent step kernel's blocks per CU at 4 M envs (HG_PERSIST_BLOCKS_PER_CU)
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for b in ${BS:-0 4 8 12 16 24}; do
  HG_PERSIST_BLOCKS_PER_CU=$b timeout -k 10 180 python bench.py --envs ${N:-4194304} --steps 200 --repeats 3 --warmup 20 --no-secondary --no-cpu-baseline --no-parity > gpurun_out/sweep.log 2>&1 || { echo "b=$b failed"; tail -3 gpurun_out/sweep.log; exit 3; }
  echo "b=$b $(grep -m1 'occupancy' gpurun_out/sweep.log) $(tail -1 gpurun_out/sweep.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"]*1e3, 3))') us"
done
