# BASELINE config 5's per-GPU shares on one GPU: 1 048 576 envs over N = 1, 2, 4, 8 ranks (the
# driver's 8-GPU run has each rank step its 1 048 576 / N envs; the data path has no collective).
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
out=gpurun_out/config5_shares.jsonl; : > $out
for n in 1048576 524288 262144 131072; do
  timeout -k 10 200 python bench.py --envs $n --steps 500 --repeats 3 --no-secondary --no-cpu-baseline --no-parity >> $out 2> gpurun_out/c5_err.log || { echo "FAILED $n"; tail -3 gpurun_out/c5_err.log; exit 3; }
done
python3 - <<'PY'
import json
for l in open("gpurun_out/config5_shares.jsonl"):
    d = json.loads(l); n = d["config"]["envs_per_gpu"]
    print(f'{n:8d} envs/GPU (1M over {1048576 // n} GPUs): {d["ms_per_step"]*1e3:7.2f} us/step  {d["value"]:.3e} env-steps/s per GPU  frac {d["roofline"]["frac"]:.3f}')
PY
