set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for v in "X=0" "HIP_FORCE_DEV_KERNARG=1" "HIP_FORCE_DEV_KERNARG=0"; do
  env $v timeout -k 10 200 python bench.py --steps 1000 --repeats 3 --no-cpu-baseline --no-parity > gpurun_out/eager.log 2>&1 || { echo "$v failed"; tail -5 gpurun_out/eager.log; exit 3; }
  echo "$v $(tail -1 gpurun_out/eager.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"]*1e3,3), "eager", round(d["step_api_eager"]["ms_per_step"]*1e3,3), "rinfo", round(d["step_with_reset_info"]["ms_per_step"]*1e3,3), "retrim", round(d.get("retrim",{}).get("ms_per_step",0)*1e3,2))')"
done
HELIGYM_AMD_LIB=$PWD/build/variants/timing.so timeout -k 10 120 python scripts/timing_probe.py > gpurun_out/phase_timing.txt 2>&1 || { echo "timing failed"; exit 4; }
cat gpurun_out/phase_timing.txt
