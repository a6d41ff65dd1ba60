# Round-4 probes: phase timing and branch flags of the step on an aged 65 536-env population
# (HG_TIMING build = the default kernel with stamps), and the 4 M-env step with and without ageing.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
HELIGYM_AMD_LIB=$PWD/build/variants/tsplit.so timeout -k 10 120 python scripts/timing_probe.py --warm 3000 > gpurun_out/phase_timing_aged.txt 2>&1 || { echo "timing failed"; tail -5 gpurun_out/phase_timing_aged.txt; exit 3; }
HELIGYM_AMD_LIB=$PWD/build/variants/tsplit.so timeout -k 10 120 python scripts/timing_probe.py --warm 0 > gpurun_out/phase_timing_fresh.txt 2>&1 || { echo "timing failed"; exit 3; }
grep -v amdgpu.ids gpurun_out/phase_timing_aged.txt | head -4; grep -h "branch flags\|waves:" gpurun_out/phase_timing_aged.txt gpurun_out/phase_timing_fresh.txt
for a in 0 30; do
  timeout -k 10 300 python bench.py --envs 4194304 --steps 200 --repeats 3 --age-seconds $a --no-secondary --no-cpu-baseline --no-parity > gpurun_out/b4m_age$a.log 2>&1 || { echo "4M age $a failed"; tail -3 gpurun_out/b4m_age$a.log; exit 4; }
  tail -1 gpurun_out/b4m_age$a.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('4M age $a', round(d['ms_per_step']*1e3,1), 'us', d['timing']['resets_in_window'])"
done
