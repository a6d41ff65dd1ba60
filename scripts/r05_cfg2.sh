# Round 5, BASELINE config 2 (4 096 envs, the small-batch helper kernel): the bench line, the kernel
# trace + PMC passes of step_help_kernel (profile_round.sh), and the per-phase lives of its stepping
# and helper waves (HG_TIMING build build/variants/timing.so, scripts/timing_probe.py).
set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 200 python bench.py --envs 4096 --no-secondary --no-cpu-baseline --no-parity > gpurun_out/cfg2_bench.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/cfg2_bench.log; exit 3; }
tail -1 gpurun_out/cfg2_bench.log > gpurun_out/cfg2_line.json
python3 -c "import json; d=json.load(open('gpurun_out/cfg2_line.json')); print('config 2:', round(d['ms_per_step']*1e3,3), 'us/step', d['roofline']['kernel'])"
TAG=${TAG:-r05cfg2} N=4096 PMC_AGE=60 TRACE_STEPS=1000 bash scripts/profile_round.sh > gpurun_out/cfg2_prof.log 2>&1 || { echo "profile failed"; tail -5 gpurun_out/cfg2_prof.log; exit 4; }
python3 - <<'PY'
import json, glob
d = json.load(open(glob.glob("gpurun_out/sum_r05cfg2/r05cfg2_pmc_summary.json")[0]))
c = d["counters_per_launch"]; w = c.get("SQ_WAVES", 1)
print("trace avg us", round((d["kernel_avg_ns_trace"] or 0) / 1e3, 3), "| per wave: VALU", round(c.get("SQ_INSTS_VALU", 0) / w, 1),
      "SALU", round(c.get("SQ_INSTS_SALU", 0) / w, 1), "| wait/wave-cycles", round(c.get("SQ_WAIT_ANY", 0) / max(c.get("SQ_WAVE_CYCLES", 1), 1), 3))
PY
for n in 4096 65536; do
  HELIGYM_AMD_LIB=$PWD/build/variants/timing.so timeout -k 10 120 python scripts/timing_probe.py --envs $n --warm 6000 > gpurun_out/timing_$n.txt 2>&1 || { echo "timing $n failed"; tail -5 gpurun_out/timing_$n.txt; exit 5; }
done
grep -v amdgpu.ids gpurun_out/timing_4096.txt | head -30
