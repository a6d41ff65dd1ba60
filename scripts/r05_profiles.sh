# Round 5 profiles of the judged kernels (the bench line reads the newest committed summaries):
# headline 65 536 envs (r05a) and the out-of-cache point 4 194 304 envs (r05b), each a rocprofv3
# kernel trace + separate --pmc passes (scripts/profile_round.sh), both on populations aged 60 s.
set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
TAG=r05a N=65536 PMC_AGE=60 bash scripts/profile_round.sh > gpurun_out/prof_r05a.log 2>&1 || { echo "r05a failed"; tail -5 gpurun_out/prof_r05a.log; exit 3; }
TAG=r05b N=4194304 PMC_AGE=60 TRACE_STEPS=200 bash scripts/profile_round.sh > gpurun_out/prof_r05b.log 2>&1 || { echo "r05b failed"; tail -5 gpurun_out/prof_r05b.log; exit 4; }
for t in r05a r05b; do python3 - $t <<'PY'
import json, sys
t = sys.argv[1]
d = json.load(open(f"gpurun_out/sum_{t}/{t}_pmc_summary.json"))
c = d["counters_per_launch"]; w = c.get("SQ_WAVES", 1)
print(t, d["envs"], "trace us", round(d["kernel_avg_ns_trace"] / 1e3, 3), "| VALU/wave", round(c["SQ_INSTS_VALU"] / w, 1),
      "SALU/wave", round(c["SQ_INSTS_SALU"] / w, 1), "| traffic", round(d["hbm_bytes_per_launch"] / 1e6, 2), "MB",
      round(d["hbm_bytes_per_launch"] / d["impl_bytes_per_launch"], 4), "x moved")
PY
done
