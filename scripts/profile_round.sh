# Profiles for the judged bench line: rocprofv3 kernel-trace --stats of the bench command, then
# separate --pmc passes (traffic + issue counters).  BENCH_ARGS adds bench.py options (e.g.
# "--reset-mode retrim --autoreset-mode next_step") and KERNEL_RE picks the kernel to summarise.  Results -> gpurun_out/prof_<tag>/ and a
# summary profiles/<tag>_pmc_summary.json written by scripts/summarize_prof.py.
set -u
cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-r01}
N=${N:-65536}
DT=${DT:-0.01}
D=gpurun_out/prof_$TAG
mkdir -p $D
export TMPDIR=/tmp
# ageing: the trace runs the bench's default (60 simulated s); the counter passes, where every dispatch
# is collected separately, age ${PMC_AGE:-20} s (the population is mixed after about 10 s, the
# time-limit cohort aside)
echo "[$TAG] trace"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace -o bench -- python3 bench.py --envs $N --dt $DT --task ${TASK:-hover} ${BENCH_ARGS:-} --steps ${TRACE_STEPS:-1000} --repeats 2 --no-secondary --no-cpu-baseline --no-parity > $D/trace.log 2>&1 || { echo "trace failed"; tail -20 $D/trace.log; exit 3; }
i=0
for set in "FETCH_SIZE" "WRITE_SIZE" \
           "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE" \
           "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  echo "[$TAG] pmc pass $i: $set"
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $set --output-format csv -d $D/pmc$i -o run -- python3 bench.py --envs $N --dt $DT --task ${TASK:-hover} ${BENCH_ARGS:-} --steps 200 --warmup 20 --repeats 1 --age-seconds ${PMC_AGE:-20} --no-secondary --no-cpu-baseline --no-parity > $D/pmc$i.log 2>&1 || { echo "pmc pass $i failed"; tail -20 $D/pmc$i.log; exit 4; }
done
python3 scripts/summarize_prof.py $D $TAG $N $DT ${TASK:-hover} > $D/summary.txt
# profiles/ does not travel back from the box, and the raw traces exceed gpurun_out's 64 MiB: keep the
# summaries, drop the per-dispatch CSVs
mkdir -p gpurun_out/sum_$TAG && cp profiles/${TAG}_* gpurun_out/sum_$TAG/ && find $D -name "*.csv" ! -name "*kernel_stats.csv" -delete
echo "[$TAG] done"
# profiles/ does not travel back from the box: rerun the summariser locally on gpurun_out/prof_$TAG
