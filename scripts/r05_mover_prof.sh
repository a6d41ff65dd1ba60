# Round 5: the measured ceiling of the step's own memory pattern past the MALL.
# scripts/ubench/mover.hip moves exactly the step kernel's 315 B per env (tile loads, action, obs via
# LDS, reward / flag bytes, tile stores) with no arithmetic (case 5: 12 waves per CU, the bulk
# kernel's occupancy) and with 1 700 VALU per lane (case 9).  Kernel trace + separate FETCH_SIZE /
# WRITE_SIZE passes at 4 194 304 envs -> gpurun_out/mover_prof/, summarised by
# scripts/summarize_mover.py into profiles/r05_mover_4m_{kernel_stats.csv,pmc_summary.json}.
set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
D=gpurun_out/mover_prof; mkdir -p $D
for c in 5 9; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace$c -o mover -- ./build/ubench/mover 4194304 $c > $D/trace$c.log 2>&1 || { echo "trace $c failed"; tail -5 $D/trace$c.log; exit 3; }
  i=0
  for set in FETCH_SIZE WRITE_SIZE; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $set --output-format csv -d $D/pmc${c}_$i -o run -- ./build/ubench/mover 4194304 $c > $D/pmc${c}_$i.log 2>&1 || { echo "pmc $c $set failed"; tail -5 $D/pmc${c}_$i.log; exit 4; }
  done
done
python3 scripts/summarize_mover.py $D 4194304 > $D/summary.txt && cat $D/summary.txt
# (the CSVs are small: 700 dispatches per case; kept for the local summariser)
