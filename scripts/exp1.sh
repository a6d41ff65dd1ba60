# experiment: async env groups; predicted-cell variant; timing probes
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
HELIGYM_AMD_LIB=$PWD/build/variants/A.so timeout -k 10 200 python scripts/groups_probe.py --envs 65536 262144 1048576 --groups 1 2 4 > gpurun_out/groups.log 2>&1 || { echo groups failed; tail gpurun_out/groups.log; exit 3; }
cat gpurun_out/groups.log
for v in TA TB; do
HELIGYM_AMD_LIB=$PWD/build/variants/$v.so timeout -k 10 120 python scripts/timing_probe.py > gpurun_out/timing_$v.log 2>&1 || { echo timing failed; tail gpurun_out/timing_$v.log; exit 3; }
echo == $v; cat gpurun_out/timing_$v.log
done
VARIANTS="A B" bash scripts/variants.sh
