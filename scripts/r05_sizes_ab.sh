# Round 5: an interleaved A/B of library variants at several BASELINE sizes (headline-only bench lines).
#   VARIANTS="cur galways" SIZES="65536 4096 262144 1048576" TAG=gear bash scripts/r05_sizes_ab.sh
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for n in ${SIZES:-65536 4096 262144 1048576}; do
  steps=1000; [ "$n" -ge 1048576 ] && steps=300
  VARIANTS="${VARIANTS:-cur}" ROUNDS=${ROUNDS:-2} TAG=${TAG:-sz}_$n \
    ARGS="--envs $n --steps $steps --repeats 3 ${EXTRA:-} --no-secondary --no-cpu-baseline --no-parity" bash scripts/ab.sh | tail -${NV:-2} || exit 3
done
