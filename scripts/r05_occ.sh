# Round 5: the bulk step variant at two waves per SIMD (173 VGPRs, the in-tree build) against three
# (HG_MIN_WAVES_BULK=3: 168 VGPRs, 24 B of scratch; build/variants/occ3.so), interleaved, at the bulk
# sizes (aged populations).  -> gpurun_out/ab_occ_<N>.jsonl
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for n in ${SIZES:-262144 1048576 4194304}; do
  VARIANTS="cur occ3" ROUNDS=${ROUNDS:-2} TAG=occ_$n \
    ARGS="--envs $n --steps 200 --repeats 3 --age-seconds ${AGE:-30} --no-secondary --no-cpu-baseline --no-parity" bash scripts/ab.sh || exit 3
done
