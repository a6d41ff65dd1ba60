# Interleaved A/B of library variants on one bench.py workload -- the one driver for every A/B of
# the kernels (round 4's one-off r04_batch*.sh scripts are folded into it).  Each (round, variant)
# runs bench.py in its own process under its own time limit; the variants alternate within a round,
# so a box's clock / thermal drift hits them alike.
#
#   VARIANTS  "cur prev gear2": cur = the in-tree library, any other name = build/variants/<name>.so
#             (scripts/build_variants.py NAME=-DFLAG=1,...)                          default "cur prev"
#   ARGS      extra bench.py arguments (default: headline workload, 1 000-step windows, 3 repeats)
#   FIELD     the bench-line value compared, a dotted path (ms_per_step, retrim.ms_per_step,
#             out_of_cache.ms_per_step, ...)                                          default ms_per_step
#   ROUNDS    interleaved rounds                                                      default 3
#   TAG       output name under gpurun_out/ (ab_<TAG>.jsonl, one bench line per run)  default ab
#
# e.g.  VARIANTS="cur nogear" ARGS="--envs 4194304 --steps 200 --no-secondary" bash scripts/ab.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
VARIANTS=${VARIANTS:-"cur prev"}
ARGS=${ARGS:-"--steps 1000 --repeats 3 --no-secondary --no-cpu-baseline --no-parity"}
FIELD=${FIELD:-ms_per_step}
ROUNDS=${ROUNDS:-3}
TAG=${TAG:-ab}
out=gpurun_out/ab_$TAG.jsonl; : > "$out"
for r in $(seq 1 "$ROUNDS"); do
  for v in $VARIANTS; do
    if [ "$v" = cur ]; then lib=$PWD/heli-gym_amd/heligym_amd/libheligym_amd.so; else lib=$PWD/build/variants/$v.so; fi
    HELIGYM_AMD_LIB=$lib timeout -k 10 300 python bench.py $ARGS > gpurun_out/ab_run.log 2>&1 \
      || { echo "variant $v (round $r) failed"; tail -5 gpurun_out/ab_run.log; exit 3; }
    tail -1 gpurun_out/ab_run.log | python3 -c "
import json, sys
d = json.loads(sys.stdin.read()); d['variant'] = '$v'; d['ab_round'] = $r
v = d
for k in '$FIELD'.split('.'): v = v[k]
print(json.dumps(d)); print('$v round $r $FIELD', v, file=sys.stderr)" >> "$out"
  done
done
python3 - "$out" "$FIELD" <<'PY'
import json, statistics, sys
path, field = sys.argv[1], sys.argv[2]
vals = {}
for line in open(path):
    d = json.loads(line)
    v = d
    for k in field.split("."):
        v = v[k]
    vals.setdefault(d["variant"], []).append(v)
for name, xs in vals.items():
    print(f"{name:12s} {field}: median {statistics.median(xs):.6g}  all {[round(x, 6) for x in xs]}")
PY
