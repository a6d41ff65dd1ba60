set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { echo "== $1"; env $1 timeout -k 10 120 python bench.py --steps 1000 --repeats 3 --no-secondary --no-cpu-baseline --no-parity > gpurun_out/envprobe.log 2>&1 || { echo failed; tail -5 gpurun_out/envprobe.log; exit 3; }; tail -1 gpurun_out/envprobe.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step']*1e3, 'us', d['timing']['window_s'])"; }
run "X=0"
run "HIP_FORCE_DEV_KERNARG=1"
run "HIP_FORCE_DEV_KERNARG=0"
run "DEBUG_CLR_GRAPH_PACKET_CAPTURE=0"
run "DEBUG_CLR_GRAPH_PACKET_CAPTURE=1"
run "HSA_NO_SCRATCH_RECLAIM=1"
