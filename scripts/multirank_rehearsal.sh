# N>1 path of bench.py with 2 ranks sharing the box's one GPU over gloo (the driver's 8-GPU run
# uses RCCL, one rank per GPU): `--gpus 2` starts its own launcher; checks the barrier /
# max-over-ranks / rank-0 JSON logic and the config-5 gather loop (observations staged through
# the host for gloo).  Timings from such a run are not a measurement.
set -eu
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
HG_BENCH_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 200 --warmup 20 --repeats 2 --no-parity \
  > gpurun_out/rehearsal.json 2> gpurun_out/rehearsal.err
python -c "import json; d=json.loads(open('gpurun_out/rehearsal.json').read().strip().splitlines()[-1]); print(d['n_gpus'], d['value'], d['config']['parallelism'], d['config']['world_size_seen'], 'cpu_baseline' in d, json.dumps(d.get('config5')))"
