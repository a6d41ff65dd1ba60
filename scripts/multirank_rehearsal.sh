# N>1 path of bench.py with 2 ranks sharing the box's one GPU over gloo (the driver's 8-GPU run
# uses RCCL, one rank per GPU); checks the barrier / max-over-ranks / rank-0 JSON logic only.
set -eu
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
HG_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 500 --warmup 20 --no-parity \
  > gpurun_out/rehearsal.json 2> gpurun_out/rehearsal.err
python -c "import json; d=json.loads(open('gpurun_out/rehearsal.json').read().strip().splitlines()[-1]); print(d['n_gpus'], d['value'], d['config']['parallelism'], 'cpu_baseline' in d)"
# ... and the BASELINE config-5 shape: observations all-gathered to every rank each step (eager)
HG_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29518 bench.py --gpus 2 --envs 131072 --steps 50 --warmup 5 --no-parity \
  --gather-obs > gpurun_out/rehearsal_gather.json 2> gpurun_out/rehearsal_gather.err
python -c "import json; d=json.loads(open('gpurun_out/rehearsal_gather.json').read().strip().splitlines()[-1]); print(d['n_gpus'], d['config']['workload'])"
