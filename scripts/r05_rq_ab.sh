export TMPDIR=/tmp; mkdir -p gpurun_out
for r in 1 2; do for v in cur early; do
  if [ $v = cur ]; then lib=$PWD/heli-gym_amd/heligym_amd/libheligym_amd.so; else lib=$PWD/build/variants/$v.so; fi
  HELIGYM_AMD_LIB=$lib timeout -k 10 400 python3 bench.py --repeats 3 --no-cpu-baseline --no-parity > gpurun_out/rq_${v}_$r.json 2> gpurun_out/rq_${v}_$r.err || { echo "$v failed"; tail -5 gpurun_out/rq_${v}_$r.err; exit 3; }
  python3 -c "
import json,sys; d=json.loads(open('gpurun_out/rq_${v}_$r.json').read().strip().splitlines()[-1])
print('$v', $r, 'head', d['ms_per_step'], 'info', d['step_with_reset_info']['ms_per_step'], 'rt', d['retrim']['ms_per_step'], 'rtn', d['retrim_next_step']['ms_per_step'], '4M', d['out_of_cache']['ms_per_step'])"
done; done
