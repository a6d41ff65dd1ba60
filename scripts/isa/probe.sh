# Static instruction counts of one stage evaluation, old (physics.h) vs new (stage_f32.h).  Analysis only.
set -e
D=${TMPDIR:-/tmp}/isa; mkdir -p $D
R=$(cd "$(dirname "$0")/../.." && pwd)
for att in "" "-DPROBE_ATT"; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fno-hip-fp32-correctly-rounded-divide-sqrt \
    -fgpu-flush-denormals-to-zero -fno-slp-vectorize -ffp-contract=on -mllvm -disable-vector-combine -DHG_ISA_HOT $att --cuda-device-only -S \
    -o $D/probe$att.s $R/scripts/isa/stage_probe.hip
  echo "attitude step included: ${att:-no}"; python3 $R/scripts/isa/probe_count.py $D/probe$att.s "$@"
done
