// Analysis only (never built into the library): one stage evaluation of the old (physics.h) and the
// new (stage_f32.h) fp32 form, each in a kernel of its own, for static instruction counts.
//   hipcc --offload-arch=gfx950 -O3 ... --cuda-device-only -S scripts/isa/stage_probe.hip
#include <string.h>
#include "../../heli-gym_amd/csrc/stage_f32.h"
#include "../../heli-gym_amd/csrc/baked.h"

using namespace hg;

__global__ void probe_new(const float* __restrict__ in, float* __restrict__ out, const Params<float>* Pa) {
    const Params<float> P = bake(*Pa);
    const int i = threadIdx.x;
    asm volatile("; PROBE begin" ::: "memory");
    const float* q = in + i * 64;
    X16 s = to_x16(q);
    StepCtx c;
    c.wb0 = f2{q[18], q[19]}; c.wb1 = f2{q[20], q[21]}; c.lon_lat = f2{q[22], q[23]}; c.mlat_lon = f2{-q[23], q[22]};
    c.W0 = q[24]; c.W1 = q[25]; c.W2 = q[26]; c.z0 = q[27];
    c.ri0 = f2{q[28], q[29]}; c.riz = f2{q[30], q[31]}; c.itb0 = f2{q[32], q[33]}; c.itbz = f2{q[34], q[35]};
    c.cz = q[36]; c.g.hi = q[37]; c.g.lo = q[38]; c.g.delta = q[39];
    Att2 a;
    a.a[0] = f2{q[40], q[41]}; a.a[1] = f2{q[42], q[43]}; a.a[2] = f2{q[44], q[45]};
    X16 k;
#ifdef PROBE_ATT
    const StepK K = step_k<true>(P);
    a = att_step(K, a, f2{q[46], q[47]}, q[48], s.pp, s.rt.y);
#endif
#ifndef PROBE_ATT
    const StepK K = step_k<true>(P);
#endif
    stage_f32<false>(P, K, c, s, a, k, nullptr);
    float* o = out + i * 18;
    from_x16(k, o);
    asm volatile("; PROBE end" ::: "memory");
}

__global__ void probe_old(const float* __restrict__ in, float* __restrict__ out, const Params<float>* Pa) {
    const Params<float> P = bake(*Pa);
    const int i = threadIdx.x;
    asm volatile("; PROBE begin" ::: "memory");
    const float* q = in + i * 64;
    Controls<float> u = controls(P, q[18], q[19], q[20], q[21]);
    const float W[3] = {q[24], q[25], q[26]};
    Ground<float> g;
    g.hi = q[37]; g.lo = q[38]; g.delta = q[39];
    Attitude<float> a;
    a.s[0] = q[40]; a.c[0] = q[41]; a.s[1] = q[42]; a.c[1] = q[43]; a.s[2] = q[44]; a.c[2] = q[45];
    float k[18], obs[17];
#ifdef PROBE_ATT
    const float e0[3] = {q[46], q[48], q[47]};
    a = attitude_step(a, e0, q + 12);
#endif
    dynamics<false>(P, q, u, W, g, a, k, obs);
    for (int j = 0; j < 18; ++j) out[i * 18 + j] = k[j];
    asm volatile("; PROBE end" ::: "memory");
}
