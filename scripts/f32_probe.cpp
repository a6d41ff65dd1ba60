// f32_probe.cpp — diagnostic only: the step kernel's fp32 helicopter step (stage_f32.h, the same
// source) compiled for the host, with the stage-4 input state exposed.  Built by
// scripts/f32_probe.py with -mfma -ffp-contract=on so that the host fuses the same multiply-adds
// the device does; what still differs from the device are the transcendental approximations
// (v_sqrt / v_rcp / v_log / v_exp are ~1 ulp on the device, correctly rounded here).  Used to
// attribute fp32 step errors (which part of the step, which term) on the CPU.
#include "../heli-gym_amd/csrc/stage_f32.h"

using hg::Params;

extern "C" {

int probe_params_size(void) { return (int)sizeof(Params<float>); }

// One helicopter step from a [27] state record: wind step, RK4 with the stage-4 input kept.
//   st4[18]: the stage-4 input state (azimuths 0), W[3]: the wind, hc: the committed ground height,
//   obs[17]: the observation, hs_out[18]: the stepped state, k4[18]: its state_dots
int probe_step(const void* params, const float2* hmap, const float* state27, const float* act4, const float* eta3,
               float* obs, float* st4, float* W, float* hc, float* hs_out, float* k4) {
    const Params<float>& P = *reinterpret_cast<const Params<float>*>(params);
    float hs[18], ws[5], carry[4], eta[3];
    for (int c = 0; c < 18; ++c) hs[c] = state27[c];
    hs[2] = hs[3] = 0.f;
    for (int c = 0; c < 5; ++c) ws[c] = state27[18 + c];
    for (int c = 0; c < 4; ++c) carry[c] = state27[23 + c];
    for (int c = 0; c < 3; ++c) eta[c] = eta3[c];
    const hg::GroundCell<float> cell = hg::ground_cell(P, hs[15], hs[16]);
    const hg::GroundTexels tex = hg::ground_fetch(hmap, cell);
    hg::wind_step_f32(P, ws, carry, eta, W);
    const hg::Ground<float> g = hg::ground_combine<float>(tex, cell);
    *hc = g.h();
    const hg::StepCtx ctx = hg::step_ctx(P, act4[0], act4[1], act4[2], act4[3], W[0], W[1], W[2], g, hs[17]);
    hg::RK4Step<false> rk;
    rk.begin(P, ctx, hs, hg::att0(hs));
    // RK4Step::finish with the stage-4 input kept
    hg::X16 k, acc, st;
    hg::stage_f32<false>(P, rk.K, ctx, rk.h, rk.a0, k, obs);
    hg::rk_stage2<true>(rk.h, k, acc, st, P.half_dt);
    hg::stage_f32<false>(P, rk.K, ctx, st, hg::att_step(rk.K, rk.a0, rk.h.pp, rk.h.rt.y, st.pp, st.rt.y), k, obs);
    hg::rk_stage2<false>(rk.h, k, acc, st, P.half_dt);
    hg::stage_f32<false>(P, rk.K, ctx, st, hg::att_step(rk.K, rk.a0, rk.h.pp, rk.h.rt.y, st.pp, st.rt.y), k, obs);
    hg::rk_stage2<false>(rk.h, k, acc, st, P.dt);
    hg::from_x16(st, st4);
    st4[2] = st4[3] = 0.f;
    hg::stage_f32<true>(P, rk.K, ctx, st, hg::att_step(rk.K, rk.a0, rk.h.pp, rk.h.rt.y, st.pp, st.rt.y), k, obs);
    hg::X16 h = rk.h;
    hg::rk_update2(h, k, acc, P.dt6);
    hg::from_x16(h, hs_out);
    hg::from_x16(k, k4);
    return 0;
}

}  // extern "C"
