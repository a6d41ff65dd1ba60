// baked.h — the default airframe's model constants as compile-time literals.
//
// The step kernel reads ~120 model constants per RK stage.  From a device copy they are scalar
// loads whose waits sit on the critical path of a launch whose waves each own a SIMD (65 536 envs
// = one wave per SIMD), and they outnumber the SGPRs (spills through VGPR lanes).  For the default
// AW109 airframe and terrain (aw109.yaml, helicopter_dynamics.py:107-154, wind_dynamics.py:21-37)
// the constants are compiled in instead (`baked_aw109.inc`, written by
// scripts/gen_baked_constants.py from derive<float>), so they become instruction literals.
// hg_create selects the baked kernel only when every baked field of the env's constants is
// bit-identical to the compiled-in value; any other airframe, terrain size or wind uses the generic
// kernel.  The fields that change per env or per setter (dt, target, episode limits, flags) are
// never baked.
#pragma once

#include "physics.h"

// Every airframe-derived field of Params (dt-, target- and option-independent).
#define HG_BAKED_FIELDS(X)                                                                          \
    X(coll0) X(coll1) X(lon0) X(lon1) X(lat0) X(lat1) X(ped0) X(ped1)                               \
    X(lapse_t0) X(ro_sea) X(rho_exp) X(wt) X(inv_mass) X(p_loss) X(vtrans) X(wl_cg_ft)              \
    X(mr_H) X(mr_D) X(mr_IS) X(mr_K1) X(mr_R) X(mr_OMEGA) X(mr_inv_OMEGA) X(mr_VTIP) X(mr_inv_VTIP) \
    X(mr_tw75) X(mr_tw50) X(mr_two3_vtip) X(mr_gam_dro) X(mr_kc_num) X(mr_DL_DB1) X(mr_DL_DA1_dro) \
    X(mr_coef) X(mr_inflow) X(mr_inv_thr_den) X(mr_inv_ct_den) X(mr_prof) X(mr_vtip2) X(mr_2_vtip)  \
    X(mr_8_asig) X(mr_inv_gam_dro) X(mr_inv_R)                                                      \
    X(tr_H) X(tr_D) X(tr_OMEGA) X(tr_VTIP) X(tr_inv_VTIP) X(tr_tw75) X(tr_tw50) X(tr_two3_vtip)     \
    X(tr_coef) X(tr_inflow) X(tr_inv_thr_den)                                                       \
    X(fus_H) X(fus_XUU) X(fus_YVV) X(fus_ZWW) X(fus_COR) X(fus_dfw_k) X(fus_dfw_c)                  \
    X(ht_D) X(ht_ZUU) X(ht_ZUW) X(ht_ZMAX) X(ht_dw_k) X(ht_dw_c)                                    \
    X(vt_H) X(vt_D) X(vt_YUU) X(vt_YUV) X(vt_YMAX) X(wn_ZUU) X(wn_ZUW) X(wn_ZMAX) X(wn_on)          \
    X(lg_K) X(lg_C) X(lg_loc[0][0]) X(lg_loc[0][1]) X(lg_loc[0][2]) X(lg_loc[1][0]) X(lg_loc[1][1]) \
    X(lg_loc[1][2]) X(lg_loc[2][0]) X(lg_loc[2][1]) X(lg_loc[2][2]) X(lg_reach)                     \
    X(Ixx) X(Iyy) X(Izz) X(Ixz) X(Ji00) X(Ji02) X(Ji11) X(Ji20) X(Ji22)                             \
    X(hm_sx) X(hm_sy) X(hm_cx) X(hm_cy) X(hm_rows) X(hm_cols) X(ns_half) X(ew_half)                 \
    X(wm[0]) X(wm[1]) X(wm[2]) X(wind_dir_cos) X(wind_dir_sin) X(w20) X(sigma_low) X(turb_level)    \
    X(tep_row[0]) X(tep_row[1]) X(tep_row[2]) X(tep_row[3]) X(tep_row[4]) X(tep_row[5])             \
    X(tep_row[6]) X(tep_row[7]) X(tep_row[8]) X(tep_row[9]) X(tep_row[10]) X(tep_row[11])           \
    X(tep_row[12]) X(n_t) X(n_t2) X(inv_n_x) X(inv_n_v) X(inv_n_a) X(fail_zdot) X(fail_ang)        \
    X(f_kc_irho) X(f_og_irho) X(f_mr_inflow_thr) X(f_tr_inflow_thr) X(f_mr_ct_k) X(f_mr_db_a)       \
    X(f_mr_db_b) X(f_hXUU) X(f_hYVV) X(f_hZWW) X(f_zd) X(f_m2_R) X(f_rho_lz) X(f_gyro[0]) X(f_gyro[1])    \
    X(f_gyro[2]) X(f_gyro[3]) X(f_gyro[4]) X(f_gyro[5])

// The fields that stay runtime values in the baked kernel (dt, task, target, limits, flags): with
// HG_BAKED_FIELDS they cover every field of Params<float> (checked below).
#define HG_RUNTIME_FIELDS(X)                                                                        \
    X(dt) X(half_dt) X(dt6) X(eta_norm) X(tgt_n[0]) X(tgt_n[1]) X(tgt_n[2]) X(vel_tgt_n)            \
    X(dwn_tgt_n) X(task) X(time_up_steps) X(success_steps) X(autoreset) X(reset_retrim)            \
    X(autoreset_next) X(max_episode_steps) X(env_templates) X(f_dpsi_mr) X(f_dpsi_tr)

namespace hg {

struct ParamWords {
    uint32_t w[sizeof(Params<float>) / 4];
};
static_assert(sizeof(ParamWords) == sizeof(Params<float>), "Params<float> must be whole dwords");

// derive<float>() of the default config (baked fields only; the rest are zero)
// HG_BAKED_INC: another airframe's image, for the run-time specialised code objects (step_rtc.hip)
#ifndef HG_BAKED_INC
#define HG_BAKED_INC "baked_aw109.inc"
#endif
constexpr Params<float> kBakedAW109 = __builtin_bit_cast(Params<float>, ParamWords{{
#include HG_BAKED_INC
}});

#define HG_FIELD_BYTES(f) +sizeof(((const Params<float>*)nullptr)->f)
static_assert(0 HG_BAKED_FIELDS(HG_FIELD_BYTES) HG_RUNTIME_FIELDS(HG_FIELD_BYTES) == sizeof(Params<float>),
              "every Params field must be listed as baked or runtime");
#undef HG_FIELD_BYTES

// The compiled-in constants with the runtime fields of R.  Built from the constant image (not by
// overwriting a copy of R field by field), so the optimiser sees one constant object plus a few
// scalar stores and keeps every field in a register or an instruction literal.
HD Params<float> bake(const Params<float>& R) {
    Params<float> P = kBakedAW109;
#define HG_RT_ONE(f) P.f = R.f;
    HG_RUNTIME_FIELDS(HG_RT_ONE)
#undef HG_RT_ONE
    return P;
}

// True when every baked field of P equals that of the constant image I (default: the compiled-in
// one) bit for bit.
inline bool bake_matches(const Params<float>& P, const Params<float>& I = kBakedAW109) {
    bool ok = true;
#define HG_BAKE_CMP(f) ok = ok && memcmp(&P.f, &I.f, sizeof(P.f)) == 0;
    HG_BAKED_FIELDS(HG_BAKE_CMP)
#undef HG_BAKE_CMP
    return ok;
}

}  // namespace hg
