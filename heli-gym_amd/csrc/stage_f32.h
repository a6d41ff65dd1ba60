// stage_f32.h — the fp32 step's helicopter RK4 (dynamics.py:158-171 over
// HelicopterDynamics.dynamics, helicopter_dynamics.py:400-489), written for gfx950 issue.
//
// physics.h states the model once for both precisions and is what the fp64 trims run; this file
// is the same model for the fp32 step kernel only, rearranged so that a lone wave (one wave per
// SIMD at 65 536 envs) issues as few instructions as possible:
//  * Packed fp32.  A wave alone issues one VALU instruction per ~4-5 cycles whether it is v_fma_f32
//    or v_pk_fma_f32 (two fmas), so every pair of like operations is written as a 2-vector: the
//    main and tail rotor's inflow / thrust / power (:203-300), the horizontal and vertical tail's
//    stall branches (:322-361), the flapping equations (:236-262), the plane rotations of the DCM
//    (kinematic.py:3-17), the RK4 combinations.  The stage state is held as pairs
//    (vi_mr, vi_tr) (b0, b1) (u, v) (w, z) (p, q) (r, theta) (phi, psi) (x, y); the rotor
//    azimuths, which no force model reads, are not part of the stepped state (az_advance).
//  * Work moved out of the stages.  The ISA density (:160-165) and the main rotor's density
//    terms (the flapping time constants ITB, ITB2_OM, :214-221) are evaluated once per step at the
//    committed altitude z0 and linearised in z - z0 (the stage altitudes differ from z0 by
//    dt * |w|: the quadratic term is below 1e-9 relative for |z - z0| < 1 ft, under half an fp32
//    ulp at 10 ft).  Thrust over density (:246 T / (2 pi rho R^2)) and the thrust coefficient
//    (:252) use (wb - vi) * coef directly: the density cancels.  The fuselage's downwash moment
//    Z_F * d_fw (:305-318) is formed as -rho/2 ZWW COR |wa_f| (ua k + c wa_f): no division, and its
//    limit 0 at wa_f = 0 comes out by itself.
//  * Branches.  The H/V-tail stall selections are selects over both (packed) forms; the landing
//    gear (:385-398) and the wing (:363-383) run only in wave-uniform branches and add their loads
//    into the totals there, so a wave off the ground with no wing pays nothing for them.
// Every rearrangement is exact in real arithmetic; the results differ from physics.h's fp32 form by
// rounding only (the parity tests hold both to the same contract against the reference).
#pragma once

#include "physics.h"

#ifndef HG_GEAR_FACTORED   // the landing-gear loads (gear_add): 3 factored over the gear's mirrored geometry with
#define HG_GEAR_FACTORED 3   // per-point selects; 1 factored, per-point branches (round 4); 2 moment only; 0 per point
#endif
#ifndef HG_MID_ANGLE_MRAD   // largest stage attitude increment (mrad) of the long-series angle addition; 0: none
#define HG_MID_ANGLE_MRAD 250
#endif
#ifndef HG_STAGE_FLAG    // diagnostic branch flags (HG_TIMING builds of heligym_amd.hip)
#define HG_STAGE_FLAG(bit) do { } while (0)
#endif
#ifndef HG_STAGE_STAMP   // diagnostic phase stamps (HG_TIMING builds of heligym_amd.hip)
#define HG_STAGE_STAMP(j, ...) do { } while (0)
#endif

namespace hg {

typedef float f2 __attribute__((ext_vector_type(2)));

// The stage state / derivative as pairs.
struct X16 {
    f2 vi;   // vi_mr, vi_tr
    f2 b;    // b0, b1 (betas)
    f2 uv;   // u, v
    f2 wz;   // w, z
    f2 pq;   // p, q
    f2 rt;   // r, theta
    f2 pp;   // phi, psi
    f2 xy;   // x, y
};

// Everything the four stage evaluations of one step share.
struct StepCtx {
    f2 wb0, wb1;          // control-only parts of the blade inflow (mr_wb0, tr_vb0), (mr_wb1, tr_vb1)
    f2 lon_lat, mlat_lon; // cyclic controls (rad): (lon, lat), (-lat, lon)
    float W0, W1, W2;     // wind NED (set_wind, :156-158)
    float z0;             // committed altitude coordinate (the density expansion point)
    f2 ri0, riz;          // (rho, 1/rho) at z0 and their z-derivatives
    f2 itb0, itbz;        // (-ITB2_OM, ITB) at z0 and their z-derivatives
    float cz;             // the gear cannot touch while z < cz (committed-ground bound, conservative)
    Ground<float> g;      // ground under the committed x, y (F6)
};

#ifndef HG_ATT_POLY   // 1: one polynomial pair for every increment up to 0.25 rad; 0: round 4's short / long series
#define HG_ATT_POLY 0
#endif
// the stage-increment polynomials of att_step (HG_ATT_POLY)
constexpr float kAttA1 = -0x1.55552p-3f, kAttA2 = 0x1.107684p-7f;
constexpr float kAttB1 = -0.5f, kAttB2 = 0x1.55551cp-5f, kAttB3 = -0x1.6b4f4ep-10f;

// The model constants the stages use as packed operands, built once per step.  As instruction
// operands a pair of constants must sit in a register pair: left to the compiler, each use
// re-materialises it with two s_mov (which a lone wave issues as slowly as a VALU instruction), so
// the pairs are made opaque (pin) and live in VGPRs across the four stages.
struct StepK {
    f2 is0;                  // (IS_MR, 0)
    f2 coef;                 // (COEF_TH_MR, COEF_TH_TR)
    f2 inflow_thr, inflow;   // inflow ODE coefficients (MR, TR)
    f2 hxy;                  // (XUU / 2, YVV / 2)
    f2 zmax, zuu, zuw;       // (HT, VT) stall / linear coefficients
    f2 one_m1, mh_h;         // (1, -1), (-H_MR, H_MR)
    f2 j0, j2, g_pq, g_qr;   // I^-1 columns for (p', r') and the gyroscopic coefficients
    f2 k1, dl_db1;           // (K1, K1), (DL_DB1, DL_DB1)
    f2 c6, c24;              // (-1/6, -1/6), (1/24, 1/24)
    f2 aa1, aa2, ab2, ab3;   // the stage-increment polynomials' coefficients (att_step), as pairs
};

// Packed products whose sign flip or lane swap is an operand modifier of v_pk_fma_f32 (op_sel /
// op_sel_hi pick each lane's half of a register pair, neg_lo / neg_hi negate a lane): the compiler
// folds a broadcast-and-negate of a scalar in its own register, but not of one lane of a pair,
// where it builds the operand with a v_xor and a v_mov first.  Written out here for the pair-lane
// cases; the host pass (never executed) gets the plain expression.
#ifndef HG_PK_ASM
#define HG_PK_ASM 1
#endif
#if defined(__HIP_DEVICE_COMPILE__) && HG_PK_ASM
#define HG_PKFMA(A, B, C, MODS, ...)                                                              \
    ({                                                                                          \
        f2 r_;                                                                                  \
        asm("v_pk_fma_f32 %0, %1, %2, %3 " MODS : "=v"(r_) : "v"(A), "v"(B), "v"(C));          \
        r_;                                                                                     \
    })
#define HG_PKMUL(A, B, MODS, ...)                                                                 \
    ({                                                                                          \
        f2 r_;                                                                                  \
        asm("v_pk_mul_f32 %0, %1, %2 " MODS : "=v"(r_) : "v"(A), "v"(B));                      \
        r_;                                                                                     \
    })
#else
#define HG_PKFMA(A, B, C, MODS, ...) (__VA_ARGS__)
#define HG_PKMUL(A, B, MODS, ...) (__VA_ARGS__)
#endif
// a.yx * (b.x, -b.x) + c
HD f2 fma_sw_bxn(f2 a, f2 b, f2 c) {
    return HG_PKFMA(a, b, c, "op_sel:[1,0,0] op_sel_hi:[0,0,1] neg_hi:[0,1,0]", a.yx * f2{b.x, -b.x} + c);
}
// a.yx * (b.y, -b.y) + c
HD f2 fma_sw_byn(f2 a, f2 b, f2 c) {
    return HG_PKFMA(a, b, c, "op_sel:[1,1,0] op_sel_hi:[0,1,1] neg_hi:[0,1,0]", a.yx * f2{b.y, -b.y} + c);
}
// a * (-b.x, b.x) + c
HD f2 fma_nbx(f2 a, f2 b, f2 c) {
    return HG_PKFMA(a, b, c, "op_sel_hi:[1,0,1] neg_lo:[0,1,0]", a * f2{-b.x, b.x} + c);
}
// a * (b.x, -b.x) - c
HD f2 fms_bxn(f2 a, f2 b, f2 c) {
    return HG_PKFMA(a, b, c, "op_sel_hi:[1,0,1] neg_lo:[0,0,1] neg_hi:[0,1,1]", a * f2{b.x, -b.x} - c);
}
// a * (b.x, -b.x)
HD f2 mul_bxn(f2 a, f2 b) {
    return HG_PKMUL(a, b, "op_sel_hi:[1,0] neg_hi:[0,1]", a * f2{b.x, -b.x});
}
// (a.y, -a.x) * b.x + c
HD f2 fma_swn_bx(f2 a, f2 b, f2 c) {
    return HG_PKFMA(a, b, c, "op_sel:[1,0,0] op_sel_hi:[0,0,1] neg_hi:[1,0,0]", f2{a.y, -a.x} * b.x + c);
}
// (a.y, -a.x) * b.y + c
HD f2 fma_swn_by(f2 a, f2 b, f2 c) {
    return HG_PKFMA(a, b, c, "op_sel:[1,1,0] op_sel_hi:[0,1,1] neg_hi:[1,0,0]", f2{a.y, -a.x} * b.y + c);
}
// (-a.y, a.x) * b.x + c
HD f2 fma_nsw_bx(f2 a, f2 b, f2 c) {
    return HG_PKFMA(a, b, c, "op_sel:[1,0,0] op_sel_hi:[0,0,1] neg_lo:[1,0,0]", f2{-a.y, a.x} * b.x + c);
}

HD void pin(f2& x) {
#if defined(__HIP_DEVICE_COMPILE__)
    asm volatile("" : "+v"(x));
#else
    (void)x;
#endif
}

// PIN: a lone wave per SIMD (the launch fits one wave per SIMD), where a scalar instruction costs the
// wave an issue slot and registers are free; with several waves per SIMD the compiler's choice
// (constants re-materialised by SALU, which co-issues with other waves' VALU) keeps VGPRs for occupancy.
template <bool PIN>
HD StepK step_k(const Params<float>& P) {
    StepK K;
    K.is0 = f2{P.mr_IS, 0.f};
    K.coef = f2{P.mr_coef, P.tr_coef};
    K.inflow_thr = f2{P.f_mr_inflow_thr, P.f_tr_inflow_thr};
    K.inflow = f2{P.mr_inflow, P.tr_inflow};
    K.hxy = f2{P.f_hXUU, P.f_hYVV};
    K.zmax = f2{P.ht_ZMAX, P.vt_YMAX};
    K.zuu = f2{P.ht_ZUU, P.vt_YUU};
    K.zuw = f2{P.ht_ZUW, P.vt_YUV};
    K.one_m1 = f2{1.f, -1.f};
    K.mh_h = f2{-P.mr_H, P.mr_H};
    K.j0 = f2{P.Ji00, P.Ji20};
    K.j2 = f2{P.Ji02, P.Ji22};
    K.g_pq = f2{P.f_gyro[0], P.f_gyro[1]};
    K.g_qr = f2{P.f_gyro[2], P.f_gyro[3]};
    K.k1 = f2{P.mr_K1, P.mr_K1};
    K.dl_db1 = f2{P.mr_DL_DB1, P.mr_DL_DB1};
    K.c6 = f2{-1.f / 6.f, -1.f / 6.f};
    K.c24 = f2{1.f / 24.f, 1.f / 24.f};
    K.aa1 = f2{kAttA1, kAttA1};
    K.aa2 = f2{kAttA2, kAttA2};
    K.ab2 = f2{kAttB2, kAttB2};
    K.ab3 = f2{kAttB3, kAttB3};
    if (!PIN) return K;
    pin(K.is0); pin(K.coef); pin(K.inflow_thr); pin(K.inflow); pin(K.hxy); pin(K.zmax); pin(K.zuu);
    pin(K.zuw); pin(K.one_m1); pin(K.mh_h); pin(K.j0); pin(K.j2); pin(K.g_pq); pin(K.g_qr); pin(K.k1);
    pin(K.dl_db1);
#if HG_ATT_POLY
    pin(K.aa1); pin(K.aa2); pin(K.ab2); pin(K.ab3);
#else
    pin(K.c6); pin(K.c24);
#endif
    return K;
}

// WindDynamics.step (dynamics.py:158-171 + wind_dynamics.py:85-125) for the fp32 step, the v and
// w filters (the same second-order form with their own time constant) packed as pairs
// Q = (vs0, ws0), R = (vs1, ws1); u is the first-order filter.  QUIRK: the update is
// s += dt k4, the stage inputs still formed from k1..k3; the wind output from the stage-4 input.
// Same operations per component as physics.h wind_step, so the same roundings.
template <bool UNIFORM = false>
HD void wind_step_f32(const Params<float>& P, float s[5], const float carry[4], const float eta[3], float W[3]) {
    const WindPar<float> w = wind_params<float, UNIFORM>(P, carry);
    const f2 A = f2{w.a_v, w.a_w}, B = f2{w.b_v, w.b_w}, E = f2{eta[1], eta[2]};
    const float U = s[0];
    const f2 Q = f2{s[1], s[3]}, R = f2{s[2], s[4]};
    const float h = P.half_dt, dt = P.dt;
    // stage 1..3 inputs: (U, Q, R) + h (kU, kQ, kR), kR = Q
    float kU = w.a_u * (eta[0] - U);
    f2 kQ = B * (E - R) - A * Q;
    float U1 = U + kU * h;
    f2 Q1 = Q + kQ * h, R1 = R + Q * h;
    kU = w.a_u * (eta[0] - U1);
    kQ = B * (E - R1) - A * Q1;
    float U2 = U + kU * h;
    f2 Q2 = Q + kQ * h, R2 = R + Q1 * h;
    kU = w.a_u * (eta[0] - U2);
    kQ = B * (E - R2) - A * Q2;
    const float U3 = U + kU * dt;
    const f2 Q3 = Q + kQ * dt, R3 = R + Q2 * dt;
    kU = w.a_u * (eta[0] - U3);
    kQ = B * (E - R3) - A * Q3;
    // output at the stage-4 input (wind_dynamics.py:111-123)
    const float ut = w.K_u * U3;
    const f2 vw = f2{w.K_v, w.K_w} * (R3 + (float)(2 * kSqrt3) * Q3);
    W[0] = P.wm[0] + (w.cos_az * ut - w.sin_az * vw.x);
    W[1] = P.wm[1] + (w.sin_az * ut + w.cos_az * vw.x);
    W[2] = P.wm[2] + vw.y;
    // update with k4 only (F3)
    s[0] = U + dt * kU;
    const f2 Qn = Q + dt * kQ, Rn = R + dt * Q3;
    s[1] = Qn.x; s[3] = Qn.y;
    s[2] = Rn.x; s[4] = Rn.y;
}

// (sin, cos) of the three attitude angles
struct Att2 {
    f2 a[3];
};

HD f2 sincos2(float x) {
    float s, c;
    m_sincos(x, &s, &c);
    return f2{s, c};
}

// The step's shared part: controls (:414-422 + the control terms of :226, :281), the density
// expansion at the committed altitude, the gear-contact bound.
HD StepCtx step_ctx(const Params<float>& P, float a0, float a1, float a2, float a3, float W0, float W1, float W2,
                    const Ground<float>& g, float z0) {
    StepCtx c;
    const float coll = P.coll0 + P.coll1 * a0;
    const float lon = P.lon0 + P.lon1 * a1;
    const float lat = P.lat0 + P.lat1 * a2;
    c.lon_lat = f2{lon, lat};
    c.mlat_lon = f2{-lat, lon};
    const float ped = P.ped0 + P.ped1 * a3;
    c.wb0 = f2{P.mr_two3_vtip, P.tr_two3_vtip} * (f2{coll, ped} + f2{P.mr_tw75, P.tr_tw75});
    c.wb1 = f2{P.mr_inv_VTIP, P.tr_inv_VTIP} * (f2{coll, ped} + f2{P.mr_tw50, P.tr_tw50});
    c.W0 = W0;
    c.W1 = W1;
    c.W2 = W2;
    c.g = g;
    c.z0 = z0;
    // ISA density rho(z) = RO_SEA (1 + l z)^e (:160-165) and d rho / dz = rho e l / (1 + l z)
    const float base = 1.f + P.lapse_t0 * z0;
    const float rho = P.ro_sea * m_exp2(P.rho_exp * m_log2(base));
    const float irho = m_rcp(rho);
    const float rz = rho * P.f_rho_lz * m_rcp(base);
    c.ri0 = f2{rho, irho};
    c.riz = f2{rz, -rz * irho * irho};
    // flapping time constants (:214-221): og = OM igam, ITB2_OM = OM / (1 + og^2), ITB = ITB2_OM og
    const float og = P.f_og_irho * irho;
    const float iD = m_rcp(1.f + og * og);
    const float itb2 = P.mr_OMEGA * iD;
    const float itb = itb2 * og;
    const float dog = P.f_og_irho * c.riz.y;            // d og / dz
    const float ditb2 = -2.f * itb2 * og * dog * iD;    // d ITB2_OM / dz
    c.itb0 = f2{-itb2, itb};
    c.itbz = f2{-ditb2, ditb2 * og + itb2 * dog};
    // a gear point's pos_z + h is at most zh + lg_reach (see tail_loads), zh = z + h
    c.cz = -P.wl_cg_ft - P.lg_reach - g.h();
    return c;
}

// Attitude of a stage from the committed one by the angle-addition formulas (physics.h
// attitude_step), on (sin, cos) pairs; a wave with a large stage increment takes the full sincos.
#if HG_ATT_POLY
// sin d = d + d^3 (A1 + A2 d^2) and cos d = 1 + d^2 (B1 + d^2 (B2 + B3 d^2)), fitted on |d| <= 0.25 rad:
// within 0.55 fp32 ulp of sin / cos over that range evaluated in fp32 (the round-4 short series: 1.19
// ulp at 0.05), so every wave up to 0.25 rad (all but ~1 % of an aged population's waves) takes this
// one branch-free form; past it the wave takes the full sincos.
template <bool MIDALL = false, bool SEL = false>   // (no long-series branch to remove here)
HD Att2 att_step(const StepK& K, const Att2& a0, f2 pp0, float th0, f2 pp, float th) {
    const f2 d01 = pp - pp0;   // phi, psi increments
    const float d2 = th - th0;
    const f2 q01 = d01 * d01;
    const f2 sd01 = (d01 * q01) * (K.aa1 + q01 * K.aa2) + d01;
    const f2 cd01 = q01 * (kAttB1 + q01 * (K.ab2 + q01 * K.ab3)) + 1.f;
    const float q2 = d2 * d2;
    const float sd2 = (d2 * q2) * (kAttA1 + q2 * kAttA2) + d2;
    const float cd2 = q2 * (kAttB1 + q2 * (kAttB2 + q2 * kAttB3)) + 1.f;
    // (sin, cos)(e + d) = (s, c) cd + (c, -s) sd
    const f2 A0 = a0.a[0], A1 = a0.a[1], A2 = a0.a[2];
    Att2 a;
    a.a[0] = fma_swn_bx(A0, sd01, A0 * cd01.x);
    a.a[1] = A1 * cd2 + f2{A1.y, -A1.x} * sd2;
    a.a[2] = fma_swn_by(A2, sd01, A2 * cd01.y);
    constexpr float kMax = 0.25f;   // (NaN increments: not in range, the full sincos)
    const bool in = m_fabs(d01.x) <= kMax && m_fabs(d01.y) <= kMax && m_fabs(d2) <= kMax;
#ifndef HG_ISA_HOT
    if (wave_any(!in)) {
        HG_STAGE_FLAG(8);
        if (!in) {
            a.a[0] = sincos2(pp.x);
            a.a[1] = sincos2(th);
            a.a[2] = sincos2(pp.y);
        }
    }
#endif
    return a;
}
#else
// MIDALL: the long series formed by every wave and selected per lane, no wave-uniform branch around
// it.  SEL: inside the wave-uniform branches, the per-lane choices as selects instead of divergent
// branches (every lane runs the series / sincos, as a divergent branch's masked lanes would).
template <bool MIDALL = false, bool SEL = false>
HD Att2 att_step(const StepK& K, const Att2& a0, f2 pp0, float th0, f2 pp, float th) {
    const f2 d01 = pp - pp0;   // phi, psi increments
    const float d2 = th - th0;
    // sin d = d - d^3/6, cos d = 1 - d^2/2 + d^4/24 (|d| <= 0.05: within 2.7e-9 / 2.2e-11)
    const f2 q01 = d01 * d01;
    const f2 sd01 = d01 + (d01 * q01) * K.c6;
    const f2 cd01 = 1.f + q01 * (-0.5f + q01 * K.c24);
    const float q2 = d2 * d2;
    const float sd2 = d2 + (d2 * q2) * K.c6.x;
    const float cd2 = 1.f + q2 * (-0.5f + q2 * K.c24.x);
    // (sin, cos)(e + d) = (s, c) cd + (c, -s) sd
    const f2 A0 = a0.a[0], A1 = a0.a[1], A2 = a0.a[2];
    Att2 a;
    a.a[0] = fma_swn_bx(A0, sd01, A0 * cd01.x);
    a.a[1] = A1 * cd2 + f2{A1.y, -A1.x} * sd2;
    a.a[2] = fma_swn_by(A2, sd01, A2 * cd01.y);
    // a lane with a larger increment (a tumbling env), in a wave-uniform branch: up to HG_MID_ANGLE_MRAD
    // the same angle addition with the series of sin d / cos d carried to d^7 / d^8 (truncation below
    // 6e-11 at 0.25 rad, so a few fp32 ulps like the short series at 0.05), past it the full sincos
    const bool small = m_fabs(d01.x) <= 0.05f && m_fabs(d01.y) <= 0.05f && m_fabs(d2) <= 0.05f;
#ifndef HG_ISA_HOT   // (analysis builds only: the hot path without its cold branches)
    if ((MIDALL && HG_MID_ANGLE_MRAD > 0) || wave_any(!small)) {
#else
    if (false) {
#endif
        HG_STAGE_FLAG(4);
#if HG_MID_ANGLE_MRAD > 0
        constexpr float kMid = HG_MID_ANGLE_MRAD * 1e-3f;   // (NaN increments: neither, the full sincos)
        const bool mid = m_fabs(d01.x) <= kMid && m_fabs(d01.y) <= kMid && m_fabs(d2) <= kMid;
        if (MIDALL || SEL || (!small && mid)) {
            const f2 ms = d01 + (d01 * q01) * (K.c6 + q01 * (1.f / 120.f + q01 * (-1.f / 5040.f)));
            const f2 mc = 1.f + q01 * (-0.5f + q01 * (K.c24 + q01 * (-1.f / 720.f + q01 * (1.f / 40320.f))));
            const float ms2 = d2 + (d2 * q2) * (K.c6.x + q2 * (1.f / 120.f + q2 * (-1.f / 5040.f)));
            const float mc2 = 1.f + q2 * (-0.5f + q2 * (K.c24.x + q2 * (-1.f / 720.f + q2 * (1.f / 40320.f))));
            const f2 m0 = fma_swn_bx(A0, ms, A0 * mc.x);
            const f2 m1 = A1 * mc2 + f2{A1.y, -A1.x} * ms2;
            const f2 m2 = fma_swn_by(A2, ms, A2 * mc.y);
            const bool take = (MIDALL || SEL) ? (!small && mid) : true;
            a.a[0] = take ? m0 : a.a[0];
            a.a[1] = take ? m1 : a.a[1];
            a.a[2] = take ? m2 : a.a[2];
        }
        if (wave_any(!mid)) {
            HG_STAGE_FLAG(8);
            if constexpr (SEL) {
                const f2 f0 = sincos2(pp.x), f1 = sincos2(th), f2s = sincos2(pp.y);
                a.a[0] = mid ? a.a[0] : f0;
                a.a[1] = mid ? a.a[1] : f1;
                a.a[2] = mid ? a.a[2] : f2s;
            } else if (!mid) {
                a.a[0] = sincos2(pp.x);
                a.a[1] = sincos2(th);
                a.a[2] = sincos2(pp.y);
            }
        }
#else
        if (!small) {
            a.a[0] = sincos2(pp.x);
            a.a[1] = sincos2(th);
            a.a[2] = sincos2(pp.y);
        }
#endif
    }
    return a;
}
#endif

// Stage parts that do not read the wind: the kinematics and the landing gear (:385-398).  Inlined in
// place in every stage; the small-batch kernel forms stage 1's (stage_pre) while a helper wave runs
// the wind step (heligym_amd.hip step_help_kernel).  The same expressions either way.
struct Kin {
    f2 sqth, n01;
    float phid, psid, n2;
};

HD Kin kinematics(const X16& s, const Att2& at) {
    // kinematic.py:3-29, :423-431.  Rotations are written so that every sign flip and lane swap is an
    // operand modifier of the packed instruction: (s, c).yx * (x, -x) etc.
    const float v = s.uv.y, p = s.pq.x, q = s.pq.y;
    const f2 SC0 = at.a[0], SC1 = at.a[1], SC2 = at.a[2];
    const float s1 = SC1.x, c1 = SC1.y;
    Kin o;
    const float ic1 = m_rcp(c1);
    o.sqth = fma_sw_bxn(SC0, s.rt, SC0 * q);                    // SC0 q + SC0.yx (r, -r) = (s0 q + c0 r, theta')
    o.phid = p + (s1 * ic1) * o.sqth.x;
    o.psid = ic1 * o.sqth.x;
    // NED velocity B^T uvw = Rz^T Ry^T Rx^T uvw
    const f2 yz1 = fma_nbx(SC0, s.wz, SC0.yx * v);              // SC0.yx v + SC0 (-w, w) = Rx^T (y, z)
    const f2 xz2 = fma_sw_bxn(SC1, s.uv, SC1 * yz1.y);         // SC1.yx (u, -u) + SC1 yz1.y = Ry^T (x, z)
    o.n01 = fma_nbx(SC2, yz1, SC2.yx * xz2.x);                 // SC2.yx xz2.x - SC2 (y, -y) = Rz^T (x, y)
    o.n2 = xz2.y;
    return o;
}

// The landing gear's loads added into the totals, only where some lane of the wave may touch
// (`ran`: the wave took the branch).  QUIRK: the moment uses the ACCUMULATED force (:397).
// ALWAYS (the lone-wave kernels, with the factored form's per-point selects): no wave-uniform skip.
// In an aged population nearly every wave has a lane within the gear's reach of the ground, so the
// skip is rarely taken, and without the branch the scheduler interleaves the gear with the rest of
// the stage (65 536 envs: 7.07 -> 6.93 us).  Waves with no lane near the ground add zeros.  With
// several waves per SIMD (the bulk variant) the skip stays: there the extra registers spill.
#ifndef HG_GEAR_ALWAYS_LONE
#define HG_GEAR_ALWAYS_LONE 1
#endif
// The attitude long series without its branch (att_step<true>): in the small-batch helper kernel
// (4 096 envs 5.27 -> 5.21 us); in the other lone-wave kernels it costs more than the branch
// (65 536 envs 6.94 -> 7.06 us; profiles/r05_gear_always_ab.txt)
#ifndef HG_MIDALL_HELP
#define HG_MIDALL_HELP 1
#endif
// The per-lane attitude choices inside its wave-uniform branches as selects, in the lone-wave kernels
// other than the helper one (65 536 envs 6.83 -> 6.79 us; 4 096 envs, the helper kernel, +0.03 us)
#ifndef HG_ATT_SEL_LONE
#define HG_ATT_SEL_LONE 1
#endif
template <bool ALWAYS = false>
HD void gear_add(const Params<float>& P, const StepCtx& c, const X16& s, const Att2& at, float n2, float& Fx, f2& Fyz,
                 float& Mx, float& My, float& Mz, bool& ran) {
    const float z = s.wz.y, p = s.pq.x, q = s.pq.y, r = s.rt.x;
    const f2 SC0 = at.a[0];
    const float s1 = at.a[1].x, c1 = at.a[1].y;
#if !defined(HG_ISA_HOT) && !defined(HG_ISA_NOGEAR)
    if ((ALWAYS && HG_GEAR_FACTORED == 3) || wave_any(z > c.cz)) {
#else
    if (false) {
#endif
        HG_STAGE_FLAG(2);
#ifdef HG_ISA_MARK
        asm volatile("; GEAR_BEGIN");
#endif
        const float zh = c.g.zh(z);
        const f2 B22 = SC0 * c1;   // (B12, B22); B02 = -s1
#if HG_GEAR_FACTORED == 2
        // Force and contact velocity per point as the reference forms them (the force bitwise the
        // per-point form); only the QUIRK moment factored: sum_i r_i x F_acc(i), F_acc(i) = S_i b with
        // S_i the running sum of the fz, is (sum_i S_i r_i) x b.
        float Fl0 = 0.f, Fl1 = 0.f, Fl2 = 0.f;
        float S = 0.f, Rx = 0.f, Ry = 0.f, Rz = 0.f;
#pragma unroll
        for (int gi = 0; gi < 3; ++gi) {
            const float rx = P.lg_loc[gi][0], ry = P.lg_loc[gi][1], rz = P.lg_loc[gi][2];
            const float pzh = zh + (-s1 * rx + B22.x * ry + B22.y * rz);   // pos_z + h
            if (-pzh - P.wl_cg_ft < 0.f) {
                const float cx = q * rz - r * ry, cy = r * rx - p * rz, cz = p * ry - q * rx;
                const float vel_z = n2 + (-s1 * cx + B22.x * cy + B22.y * cz);
                const float fz = -(P.lg_C * vel_z + P.lg_K * pzh) + (float)kEps;
                Fl0 += -s1 * fz; Fl1 += B22.x * fz; Fl2 += B22.y * fz;
                S = gi == 0 ? fz : S + fz;
                Rx = rx != 0.f ? (gi == 0 ? S * rx : fmaf(S, rx, Rx)) : Rx;
                Ry = ry != 0.f ? (gi == 0 ? S * ry : fmaf(S, ry, Ry)) : Ry;
                Rz = rz != 0.f ? (gi == 0 ? S * rz : fmaf(S, rz, Rz)) : Rz;
            }
        }
        const float bx = -s1, by = B22.x, bz = B22.y;
        const float Ml0 = Ry * bz - Rz * by, Ml1 = Rz * bx - Rx * bz, Ml2 = Rx * by - Ry * bx;
#elif HG_GEAR_FACTORED == 3
        // Factored as below, with the gear's own geometry: the reference places the nose wheel at
        // (x0, 0, zr) and the two mains at (x1, +-y1, zr) (helicopter_dynamics.py:123-126: one
        // waterline, the mains mirrored about the centre line), so b.r_i = bz zr + bx x_i (+- by y1)
        // and r_i.(b x omega) = zr uz + x_i ux (+- y1 uy) share their first terms, and the per-point
        // contact tests are selects (no divergent branch per point).  QUIRK kept: the moment of point
        // i uses the force accumulated up to it, and only points in contact add a moment.
        const float bx = -s1, by = B22.x, bz = B22.y;
        const float ux = by * r - bz * q, uy = bz * p - bx * r, uz = bx * q - by * p;   // b x omega
        const float x0 = P.lg_loc[0][0], x1 = P.lg_loc[1][0], y1 = P.lg_loc[1][1], zr = P.lg_loc[0][2];
        const float pz_c = zh + bz * zr, v_c = n2 + zr * uz;
        const float pz_m = pz_c + bx * x1, v_m = v_c + x1 * ux;
        const float pz[3] = {pz_c + bx * x0, pz_m + by * y1, pz_m - by * y1};   // pos_z + h
        const float vz[3] = {v_c + x0 * ux, v_m + y1 * uy, v_m - y1 * uy};      // contact velocity
        float w[3], S = 0.f;
#pragma unroll
        for (int gi = 0; gi < 3; ++gi) {
            const bool in = -pz[gi] - P.wl_cg_ft < 0.f;
            const float fz = -(P.lg_C * vz[gi] + P.lg_K * pz[gi]) + (float)kEps;
            S = in ? S + fz : S;
            w[gi] = in ? S : 0.f;
        }
        const float Rx = (w[1] + w[2]) * x1 + w[0] * x0, Ry = (w[1] - w[2]) * y1, Rz = ((w[0] + w[1]) + w[2]) * zr;
        const float Fl0 = S * bx, Fl1 = S * by, Fl2 = S * bz;
        const float Ml0 = Ry * bz - Rz * by, Ml1 = Rz * bx - Rx * bz, Ml2 = Rx * by - Ry * bx;
#elif HG_GEAR_FACTORED
        // Factored: every contact force is fz_i b with b = (-s1, B22) the third DCM column, so the
        // accumulated force after point i is S_i b (S_i the running sum of the fz), the QUIRK moment
        // sum_i r_i x (S_i b) = (sum_i S_i r_i) x b, and the contact velocity n2 + b.(omega x r_i) =
        // n2 + r_i.(b x omega).  The same sums in another order: 4 instead of 12 operations per contact
        // point for the loads, 3 instead of 9 for the velocity.
        const float bx = -s1, by = B22.x, bz = B22.y;
        const float ux = by * r - bz * q, uy = bz * p - bx * r, uz = bx * q - by * p;   // b x omega
        float S = 0.f, Rx = 0.f, Ry = 0.f, Rz = 0.f;
#pragma unroll
        for (int gi = 0; gi < 3; ++gi) {
            const float rx = P.lg_loc[gi][0], ry = P.lg_loc[gi][1], rz = P.lg_loc[gi][2];
            const float pzh = zh + (-s1 * rx + B22.x * ry + B22.y * rz);   // pos_z + h
            if (-pzh - P.wl_cg_ft < 0.f) {
                float ru = rx != 0.f ? rx * ux : 0.f;   // r . (b x omega)
                ru = ry != 0.f ? fmaf(ry, uy, ru) : ru;
                ru = rz != 0.f ? fmaf(rz, uz, ru) : ru;
                const float vel_z = n2 + ru;
                const float fz = -(P.lg_C * vel_z + P.lg_K * pzh) + (float)kEps;
                // (the first point starts the sums; a zero coordinate of a compiled-in gear point drops
                // its term, here and above)
                S = gi == 0 ? fz : S + fz;
                Rx = rx != 0.f ? (gi == 0 ? S * rx : fmaf(S, rx, Rx)) : Rx;
                Ry = ry != 0.f ? (gi == 0 ? S * ry : fmaf(S, ry, Ry)) : Ry;
                Rz = rz != 0.f ? (gi == 0 ? S * rz : fmaf(S, rz, Rz)) : Rz;
            }
        }
        const float Fl0 = S * bx, Fl1 = S * by, Fl2 = S * bz;
        const float Ml0 = Ry * bz - Rz * by, Ml1 = Rz * bx - Rx * bz, Ml2 = Rx * by - Ry * bx;
#else
        float Fl0 = 0.f, Fl1 = 0.f, Fl2 = 0.f, Ml0 = 0.f, Ml1 = 0.f, Ml2 = 0.f;
#pragma unroll
        for (int gi = 0; gi < 3; ++gi) {
            const float rx = P.lg_loc[gi][0], ry = P.lg_loc[gi][1], rz = P.lg_loc[gi][2];
            const float pzh = zh + (-s1 * rx + B22.x * ry + B22.y * rz);   // pos_z + h
            if (-pzh - P.wl_cg_ft < 0.f) {
                const float cx = q * rz - r * ry, cy = r * rx - p * rz, cz = p * ry - q * rx;
                const float vel_z = n2 + (-s1 * cx + B22.x * cy + B22.y * cz);
                const float fz = -(P.lg_C * vel_z + P.lg_K * pzh) + (float)kEps;
                Fl0 += -s1 * fz; Fl1 += B22.x * fz; Fl2 += B22.y * fz;
                Ml0 += ry * Fl2 - rz * Fl1;
                Ml1 += rz * Fl0 - rx * Fl2;
                Ml2 += rx * Fl1 - ry * Fl0;
            }
        }
#endif
        Fx += Fl0;
        Fyz += f2{Fl1, Fl2};
        Mx += Ml0;
        My += Ml1;
        Mz += Ml2;
        ran = true;
#ifdef HG_ISA_MARK
        asm volatile("; GEAR_END");
#endif
    }
}

// Stage 1's wind-independent part, formed ahead (the small-batch kernel)
struct StagePre {
    Kin kin;
    bool gear;
    float Fl0, Ml0, Ml1, Ml2;
    f2 Fl12;
};

template <bool ALWAYS = false>
HD StagePre stage_pre(const Params<float>& P, const StepCtx& c, const X16& s, const Att2& at) {
    StagePre o;
    o.kin = kinematics(s, at);
    o.gear = false;
    // (-0 + x == x for every x, so the totals later add exactly what the inline form adds)
    o.Fl0 = -0.f; o.Fl12 = f2{-0.f, -0.f}; o.Ml0 = -0.f; o.Ml1 = -0.f; o.Ml2 = -0.f;
    gear_add<ALWAYS>(P, c, s, at, o.kin.n2, o.Fl0, o.Fl12, o.Ml0, o.Ml1, o.Ml2, o.gear);
    return o;
}

// One evaluation of the model at stage state s (helicopter_dynamics.py:400-489) -> derivatives k;
// with OBS also the 17 observations (:471-488) and the total power.
template <bool OBS, bool PRE = false, bool ALWAYS = false>
HD void stage_f32(const Params<float>& P, const StepK& K, const StepCtx& c, const X16& s, const Att2& at, X16& k,
                  float* __restrict__ obs, const StagePre* pre = nullptr) {
#ifdef HG_ISA_MARKS
    asm volatile("; HGMARK stage begin");
#endif
    const float u = s.uv.x, v = s.uv.y, w = s.wz.x, z = s.wz.y, p = s.pq.x, q = s.pq.y, r = s.rt.x;
    const f2 SC0 = at.a[0], SC1 = at.a[1], SC2 = at.a[2];
    const float s0 = SC0.x, c0 = SC0.y, s1 = SC1.x, c1 = SC1.y, s2 = SC2.x, c2 = SC2.y;

    (void)s0; (void)c0; (void)s2; (void)c2;
    // ---- kinematics (kinematic.py:3-29, :423-431)
    const Kin kin = PRE ? pre->kin : kinematics(s, at);
    const f2 sqth = kin.sqth;
    const float phid = kin.phid, psid = kin.psid;
    const f2 n01 = kin.n01;
    const float n2 = kin.n2;
    // air-relative body velocity uvw - B W, B = Rx Ry Rz
    const f2 ab = SC2.yx * f2{c.W0, -c.W0} + SC2 * c.W1;       // Rz W (x, y)
    const f2 xg = SC1.yx * ab.x + SC1 * f2{-c.W2, c.W2};       // Ry (x, z)
    const f2 yzw = fma_sw_byn(SC0, ab, SC0 * xg.y);            // SC0 xg.y + SC0.yx (ab.y, -ab.y) = Rx (y, z)
    const float ua = u - xg.x;
    const f2 vwa = f2{v, w} - yzw;
    const float va = vwa.x, wa = vwa.y;
    const f2 B12 = SC0 * c1;                                   // (B12, B22); B02 = -s1

    // ---- density and the main rotor's density terms, linear in z - z0 (see the file comment)
    const float dz = z - c.z0;
    const f2 ri = c.ri0 + c.riz * dz;
    const float rho = ri.x, irho = ri.y;
    const f2 itb = c.itb0 + c.itbz * dz;                       // (-ITB2_OM, ITB)

    // ---- main rotor (:203-270) and tail rotor (:272-300), packed as (MR, TR)
    const f2 B = s.b;
    const f2 BM = B - K.is0;                        // (b0 - IS, b1)
    const float ua2 = ua * ua;
    const float wr = wa + BM.x * ua - BM.y * va;               // (:222-224)
    const float wq = wa + q * P.tr_D;                          // (:276-279)
    const float vr = -(va - r * P.tr_D + p * P.tr_H);
    const f2 vav = f2{va, wq};
    const f2 vadv = vav * vav + ua2;                           // (ua^2 + va^2, wq^2 + ua^2)
    const f2 wrvr = f2{wr, vr};
    const f2 wb = wrvr + c.wb0 + vadv * c.wb1;                 // blade-relative inflow (:226, :281)
    const f2 dth = wb - s.vi;                                  // thrust = dth rho coef (:246, :284)
    const f2 thr = dth * (rho * K.coef);
    const f2 dw = wrvr - s.vi;
    const f2 sq = dw * dw + vadv;
    const f2 sr = f2{m_sqrt(sq.x), m_sqrt(sq.y)};
    // inflow ODEs (:247-249, :285-286)
    const f2 dvi = dth * K.inflow_thr - K.inflow * (s.vi * sr);
    const f2 pw = thr * dw;                                    // -(induced power) of each rotor (:250, :292)
    const float power_mr = rho * P.mr_prof * (P.mr_vtip2 + 3.f * vadv.x) - pw.x;
    const float power_tr = -pw.y;
    // flapping (:228-262)
    float CT = dth.x * P.f_mr_ct_k;
    CT = CT > 0.f ? CT : 0.f;
    const float DB1DV = P.f_mr_db_a * CT + m_sqrt(P.f_mr_db_b * CT);
    const bool wake = m_fabs(ua) > P.vtrans;
    const float f1 = wake ? 2.f : 1.f, f3n = wake ? -3.f : -1.f;
    const float KC = P.mr_K1 + P.f_kc_irho * irho;
    // (a_sum, b_sum) = (b1 - lat + KC b0 + DB1DV va f1, b0 + lon - KC b1 - DB1DV ua f3)
    const f2 absum = (B.yx + c.mlat_lon) + B * f2{KC, -KC} + DB1DV * f2{va * f1, ua * f3n};
    // (b0', b1') = (-ITB2_OM a_sum - ITB b_sum - q, ITB2_OM b_sum - ITB a_sum - p)
    const f2 dB = fms_bxn(absum, itb, absum.yx * itb.y + s.pq.yx);
    // forces and moments of the main rotor (:264-269): (X, Y) = -T (b0 - IS, -b1), Z = -T
    const f2 XYn = mul_bxn(BM, thr);                           // BM (T, -T) = -(X_MR, Y_MR)
    const float DL_DA1 = rho * P.mr_DL_DA1_dro;
    // (b0 + lon - K1 b1, lat - b1 - K1 b0)
    const f2 inner = B * K.one_m1 + c.lon_lat - K.k1 * B.yx;
    // (L, M) = H (Y, -X) + DL_DB1 (b1, b0) + DL_DA1 inner
    const f2 LM_MR = XYn.yx * K.mh_h + K.dl_db1 * B.yx + DL_DA1 * inner;

    // ---- fuselage (:302-320)
    const float wa_f0 = wa - s.vi.x;
    const float wa_f = wa_f0 > 0.f ? wa_f0 + (float)kEps : wa_f0;
    const f2 XY_F = (rho * K.hxy) * f2{m_fabs(ua) * ua, m_fabs(va) * va};
    const float awf = m_fabs(wa_f);
    const float Z_F = rho * P.f_hZWW * (awf * wa_f);
    const float zd = rho * P.f_zd * awf * (ua * P.fus_dfw_k + P.fus_dfw_c * wa_f);   // Z_F d_fw
    const float power_fus = -(XY_F.x * ua + XY_F.y * va + Z_F * wa_f);
    const float p_extra = power_fus - P.wt * n2;                 // + climb power (:435, :446-447)

    // ---- horizontal (:322-345) and vertical (:347-361) tail, packed as (HT, VT)
    const float v_dw = m_max(-wa_f0, (float)kEps);
    const float d_dw = ua * m_rcp(v_dw) * P.ht_dw_k - P.ht_dw_c;
    const float eps_ht = (d_dw > 0.f && d_dw < P.mr_R) ? 2.f + d_dw * P.f_m2_R : 0.f;
    const float wa_ht = wa - eps_ht * s.vi.x + P.ht_D * q;
    const float va_vt = va + s.vi.y - P.vt_D * r;
    const f2 X = f2{wa_ht, va_vt};
    const float aua = m_fabs(ua);
    const f2 S2 = X * X + f2{vadv.x, ua2};
    const f2 stall = K.zmax * f2{m_sqrt(S2.x), m_sqrt(S2.y)} * X;
    const f2 lin = (K.zuu * ua + K.zuw * X) * aua;
    const float lim = 0.3f * aua;
    const f2 ZY = (0.5f * rho) * f2{m_fabs(wa_ht) > lim ? stall.x : lin.x, m_fabs(va_vt) > lim ? stall.y : lin.y};

    // ---- totals (:446-459)
    float Fx = XY_F.x - XYn.x - P.wt * s1;
    f2 Fyz = f2{XY_F.y - XYn.y, Z_F - thr.x} + f2{thr.y + ZY.y, ZY.x} + P.wt * B12;
    float Mx = LM_MR.x + XY_F.y * P.fus_H + thr.y * P.tr_H + ZY.y * P.vt_H;
    float My = LM_MR.y + (zd - XY_F.x * P.fus_H) + ZY.x * P.ht_D - thr.x * P.mr_D;
    const float pmain = power_mr + p_extra;
    float Mz = pmain * P.mr_inv_OMEGA - thr.y * P.tr_D - ZY.y * P.vt_D;
    float power = pmain + power_tr;
    // wing (:363-383); the AW109 has none (uniform branch)
    if (P.wn_on) {
        const float wa_w = wa - s.vi.x;
        const float vta2 = ua * ua + wa_w * wa_w;
        const float qq = P.wn_ZUU * ua * ua + P.wn_ZUW * ua * wa_w;
        const float rh = 0.5f * rho;
        const float Z_WN = m_fabs(wa_w) > lim ? rh * P.wn_ZMAX * m_sqrt(vta2) * wa_w : rh * qq;
        const float X_WN = -rh * (float)(1.0 / kPi) * m_rcp(vta2) * qq * qq;
        Fx += X_WN;
        Fyz.y += Z_WN;
        power += m_fabs(X_WN * ua);
    }
    // landing gear (:385-398)
    if constexpr (PRE) {
        if (pre->gear) {
            Fx += pre->Fl0;
            Fyz += pre->Fl12;
            Mx += pre->Ml0;
            My += pre->Ml1;
            Mz += pre->Ml2;
        }
    } else {
        bool ran = false;
        gear_add<ALWAYS>(P, c, s, at, n2, Fx, Fyz, Mx, My, Mz, ran);
    }

    // ---- equations of motion (:448-470)
    // uvw' = F / m - pqr x uvw
    // F / m + r (v, -u) + w (-q, p)
    const f2 duv = fma_nsw_bx(s.pq, s.wz, fma_swn_bx(s.uv, s.rt, f2{Fx, Fyz.x} * P.inv_mass));
    const float dw_ = Fyz.y * P.inv_mass + (q * u - p * v);
    // pqr' = I^-1 (M - pqr x I pqr), I = [[Ixx,0,Ixz],[0,Iyy,0],[Ixz,0,Izz]]: the gyroscopic term is
    // (Ixz pq + (Izz-Iyy) qr, (Ixx-Izz) pr + Ixz (r^2 - p^2), (Iyy-Ixx) pq - Ixz qr) and I^-1 couples
    // p and r only, so (p', r') = J0 Mx + J2 Mz + Cpq pq + Cqr qr, q' = Ji11 My + Cpr pr + Crr (r^2 - p^2)
    // with the coefficients folded on the host (derive: f_gyro)
    const float pq_ = p * q;
    const f2 qrpr = s.pq.yx * r;                               // (q r, p r)
    const float rrpp = r * r - p * p;
    const f2 dpr = K.j0 * Mx + K.j2 * Mz + K.g_pq * pq_ + K.g_qr * qrpr.x;
    const float dq = P.Ji11 * My + P.f_gyro[4] * qrpr.y + P.f_gyro[5] * rrpp;
    k.vi = dvi;
    k.b = dB;
    k.uv = duv;
    k.wz = f2{dw_, n2};
    k.pq = f2{dpr.x, dq};
    k.rt = f2{dpr.y, sqth.y};
    k.pp = f2{phid, psid};
    k.xy = n01;
    if (OBS) {   // the observation at this stage's input state (:471-488)
        obs[0] = (power + P.p_loss) * (float)(1.0 / 550.0);
        obs[1] = ua; obs[2] = va; obs[3] = wa;
        obs[4] = n01.x; obs[5] = n01.y; obs[6] = n2;
        obs[7] = s.pp.x; obs[8] = s.rt.y; obs[9] = s.pp.y;
        obs[10] = p; obs[11] = q; obs[12] = r;
        obs[13] = s.xy.x; obs[14] = s.xy.y; obs[15] = -z; obs[16] = -c.g.zh(z);
    }
}

// RK combinations on the pairs (dynamics.py:166-168): st = hs + h k, acc (+)= (2) k
template <bool FIRST>
HD void rk_stage2(const X16& hs, const X16& k, X16& acc, X16& st, float h) {
#define HG_RK_PAIR(f)                                   \
    acc.f = FIRST ? k.f : acc.f + 2.f * k.f;            \
    st.f = hs.f + k.f * h;
    HG_RK_PAIR(vi) HG_RK_PAIR(b) HG_RK_PAIR(uv) HG_RK_PAIR(wz) HG_RK_PAIR(pq) HG_RK_PAIR(rt) HG_RK_PAIR(pp)
    HG_RK_PAIR(xy)
#undef HG_RK_PAIR
}

HD void rk_update2(X16& hs, const X16& k, const X16& acc, float dt6) {
#define HG_RK_UPD(f) hs.f = hs.f + (acc.f + k.f) * dt6;
    HG_RK_UPD(vi) HG_RK_UPD(b) HG_RK_UPD(uv) HG_RK_UPD(wz) HG_RK_UPD(pq) HG_RK_UPD(rt) HG_RK_UPD(pp) HG_RK_UPD(xy)
#undef HG_RK_UPD
}

HD X16 to_x16(const float* s) {
    X16 x;
    x.vi = f2{s[0], s[1]};
    x.b = f2{s[4], s[5]};
    x.uv = f2{s[6], s[7]};
    x.wz = f2{s[8], s[17]};
    x.pq = f2{s[9], s[10]};
    x.rt = f2{s[11], s[13]};
    x.pp = f2{s[12], s[14]};
    x.xy = f2{s[15], s[16]};
    return x;
}

HD void from_x16(const X16& x, float* s) {   // (s[2], s[3], the rotor azimuths, are not in X16)
    s[0] = x.vi.x; s[1] = x.vi.y;
    s[4] = x.b.x; s[5] = x.b.y;
    s[6] = x.uv.x; s[7] = x.uv.y;
    s[8] = x.wz.x; s[17] = x.wz.y;
    s[9] = x.pq.x; s[10] = x.pq.y;
    s[11] = x.rt.x; s[13] = x.rt.y;
    s[12] = x.pp.x; s[14] = x.pp.y;
    s[15] = x.xy.x; s[16] = x.xy.y;
}

// One RK4 step of the 18-state model (dynamics.py:158-171): hs advanced in place, k4 (the
// reference's state_dots, what the reward reads) in d, the stage-4 observation in obs.
// (sin, cos) of the committed attitude (phi, theta, psi = hs[12], hs[13], hs[14])
HD Att2 att0(const float* hs) {
    Att2 a0;
    a0.a[0] = sincos2(hs[12]);
    a0.a[1] = sincos2(hs[13]);
    a0.a[2] = sincos2(hs[14]);
    return a0;
}

#ifndef HG_PIN_CONSTANTS
#define HG_PIN_CONSTANTS 1
#endif
// One RK4 step in two parts: begin() forms what stage 1 needs that does not read the wind (the
// small-batch kernel runs it while its helper wave steps the wind), finish() the rest.
template <bool LONE, bool PRE1 = false>
struct RK4Step {
    static constexpr bool kGearAlways = LONE && HG_GEAR_ALWAYS_LONE;
    static constexpr bool kMidAll = LONE && PRE1 && HG_MIDALL_HELP;   // PRE1: the helper kernel
    static constexpr bool kAttSel = LONE && !PRE1 && HG_ATT_SEL_LONE;   // (not the helper kernel)
    X16 h;
    Att2 a0;
    StepK K;
    StagePre pre1;
    HD void begin(const Params<float>& P, const StepCtx& c, const float* hs, const Att2& a) {
        begin(P, c, hs, a, step_k<LONE && HG_PIN_CONSTANTS>(P));
    }
    // with the constant pairs built by the caller (the step kernel builds them before its state loads
    // arrive, where a lone wave's pin moves cost nothing: it waits for the loads anyway)
    HD void begin(const Params<float>& P, const StepCtx& c, const float* hs, const Att2& a, const StepK& k) {
        h = to_x16(hs);
        a0 = a;
        K = k;
        if constexpr (PRE1) pre1 = stage_pre<kGearAlways>(P, c, h, a0);
    }
    HD void finish(const Params<float>& P, const StepCtx& c, float* __restrict__ hs, float* __restrict__ d,
                   float* __restrict__ obs);
};

template <bool LONE, bool PRE1>
HD void RK4Step<LONE, PRE1>::finish(const Params<float>& P, const StepCtx& c, float* __restrict__ hs,
                                   float* __restrict__ d, float* __restrict__ obs) {
    X16 k, acc, st;
    stage_f32<false, PRE1, kGearAlways>(P, K, c, h, a0, k, obs, &pre1);
    HG_STAGE_STAMP(5, "v"(k.uv.x), "v"(k.pq.y));
    rk_stage2<true>(h, k, acc, st, P.half_dt);
    stage_f32<false, false, kGearAlways>(P, K, c, st, att_step<kMidAll, kAttSel>(K, a0, h.pp, h.rt.y, st.pp, st.rt.y), k, obs);
    HG_STAGE_STAMP(6, "v"(k.uv.x), "v"(k.pq.y));
    rk_stage2<false>(h, k, acc, st, P.half_dt);
    stage_f32<false, false, kGearAlways>(P, K, c, st, att_step<kMidAll, kAttSel>(K, a0, h.pp, h.rt.y, st.pp, st.rt.y), k, obs);
    HG_STAGE_STAMP(7, "v"(k.uv.x), "v"(k.pq.y));
    rk_stage2<false>(h, k, acc, st, P.dt);
    stage_f32<true, false, kGearAlways>(P, K, c, st, att_step<kMidAll, kAttSel>(K, a0, h.pp, h.rt.y, st.pp, st.rt.y), k, obs);
    rk_update2(h, k, acc, P.dt6);
    from_x16(h, hs);
    // (the rotor azimuths hs[2], hs[3] are not stepped here: see az_advance)
    from_x16(k, d);
    d[2] = P.mr_OMEGA;
    d[3] = P.tr_OMEGA;
}

template <bool LONE>
HD void rk4_step_f32(const Params<float>& P, const StepCtx& c, float* __restrict__ hs, float* __restrict__ d,
                     float* __restrict__ obs, const Att2& a0) {
    RK4Step<LONE> rk;
    rk.begin(P, c, hs, a0);
    rk.finish(P, c, hs, d, obs);
}

template <bool LONE>
HD void rk4_step_f32(const Params<float>& P, const StepCtx& c, float* __restrict__ hs, float* __restrict__ d,
                     float* __restrict__ obs) {
    rk4_step_f32<LONE>(P, c, hs, d, obs, att0(hs));
}

}  // namespace hg
