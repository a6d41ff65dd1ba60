// physics.h — Heffley–Mnich minimum-complexity helicopter model + Dryden turbulence, written once
// as __host__ __device__ templates: instantiated with float in the gfx950 step kernel
// (heligym_amd.hip) and with double in the host trim (trim.h).
//
// Each function cites the reference code it re-states (paths relative to
// /root/reference/heligym/envs/).  Quirks of the reference are kept on purpose and marked QUIRK.
#pragma once

#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#define HD __host__ __device__ __forceinline__

namespace hg {

// ------------------------------------------------------------------------------------------
// math helpers: one overload per precision.  fp32 device versions use the hardware
// transcendental units (v_log_f32 / v_exp_f32 / v_sqrt_f32).
HD float m_sqrt(float x) { return sqrtf(x); }
#if defined(__HIP_DEVICE_COMPILE__) && !defined(HG_SQRT_LIBM)
// fp64 on the device (the re-trim kernels): v_rsq_f64 and a Goldschmidt iteration with a final fused
// correction (within an ulp of the correctly rounded root for the model's positive normal
// arguments), instead of the library sqrt's scaling for denormals and its special-case selects;
// 0 -> 0 and a negative or NaN argument -> NaN, as the library's.
HD double m_sqrt(double x) {
    const double r = __builtin_amdgcn_rsq(x);
    double g = x * r, h = 0.5 * r;
    const double e = fma(-g, h, 0.5);
    g = fma(g, e, g);
    h = fma(h, e, h);
    const double d = fma(-g, g, x);
    g = fma(d, h, g);
    return x == 0.0 ? x : g;
}
#else
HD double m_sqrt(double x) { return sqrt(x); }
#endif
HD float m_fabs(float x) { return fabsf(x); }
HD double m_fabs(double x) { return fabs(x); }
HD float m_floor(float x) { return floorf(x); }
HD double m_floor(double x) { return floor(x); }
HD float m_fmod(float x, float y) { return fmodf(x, y); }
HD double m_fmod(double x, double y) { return fmod(x, y); }
// fp32 sin/cos for the attitude angles (|x| <= ~4 rad: wrapped euler angles plus one RK stage
// increment): Cody-Waite reduction by pi/2 (3-part constant) and minimax polynomials on
// [-pi/4, pi/4]; ~1 ulp, ~25 VALU ops for both, no Payne-Hanek slow path (libm sincosf spills a
// 36-byte scratch table for it).  Larger |x| keeps working with degrading absolute accuracy.
HD void m_sincos(float x, float* s, float* c) {
    const float k = rintf(x * 0.636619772367581343f);
    float r = fmaf(k, -1.57079637050628662109375f, x);
    r = fmaf(k, 4.37113900018624283e-8f, r);
    r = fmaf(k, 1.71512451e-15f, r);
    const float r2 = r * r;
    // sin(r) ~ r + r^3 (s1 + r^2 (s2 + r^2 s3)), cos(r) ~ 1 + r^2 (c1 + r^2 (c2 + r^2 (c3 + r^2 c4)))
    float sp = fmaf(r2, -1.9515295891e-4f, 8.3321608736e-3f);
    sp = fmaf(r2, sp, -1.6666654611e-1f);
    const float sr = fmaf(r * r2, sp, r);
    float cp = fmaf(r2, 2.443315711809948e-5f, -1.388731625493765e-3f);
    cp = fmaf(r2, cp, 4.166664568298827e-2f);
    cp = fmaf(r2, cp, -0.5f);
    const float cr = fmaf(r2, cp, 1.0f);
    const int q = (int)k;
    const bool swap = q & 1;
    const float ss = swap ? cr : sr, cc = swap ? sr : cr;
    *s = (q & 2) ? -ss : ss;
    *c = ((q + 1) & 2) ? -cc : cc;
}
#if defined(__HIP_DEVICE_COMPILE__)
// fp64 on the device (the re-trim kernel, retrim.hip): sin and cos from one reduction -- Cody-Waite
// by pi/2 with fused multiply-adds (3-part constant, exact enough for |x| < 1e5; trim attitudes are
// below pi) and the fdlibm kernel polynomials __kernel_sin / __kernel_cos on [-pi/4, pi/4] (about
// 1 ulp, like the host's libm, which the trims do not reproduce bitwise either) -- instead of two
// library calls with separate reductions and a Payne-Hanek path each.
HD void m_sincos(double x, double* s, double* c) {
    const double k = rint(x * 0.63661977236758134308);
    double r = fma(k, -1.57079632679489655800e+00, x);
    r = fma(k, -6.12323399573676603587e-17, r);
    r = fma(k, 1.49738490485916983e-33, r);
    const double z = r * r, v = z * r;
    const double sp = fma(z, fma(z, fma(z, fma(z, 1.58969099521155010221e-10, -2.50507602534068634195e-08),
                                        2.75573137070700676789e-06), -1.98412698298579493134e-04),
                          8.33333333332248946124e-03);
    const double sr = fma(v, fma(z, sp, -1.66666666666666324348e-01), r);
    const double cp = z * fma(z, fma(z, fma(z, fma(z, fma(z, -1.13596475577881948265e-11, 2.08757232129817482790e-09),
                                                  -2.75573143513906633035e-07), 2.48015872894767294178e-05),
                                     -1.38888888888741095749e-03), 4.16666666666666019037e-02);
    const double hz = 0.5 * z, w = 1.0 - hz;
    const double cr = w + (((1.0 - w) - hz) + z * cp);
    const int q = (int)k;
    const double ss = (q & 1) ? cr : sr, cc = (q & 1) ? sr : cr;
    *s = (q & 2) ? -ss : ss;
    *c = ((q + 1) & 2) ? -cc : cc;
}
#else
HD void m_sincos(double x, double* s, double* c) { *s = sin(x); *c = cos(x); }
#endif
// x / c for a model constant c with its reciprocal ic = 1 / c: on the device one product and a
// fused-multiply-add correction (the quotient to within an ulp, no division sequence); the host
// divides.
HD double m_div_c(double x, double c, double ic) {
#if defined(__HIP_DEVICE_COMPILE__)
    const double q = x * ic;
    return fma(fma(-q, c, x), ic, q);
#else
    (void)ic;
    return x / c;
#endif
}

// sin/cos of the three attitude angles (kinematic.py:4-5,21-22).
template <typename R>
struct Attitude {
    R s[3], c[3];
};

template <typename R>
HD Attitude<R> attitude(const R* eul) {
    Attitude<R> a;
#pragma unroll
    for (int j = 0; j < 3; ++j) m_sincos(eul[j], &a.s[j], &a.c[j]);
    return a;
}

// Attitude of a RK stage from the committed attitude: sin/cos(e + d) by the angle-addition
// formulas with short Taylor series for the stage increment d.  For |d| <= 0.05 rad (attitude
// rates below 5 rad/s at dt 0.01, 2.5 rad/s at dt 0.02) sin d = d - d^3/6 and
// cos d = 1 - d^2/2 + d^4/24 are within 2.7e-9 and 2.2e-11; a lane with a larger increment (a
// tumbling, diverging env) takes the full sincos.
template <typename R>
HD Attitude<R> attitude_step(const Attitude<R>& a0, const R* eul0, const R* eul) {
    Attitude<R> a;
    bool big = false;
    R sd[3], cd[3];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        const R d = eul[j] - eul0[j];
        const R d2 = d * d;
        big = big || !(m_fabs(d) <= (R)0.05);
        sd[j] = d + (d * d2) * (R)(-1.0 / 6.0);
        cd[j] = (R)1 + d2 * ((R)-0.5 + d2 * (R)(1.0 / 24.0));
    }
    if (big) return attitude(eul);
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        a.s[j] = a0.s[j] * cd[j] + a0.c[j] * sd[j];
        a.c[j] = a0.c[j] * cd[j] - a0.s[j] * sd[j];
    }
    return a;
}
// x^e for x > 0 (ISA density ratio, Dryden scale lengths)
HD float m_pow(float x, float e) { return exp2f(e * log2f(x)); }
HD double m_pow(double x, double e) { return pow(x, e); }
HD float m_log2(float x) { return log2f(x); }
HD double m_log2(double x) { return log2(x); }
HD float m_exp2(float x) { return exp2f(x); }
HD double m_exp2(double x) { return exp2(x); }
// Reciprocal: the hardware v_rcp_f32 (1 ulp) on the device instead of a full IEEE division.
HD float m_rcp(float x) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_rcpf(x);
#else
    return 1.0f / x;
#endif
}
#if defined(__HIP_DEVICE_COMPILE__)
// fp64 on the device (the re-trim kernel): v_rcp_f64 and two fused Newton steps (within an ulp for
// finite non-zero x; the trim model's reciprocals are of cos(theta), 1 + og^2, the fuselage and tail
// downwash speeds)
HD double m_rcp(double x) {
    double r = __builtin_amdgcn_rcp(x);
    r = fma(r, fma(-x, r, 1.0), r);
    return fma(r, fma(-x, r, 1.0), r);
}
#else
HD double m_rcp(double x) { return 1.0 / x; }
#endif
// True when any lane of the wave has `c` (a uniform skip for rarely taken, costly branches).
HD bool wave_any(bool c) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __any(c);
#else
    return c;
#endif
}
template <typename R> HD R m_sign(R x) { return (R)((x > (R)0) - (x < (R)0)); }
template <typename R> HD R m_max(R a, R b) { return a > b ? a : b; }

constexpr double kPi = 3.14159265358979323846;
constexpr double kEps = 1e-4;                  // helicopter_dynamics.py:15, wind_dynamics.py:10
constexpr double kSqrt3 = 1.7320508075688772;  // wind_dynamics.py:12
constexpr double kTwoDPi = 0.6366197723675814; // wind_dynamics.py:13

// ------------------------------------------------------------------------------------------
// Derived model constants (helicopter_dynamics.py:107-154, wind_dynamics.py:21-37,
// helicopter.py:63-68).  Computed once on the host in double (model.cpp) and cast to R.
// Passed to the kernel by value, so every constant is a scalar (SGPR) operand.
template <typename R>
struct Params {
    R dt, half_dt, dt6;
    // control mixing u = c0 + c1 * action (helicopter_dynamics.py:414-422)
    R coll0, coll1, lon0, lon1, lat0, lat1, ped0, ped1;
    // ISA atmosphere rho = RO_SEA * (1 - LAPSE/T0 * alt)^rho_exp (:160-165)
    R lapse_t0, ro_sea, rho_exp;
    R wt, inv_mass, p_loss, vtrans, wl_cg_ft;
    // main rotor
    R mr_H, mr_D, mr_IS, mr_K1, mr_R, mr_OMEGA, mr_inv_OMEGA, mr_VTIP, mr_inv_VTIP;
    R mr_tw75, mr_tw50, mr_two3_vtip, mr_gam_dro, mr_kc_num, mr_DL_DB1, mr_DL_DA1_dro, mr_coef;
    R mr_inflow, mr_inv_thr_den, mr_inv_ct_den, mr_prof, mr_vtip2, mr_2_vtip, mr_8_asig;
    R mr_inv_gam_dro, mr_inv_R;
    // tail rotor
    R tr_H, tr_D, tr_OMEGA, tr_VTIP, tr_inv_VTIP, tr_tw75, tr_tw50, tr_two3_vtip, tr_coef;
    R tr_inflow, tr_inv_thr_den;
    // fuselage
    R fus_H, fus_XUU, fus_YVV, fus_ZWW, fus_COR, fus_dfw_k, fus_dfw_c;
    // horizontal / vertical tail, wing
    R ht_D, ht_ZUU, ht_ZUW, ht_ZMAX, ht_dw_k, ht_dw_c;
    R vt_H, vt_D, vt_YUU, vt_YUV, vt_YMAX;
    R wn_ZUU, wn_ZUW, wn_ZMAX;
    int32_t wn_on;
    // landing gear
    R lg_K, lg_C, lg_loc[3][3], lg_reach;   // lg_reach: max |r_g| plus a rounding margin
    // inertia: I = [[Ixx,0,Ixz],[0,Iyy,0],[Ixz,0,Izz]] (Ixz = -IXZ), and its inverse
    R Ixx, Iyy, Izz, Ixz, Ji00, Ji02, Ji11, Ji20, Ji22;
    // terrain (helicopter_dynamics.py:167-195)
    R hm_sx, hm_sy, hm_cx, hm_cy, ns_half, ew_half;
    int32_t hm_rows, hm_cols;
    // Dryden wind (wind_dynamics.py:21-83)
    R wm[3], wind_dir_cos, wind_dir_sin, w20, sigma_low, turb_level, eta_norm;
    R tep_row[13];   // TEP table interpolated at turb_level, per altitude key (tep_row_values)
    // folded products of the constants above for the packed fp32 step (stage_f32.h)
    R f_kc_irho, f_og_irho;              // KC = K1 + f_kc_irho / rho; og = f_og_irho / rho (:214-220)
    R f_mr_inflow_thr, f_tr_inflow_thr;  // inflow * coef / (2 pi R^2): the inflow ODE's thrust term per (wb - vi)
    R f_mr_ct_k;                         // CT = max((wb - vi) * f_mr_ct_k, 0)
    R f_mr_db_a, f_mr_db_b;              // DB1DV = f_mr_db_a CT + sqrt(f_mr_db_b CT)
    R f_hXUU, f_hYVV, f_hZWW, f_zd;      // 0.5 XUU, 0.5 YVV, 0.5 ZWW; -0.5 ZWW COR (fuselage downwash moment)
    R f_m2_R;                            // -2 / R_MR (H-tail downwash factor)
    R f_rho_lz;                          // rho_exp * lapse / T0 (d ln rho / dz = f_rho_lz / (1 + lapse/T0 z))
    R f_gyro[6];                         // I^-1 (pqr x I pqr) coefficients: p', r' of pq, qr; q' of pr, r^2 - p^2
    R f_dpsi_mr, f_dpsi_tr;              // dt * Omega (rotor azimuth per step; runtime: depends on dt)
    // task (helicopter.py:63-68, helicopter_with_tasks.py)
    R n_t, n_t2, inv_n_x, inv_n_v, inv_n_a, tgt_n[3], vel_tgt_n, dwn_tgt_n;
    R fail_zdot, fail_ang;
    int32_t task, time_up_steps, success_steps, autoreset, reset_retrim;
    int32_t autoreset_next, max_episode_steps;   // next-step auto-reset; TimeLimit (INT32_MAX: off)
    int32_t env_templates;                       // per-env reset templates set (hg_set_reset_templates)
};

// Reset template: trimmed heli state, zero turbulence state, carry and observation.
template <typename R>
struct Template {
    R heli[18];
    R carry[4];
    R obs[17];
};

template <typename R>
struct Controls {
    R coll, lon, lat, ped;
    // the control-only parts of the rotors' blade-relative inflow (:226, :281), fixed over a step
    R mr_wb0, mr_wb1, tr_vb0, tr_vb1;
};

// helicopter_dynamics.py:414-422 (no clipping of the action, like the reference).
template <typename R>
HD Controls<R> controls(const Params<R>& P, R a0, R a1, R a2, R a3) {
    Controls<R> u;
    u.coll = P.coll0 + P.coll1 * a0;
    u.lon = P.lon0 + P.lon1 * a1;
    u.lat = P.lat0 + P.lat1 * a2;
    u.ped = P.ped0 + P.ped1 * a3;
    u.mr_wb0 = P.mr_two3_vtip * (u.coll + P.mr_tw75);
    u.mr_wb1 = P.mr_inv_VTIP * (u.coll + P.mr_tw50);
    u.tr_vb0 = P.tr_two3_vtip * (u.ped + P.tr_tw75);
    u.tr_vb1 = P.tr_inv_VTIP * (u.ped + P.tr_tw50);
    return u;
}

// utils.py:3-4 — floor-mod wrap to [-pi, pi).
template <typename R>
HD R pi_bound(R x) {
    const R twopi = (R)(2 * kPi);
    R r = x + (R)kPi;
    r = r - twopi * m_floor(r * (R)(1.0 / (2 * kPi)));   // floor-mod, one step
    r = r < (R)0 ? r + twopi : (r >= twopi ? r - twopi : r);
    return r - (R)kPi;
}

// helicopter_dynamics.py:167-195.  Three-point interpolated ground height at the COMMITTED (x, y).
// The reference's scheme is discontinuous across cell edges, and the map centre (x = y = 0, where
// every default trim starts) sits exactly on one; so the cell index must be decided exactly as the
// fp64 reference decides it.  With an integer centre c, floor(x*s + c) = c + floor(x*s) exactly,
// so the index comes from floor(x*s) (its sign is exact) instead of an fp32 x*s + c that rounds
// to c for |x| below ~1e-4 ft.  Indices are clamped as integers as well, so a non-finite position
// can never address outside the map.
template <typename R>
HD void map_coord(R t, int c, int hi, int* idx, R* frac) {
    // x_loc = t + c clamped to [0, hi] (hi = rows - 1) -> (index, fraction) with x_loc = index + fraction
    if (!(t > (R)(-c))) {            // x_loc <= 0 (and NaN) -> 0
        *idx = 0;
        *frac = (R)0;
    } else if (t >= (R)(hi - c)) {   // x_loc >= hi -> hi
        *idx = hi;
        *frac = (R)0;
    } else {
        const R fl = m_floor(t);
        *idx = (int)fl + c;
        *frac = t - fl;
    }
}

// Terrain texel = float2 {hi, lo} with hi + lo = the fp64 height (ft): the contact spring
// K * (pos_z + h) and the ground altitude need h to better than one fp32 ulp of ~1500 ft.
template <typename R>
struct Ground {
    R hi, lo, delta;   // h = (hi + lo) + delta; hi = the texel read before the edge decrement
    HD R h() const { return (hi + lo) + delta; }
    // z + h with the large cancellation done first (exact in fp32: Sterbenz lemma)
    HD R zh(R z) const { return ((z + hi) + lo) + delta; }
};

// The three texels and fractions for a position (split so the kernel can prefetch texels).
template <typename R>
struct GroundCell {
    int mid, north, east;   // texel indices: mid read before the edge decrement (:188), then (:191-192)
    R fx, fy;               // fractions, with the post-decrement index (:194)
};

template <typename R>
HD GroundCell<R> ground_cell(const Params<R>& P, R x, R y) {
    const int rows = P.hm_rows, cols = P.hm_cols;
    int xi, yi;
    R fx, fy;
    map_coord(x * P.hm_sx, rows / 2, rows - 1, &xi, &fx);
    map_coord(y * P.hm_sy, cols / 2, rows - 1, &yi, &fy);   // QUIRK: y clamps to shape[0] (:182-183)
    GroundCell<R> c;
    c.mid = yi * cols + xi;
    if (xi == rows - 1) { xi = rows - 2; fx += (R)1; }   // (:189-190) edge decrement
    if (yi == cols - 1) { yi = cols - 2; fy += (R)1; }
    c.north = yi * cols + xi + 1;
    c.east = (yi + 1) * cols + xi;
    c.fx = fx;
    c.fy = fy;
    return c;
}

struct GroundTexels {
    float2 m, n, e;
};

template <typename R>
HD GroundTexels ground_fetch(const float2* __restrict__ hmap, const GroundCell<R>& c) {
    return GroundTexels{hmap[c.mid], hmap[c.north], hmap[c.east]};
}

template <typename R>
HD Ground<R> ground_combine(const GroundTexels& t, const GroundCell<R>& c) {
    Ground<R> g;
    g.hi = (R)t.m.x;
    g.lo = (R)t.m.y;
    const R dn = ((R)t.n.x - (R)t.m.x) + ((R)t.n.y - (R)t.m.y);
    const R de = ((R)t.e.x - (R)t.m.x) + ((R)t.e.y - (R)t.m.y);
    g.delta = dn * c.fx + de * c.fy;   // (:194)
    return g;
}

template <typename R>
HD Ground<R> ground_height(const Params<R>& P, const float2* __restrict__ hmap, R x, R y) {
    const GroundCell<R> c = ground_cell(P, x, y);
    return ground_combine<R>(ground_fetch(hmap, c), c);
}

// ------------------------------------------------------------------------------------------
// Dryden turbulence (wind_dynamics.py:54-125)

template <typename R>
struct WindPar {
    R a_u, a_v, b_v, a_w, b_w;   // 1/t_u, 1/t_v, 1/(4 t_v^2), 1/t_w, 1/(4 t_w^2)
    R K_u, K_v, K_w;             // sigma * sqrt(2/pi * t)
    R cos_az, sin_az;
};

// lookup.py:146-183 (get_value_2D) on the 7x12 TEP table: row key = turbulence level, column
// key = ground altitude; clamped linear interpolation, no extrapolation.
// MIL-HDBK-1797 turbulence exceedance table as the reference fills its LookUpTable(7,12)
// (wind_dynamics.py:29-37): row 0 = altitude keys, column 0 = level keys.
#define HG_TEP_TABLE                                                                              \
    {{0.f, 500.f, 1750.f, 3750.f, 7500.f, 15000.f, 25000.f, 35000.f, 45000.f, 55000.f, 65000.f,   \
      75000.f, 80000.f},                                                                          \
     {1.f, 3.2f, 2.2f, 1.5f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f},                        \
     {2.f, 4.2f, 3.6f, 3.3f, 1.6f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f},                       \
     {3.f, 6.6f, 6.9f, 7.4f, 6.7f, 4.6f, 2.7f, 0.4f, 0.f, 0.f, 0.f, 0.f, 0.f},                    \
     {4.f, 8.6f, 9.6f, 10.6f, 10.1f, 8.0f, 6.6f, 5.0f, 4.2f, 2.7f, 0.f, 0.f, 0.f},                \
     {5.f, 11.8f, 13.0f, 16.0f, 15.1f, 11.6f, 9.7f, 8.1f, 8.2f, 7.9f, 4.9f, 3.2f, 2.1f},          \
     {6.f, 15.6f, 17.6f, 23.0f, 23.6f, 22.1f, 20.0f, 16.0f, 15.1f, 12.1f, 7.9f, 6.2f, 5.1f},      \
     {7.f, 18.7f, 21.5f, 28.4f, 30.2f, 30.7f, 31.0f, 25.2f, 23.1f, 17.5f, 10.7f, 8.4f, 7.2f}}

constexpr float kTep[8][13] = HG_TEP_TABLE;

// lookup.py:146-183 (get_value_2D) on the 7x12 TEP table: row key = turbulence level, column
// key = ground altitude; clamped linear interpolation, no extrapolation.  The reference caches
// the last bracket index, which only changes where its search starts, not the bracket found.
// Split in two: the row interpolation depends only on the (per-model) turbulence level and is
// done once on the host into Params::tep_row; the per-env column bracket is found by comparing
// against the literal altitude keys (no dependent table loads on the device).
template <typename R>
void tep_row_values(R rowKey, R out[13]) {
    int r = 2;
    for (int k = 0; k < 5; ++k) r += (r < 7 && (R)kTep[r][0] < rowKey) ? 1 : 0;
    const R r0 = (R)kTep[r - 1][0], r1 = (R)kTep[r][0];
    R rF = (rowKey - r0) / (r1 - r0);
    rF = rF > (R)1 ? (R)1 : (rF < (R)0 ? (R)0 : rF);
    for (int c = 0; c < 13; ++c) {
        const R a0 = (R)kTep[r - 1][c], a1 = (R)kTep[r][c];
        out[c] = rF * (a1 - a0) + a0;
    }
}

template <typename R>
HD R tep_lookup(const R* __restrict__ row, R colKey) {
    // bracket c = 2 + #{j in [2, 12): key_j < colKey} (keys increase); k0/k1 and the row values at
    // c - 1 and c by compare-and-select
    R k0 = (R)kTep[0][1], k1 = (R)kTep[0][2], v0 = row[1], v1 = row[2];
#pragma unroll
    for (int j = 2; j < 12; ++j) {
        const bool up = (R)kTep[0][j] < colKey;
        k0 = up ? (R)kTep[0][j] : k0;
        k1 = up ? (R)kTep[0][j + 1] : k1;
        v0 = up ? row[j] : v0;
        v1 = up ? row[j + 1] : v1;
    }
    R cF = (colKey - k0) / (k1 - k0);
    cF = cF > (R)1 ? (R)1 : (cF < (R)0 ? (R)0 : cF);
    return v0 + cF * (v1 - v0);
}

// wind_dynamics.py:54-83 (_calc_params) folded with the stage-invariant part of :92-99, 112-118.
// UNIFORM (the lone-wave kernels): the low-altitude form for every lane and the others in a
// wave-uniform branch taken only when some lane is above 1000 ft -- the same values, one block
// instead of a divergent if / else around the common case (65 536 envs: -0.07 us; the bulk variant
// keeps the if / else)
template <typename R, bool UNIFORM = false>
HD WindPar<R> wind_params(const Params<R>& P, const R carry[4]) {
    const R vx = carry[0] + P.wm[0], vy = carry[1] + P.wm[1], vz = carry[2] + P.wm[2];
    const R vel = m_sqrt(vx * vx + vy * vy + vz * vz);
    const R h = carry[3];
    R Lu, Lv, Lw, s_u, s_v, s_w, ca, sa;
    auto low_alt = [&]() {                    // low altitude
        const R hl = m_max(h, (R)10);
        const R lb = m_log2((R)0.177 + (R)0.000823 * hl);
        Lu = hl * m_exp2((R)-1.2 * lb);
        Lv = (R)0.5 * Lu;
        Lw = (R)0.5 * hl;
        s_w = P.sigma_low;
        s_u = s_w * m_exp2((R)-0.4 * lb);
        s_v = s_u;
        ca = P.wind_dir_cos;
        sa = P.wind_dir_sin;
    };
    auto mid_high_alt = [&]() {
        R ax, ay;
        if (h >= (R)2000) {                   // high altitude
            Lu = (R)1750; Lv = (R)875; Lw = (R)875;
            s_u = tep_lookup(P.tep_row, h);
            ax = vx; ay = vy;
        } else {                              // medium: blend of the two (QUIRK: Lw = Lu, :76)
            const R r = (h - (R)1000) * (R)0.001;
            Lu = (R)1000 + r * (R)750;
            Lv = (R)0.5 * Lu;
            Lw = Lu;
            s_u = P.sigma_low + r * (tep_lookup(P.tep_row, h) - P.sigma_low);
            ax = vx * r + P.wm[0] * ((R)1 - r);
            ay = vy * r + P.wm[1] * ((R)1 - r);
        }
        s_v = s_u; s_w = s_u;
        // cos/sin of atan2(ay, ax) without the transcendental (atan2(0,0) = 0)
        const R hyp = m_sqrt(ax * ax + ay * ay);
        const bool z = !(hyp > (R)0);
        const R ih = z ? (R)0 : m_rcp(hyp);
        ca = z ? (R)1 : ax * ih;
        sa = z ? (R)0 : ay * ih;
    };
    const bool low = h <= (R)1000;   // (a NaN altitude: not low, as the reference's if / else)
    if constexpr (UNIFORM) {
        low_alt();
        if (wave_any(!low))
            if (!low) mid_high_alt();
    } else {
        if (low) low_alt();
        else mid_high_alt();
    }
    const R iv = m_rcp(vel + (R)kEps);
    const R t_u = Lu * iv, t_v = Lv * iv, t_w = Lw * iv;
    WindPar<R> w;
    w.a_u = m_rcp(t_u);
    w.a_v = m_rcp(t_v);
    w.b_v = (R)0.25 * w.a_v * w.a_v;
    w.a_w = m_rcp(t_w);
    w.b_w = (R)0.25 * w.a_w * w.a_w;
    w.K_u = s_u * m_sqrt((R)kTwoDPi * t_u);
    w.K_v = s_v * m_sqrt((R)kTwoDPi * t_v);
    w.K_w = s_w * m_sqrt((R)kTwoDPi * t_w);
    w.cos_az = ca;
    w.sin_az = sa;
    return w;
}

// wind_dynamics.py:101-109
template <typename R>
HD void wind_f(const WindPar<R>& w, const R eta[3], const R s[5], R d[5]) {
    d[0] = w.a_u * (eta[0] - s[0]);
    d[1] = w.b_v * (eta[1] - s[2]) - w.a_v * s[1];
    d[2] = s[1];
    d[3] = w.b_w * (eta[2] - s[4]) - w.a_w * s[3];
    d[4] = s[3];
}

// WindDynamics.step (dynamics.py:158-171 + wind_dynamics.py:85-125).  QUIRK: the
// derivative object is aliased across the RK stages, so the update is s += dt * k4; the stage
// inputs are still formed from k1..k3.  Wind output from the stage-4 input state.
template <typename R>
HD void wind_step(const Params<R>& P, R s[5], const R carry[4], const R eta[3],
                  R W[3]) {
    const WindPar<R> w = wind_params(P, carry);
    R k[5], st[5];
    wind_f(w, eta, s, k);
#pragma unroll
    for (int i = 0; i < 5; ++i) st[i] = s[i] + k[i] * P.half_dt;
    wind_f(w, eta, st, k);
#pragma unroll
    for (int i = 0; i < 5; ++i) st[i] = s[i] + k[i] * P.half_dt;
    wind_f(w, eta, st, k);
#pragma unroll
    for (int i = 0; i < 5; ++i) st[i] = s[i] + k[i] * P.dt;
    wind_f(w, eta, st, k);
    const R ut = w.K_u * st[0];
    const R vt = w.K_v * (st[2] + (R)(2 * kSqrt3) * st[1]);
    const R wt = w.K_w * (st[4] + (R)(2 * kSqrt3) * st[3]);
    W[0] = P.wm[0] + (w.cos_az * ut - w.sin_az * vt);
    W[1] = P.wm[1] + (w.sin_az * ut + w.cos_az * vt);
    W[2] = P.wm[2] + wt;
#pragma unroll
    for (int i = 0; i < 5; ++i) s[i] = s[i] + P.dt * k[i];
}

// ------------------------------------------------------------------------------------------
// HelicopterDynamics.dynamics (helicopter_dynamics.py:400-489), in parts: the kinematics every
// force model uses (frame), two groups of component models (main_loads: main rotor + fuselage;
// tail_loads: tail rotor, tails, wing, landing gear), and the equations of motion (eom) that add
// the two groups.  dynamics() chains them for one lane; the two-wave step kernel evaluates the two
// groups on different waves.  Same arithmetic either way, so the results are bitwise identical.
// s: [vi_mr vi_tr psi_mr psi_tr b0 b1 u v w p q r phi theta psi x y z]; W: wind NED; gc: ground
// height under the COMMITTED position (F6).

// Stage-input kinematics (:423-445, kinematic.py:3-29, ISA density :160-165).
// A pair of R as a vector (packed fp32 on the device for R = float).
template <typename R>
struct V2T {
    typedef R type __attribute__((ext_vector_type(2)));
};
template <typename R>
using V2 = typename V2T<R>::type;

template <typename R>
struct Frame {
    R B02, B12, B22;     // third column of the earth->body DCM (gravity, landing gear)
    R phid, thd, psid;   // euler rates
    R n0, n1, n2;        // NED velocity B^T uvw
    R ua, va, wa;        // air-relative body velocity uvw - B W
    R rho, irho;         // density at -z and its reciprocal
    R zh;                // z + h under the committed position
};

// ISA density at the altitude -z (helicopter_dynamics.py:160-165)
template <typename R>
HD R atmosphere_rho(const Params<R>& P, R z) {
    return P.ro_sea * m_pow((R)1 + P.lapse_t0 * z, P.rho_exp);
}

template <typename R>
HD Frame<R> frame(const Params<R>& P, const R* __restrict__ s, const R W[3], const Ground<R>& gc,
                  const Attitude<R>& att, const R* rho_irho = nullptr) {
    const R uu = s[6], vv = s[7], ww = s[8], p = s[9], q = s[10], r = s[11];
    const R s0 = att.s[0], c0 = att.c[0], s1 = att.s[1], c1 = att.c[1], s2 = att.s[2], c2 = att.c[2];
    Frame<R> f;
    // euler rates T(phi, theta) pqr (kinematic.py:20-29)
    const R ic1 = m_rcp(c1);
    const R t1 = s1 * ic1;
    if constexpr (sizeof(R) == sizeof(double)) {
        // fp64 (the trims): the reference's form, B = Rx Ry Rz formed as a matrix (kinematic.py:3-17)
        // and applied to uvw and W (:428-431).  The trim's Newton path is sensitive to the operation
        // order at ill-conditioned points, so it follows the reference's as closely as possible.
        const R B00 = c1 * c2, B01 = c1 * s2, B02 = -s1;
        const R s0s1 = s0 * s1, c0s1 = c0 * s1;
        const R B10 = s0s1 * c2 - c0 * s2, B11 = s0s1 * s2 + c0 * c2, B12 = s0 * c1;
        const R B20 = c0s1 * c2 + s0 * s2, B21 = c0s1 * s2 - s0 * c2, B22 = c0 * c1;
        f.B02 = B02;
        f.B12 = B12;
        f.B22 = B22;
        f.phid = p + (s0 * t1) * q + (c0 * t1) * r;
        f.thd = c0 * q - s0 * r;
        f.psid = (s0 * ic1) * q + (c0 * ic1) * r;
        f.n0 = B00 * uu + B10 * vv + B20 * ww;
        f.n1 = B01 * uu + B11 * vv + B21 * ww;
        f.n2 = B02 * uu + B12 * vv + B22 * ww;
        f.ua = uu - (B00 * W[0] + B01 * W[1] + B02 * W[2]);
        f.va = vv - (B10 * W[0] + B11 * W[1] + B12 * W[2]);
        f.wa = ww - (B20 * W[0] + B21 * W[1] + B22 * W[2]);
    } else {
        // fp32 (the step): B applied as its three plane rotations on pairs of components (packed
        // fp32) rather than formed; only its third column (gravity, landing gear) is needed.
        const V2<R> b12_22 = c1 * V2<R>{s0, c0};
        f.B02 = -s1;
        f.B12 = b12_22.x;
        f.B22 = b12_22.y;
        const R sq_cr = s0 * q + c0 * r;
        f.phid = p + t1 * sq_cr;
        f.thd = c0 * q - s0 * r;
        f.psid = ic1 * sq_cr;
        // ned = B^T uvw = Rz^T Ry^T Rx^T uvw
        const V2<R> yz1 = vv * V2<R>{c0, s0} + ww * V2<R>{-s0, c0};        // Rx^T: (y, z)
        const V2<R> xz2 = uu * V2<R>{c1, -s1} + yz1.y * V2<R>{s1, c1};     // Ry^T: (x, z)
        const V2<R> n01 = xz2.x * V2<R>{c2, s2} + yz1.x * V2<R>{-s2, c2};  // Rz^T: (x, y)
        f.n0 = n01.x;
        f.n1 = n01.y;
        f.n2 = xz2.y;
        // uvw_air = uvw - B W = uvw - Rx Ry Rz W
        const V2<R> ab = W[0] * V2<R>{c2, -s2} + W[1] * V2<R>{s2, c2};     // Rz W: (x, y)
        const V2<R> xg = ab.x * V2<R>{c1, s1} + W[2] * V2<R>{-s1, c1};     // Ry: (x, z)
        const V2<R> yz = xg.y * V2<R>{s0, c0} + ab.y * V2<R>{c0, -s0};     // Rx: (y, z)
        f.ua = uu - xg.x;
        f.va = vv - yz.x;
        f.wa = ww - yz.y;
    }
    if (rho_irho) {   // the trims: the altitude is fixed, so the density is evaluated once per trim
        f.rho = rho_irho[0];
        f.irho = rho_irho[1];
    } else {
        f.rho = atmosphere_rho(P, s[17]);
        f.irho = m_rcp(f.rho);
    }
    // z + h with the large cancellation first (Ground::zh): the stiff gear spring K * (pos_z + h)
    // keeps its precision near the ground
    f.zh = gc.zh(s[17]);
    return f;
}

// Forces, moments and power of a group of components, and the derivatives of the states the group
// owns (main: vi_mr, b0, b1; tail: vi_tr).
template <typename R>
struct Loads {
    R d[3];
    R F[3], M[3];
    R power;
};

// Main rotor (:203-270) and fuselage (:302-320).
template <typename R>
HD Loads<R> main_loads(const Params<R>& P, const R* __restrict__ s, const Controls<R>& u, const Frame<R>& f) {
    const R vi_mr = s[0], b0 = s[4], b1 = s[5], p = s[9], q = s[10];
    const R ua = f.ua, va = f.va, wa = f.wa, rho = f.rho, irho = f.irho;
    Loads<R> o;
    // ---- main rotor
    const R igam = irho * P.mr_inv_gam_dro;
    const R KC = P.mr_kc_num * igam + P.mr_K1;
    const R og = P.mr_OMEGA * igam;
    const R ITB2_OM = P.mr_OMEGA * m_rcp((R)1 + og * og);
    const R ITB = ITB2_OM * og;
    const R DL_DA1 = rho * P.mr_DL_DA1_dro;
    const R vadv2 = ua * ua + va * va;
    const R wr = wa + (b0 - P.mr_IS) * ua - b1 * va;
    const R wb = wr + u.mr_wb0 + vadv2 * u.mr_wb1;
    const R thr = (wb - vi_mr) * rho * P.mr_coef;
    const R dw = wr - vi_mr;
    o.d[0] = P.mr_inflow * (thr * irho * P.mr_inv_thr_den - vi_mr * m_sqrt(vadv2 + dw * dw));
    const R power_mr = thr * (vi_mr - wr) + rho * P.mr_prof * (P.mr_vtip2 + (R)3 * vadv2);
    R CT = thr * irho * P.mr_inv_ct_den;
    CT = CT > (R)0 ? CT : (R)0;
    const R DB1DV = P.mr_2_vtip * (P.mr_8_asig * CT + m_sqrt((R)0.5 * CT));
    const R wake = m_fabs(ua) > P.vtrans ? (R)1 : (R)0;
    const R a_sum = b1 - u.lat + KC * b0 + DB1DV * va * ((R)1 + wake);
    const R b_sum = b0 + u.lon - KC * b1 - DB1DV * ua * ((R)1 + (R)2 * wake);
    o.d[1] = -ITB * b_sum - ITB2_OM * a_sum - q;
    o.d[2] = -ITB * a_sum + ITB2_OM * b_sum - p;
    const R X_MR = -thr * (b0 - P.mr_IS), Y_MR = thr * b1, Z_MR = -thr;
    const R L_MR = Y_MR * P.mr_H + P.mr_DL_DB1 * b1 + DL_DA1 * (b0 + u.lon - P.mr_K1 * b1);
    const R M_MR = Z_MR * P.mr_D - X_MR * P.mr_H + P.mr_DL_DB1 * b0 + DL_DA1 * (-b1 + u.lat - P.mr_K1 * b0);
    // ---- fuselage
    R wa_f = wa - vi_mr;
    wa_f = wa_f > (R)0 ? wa_f + (R)kEps : wa_f;
    const R d_fw = ((ua * m_rcp(-wa_f)) * P.fus_dfw_k - P.fus_dfw_c) * P.fus_COR;
    const R rh = (R)0.5 * rho;
    const R X_F = rh * P.fus_XUU * m_fabs(ua) * ua;
    const R Y_F = rh * P.fus_YVV * m_fabs(va) * va;
    const R Z_F = rh * P.fus_ZWW * m_fabs(wa_f) * wa_f;
    const R power_fus = -X_F * ua - Y_F * va - Z_F * wa_f;
    // Z_F * d_fw -> 0 as wa_f -> 0 (Z_F ~ wa_f^2, d_fw ~ 1/wa_f).  At wa_f == 0 exactly the reference's
    // expression is 0 * inf = NaN; in its fp64 arithmetic that point is never hit, while this fp32
    // restatement lands on it about once per 1e9 stage evaluations (a descending helicopter with
    // w_air == vi_mr), which would leave the env NaN until its time limit.  The fp32 step takes the
    // limit there; the fp64 trims keep the reference's expression.
    R zd = Z_F * d_fw;
    if constexpr (sizeof(R) == sizeof(float)) zd = wa_f == (R)0 ? (R)0 : zd;
    // climb and fuselage power load the main rotor's torque (:446-447)
    const R power_climb = P.wt * (-f.n2);
    const R p_extra = power_climb + power_fus;
    o.F[0] = X_MR + X_F;
    o.F[1] = Y_MR + Y_F;
    o.F[2] = Z_MR + Z_F;
    o.M[0] = L_MR + Y_F * P.fus_H;
    o.M[1] = M_MR + (zd - X_F * P.fus_H);
    o.M[2] = power_mr * P.mr_inv_OMEGA + p_extra * P.mr_inv_OMEGA;
    o.power = power_mr + p_extra;
    return o;
}

// Tail rotor (:272-300), horizontal tail (:322-345), vertical tail (:347-361), wing (:363-383),
// landing gear (:385-398).
template <typename R>
HD Loads<R> tail_loads(const Params<R>& P, const R* __restrict__ s, const Controls<R>& u, const Frame<R>& f) {
    const R vi_mr = s[0], vi_tr = s[1], p = s[9], q = s[10], r = s[11];
    const R ua = f.ua, va = f.va, wa = f.wa, rho = f.rho, irho = f.irho;
    Loads<R> o;
    // ---- tail rotor
    const R wq = wa + q * P.tr_D;
    const R vadv2t = wq * wq + ua * ua;
    const R vr = -(va - r * P.tr_D + p * P.tr_H);
    const R vb = vr + u.tr_vb0 + vadv2t * u.tr_vb1;
    const R thr_t = (vb - vi_tr) * rho * P.tr_coef;
    const R dwt = vr - vi_tr;
    o.d[0] = P.tr_inflow * (thr_t * irho * P.tr_inv_thr_den - vi_tr * m_sqrt(vadv2t + dwt * dwt));
    o.d[1] = (R)0;
    o.d[2] = (R)0;
    const R power_tr = thr_t * (vi_tr - vr);
    const R rh = (R)0.5 * rho;
    // ---- horizontal tail
    const R v_dw = m_max(vi_mr - wa, (R)kEps);
    const R d_dw = ua * m_rcp(v_dw) * P.ht_dw_k - P.ht_dw_c;
    const R eps_ht = (d_dw > (R)0 && d_dw < P.mr_R) ? (R)2 * ((R)1 - d_dw * P.mr_inv_R) : (R)0;
    const R wa_ht = wa - eps_ht * vi_mr + P.ht_D * q;
    const R aua = m_fabs(ua);
    R Z_HT;
    if (m_fabs(wa_ht) > (R)0.3 * aua)
        Z_HT = rh * P.ht_ZMAX * m_sqrt(ua * ua + va * va + wa_ht * wa_ht) * wa_ht;
    else
        Z_HT = rh * (P.ht_ZUU * aua * ua + P.ht_ZUW * aua * wa_ht);
    // ---- vertical tail
    const R va_vt = va + vi_tr - P.vt_D * r;
    R Y_VT;
    if (m_fabs(va_vt) > (R)0.3 * aua)
        Y_VT = rh * P.vt_YMAX * m_sqrt(ua * ua + va_vt * va_vt) * va_vt;
    else
        Y_VT = rh * (P.vt_YUU * aua * ua + P.vt_YUV * aua * va_vt);
    // ---- wing; the AW109 has none (ZUW = 0), the branch is uniform.  Absent loads are -0: x + (-0)
    // is x for every x, so the sums below fold away (x + (+0) is not foldable: -0 + +0 = +0).
    R X_WN = (R)-0.0, Z_WN = (R)-0.0;
    if (P.wn_on) {
        const R wa_w = wa - vi_mr;
        const R vta2 = ua * ua + wa_w * wa_w;
        const R qq = P.wn_ZUU * ua * ua + P.wn_ZUW * ua * wa_w;
        Z_WN = m_fabs(wa_w) > (R)0.3 * aua ? rh * P.wn_ZMAX * m_sqrt(vta2) * wa_w : rh * qq;
        X_WN = -rh * (R)(1.0 / kPi) * m_rcp(vta2) * qq * qq;
    }
    const R power_wn = P.wn_on ? m_fabs(X_WN * ua) : (R)-0.0;
    // ---- landing gear.  QUIRK: the moment uses the ACCUMULATED force (:397).
    R Fl0 = (R)-0.0, Fl1 = (R)-0.0, Fl2 = (R)-0.0, Ml0 = (R)-0.0, Ml1 = (R)-0.0, Ml2 = (R)-0.0;
    const R zh = f.zh, B02 = f.B02, B12 = f.B12, B22 = f.B22;
    // Contact is rare.  A gear point's pos_z + h is zh + (B^T r_g)_z <= zh + |r_g|, so no point can
    // touch while zh + max|r_g| <= -WL_CG/12 (lg_reach carries a rounding margin): the wave skips
    // the per-point tests and the spring-damper code unless one of its lanes is that close.
    if (wave_any(zh + P.lg_reach > -P.wl_cg_ft))
#pragma unroll
    for (int g = 0; g < 3; ++g) {
        const R rx = P.lg_loc[g][0], ry = P.lg_loc[g][1], rz = P.lg_loc[g][2];
        const R pzh = zh + (B02 * rx + B12 * ry + B22 * rz);   // pos_z + h
        if (-pzh - P.wl_cg_ft < (R)0) {                        // -pos_z - (h + WL_CG/12) < 0
            const R cx = q * rz - r * ry, cy = r * rx - p * rz, cz = p * ry - q * rx;
            const R vel_z = f.n2 + (B02 * cx + B12 * cy + B22 * cz);
            const R fz = -(P.lg_C * vel_z + P.lg_K * pzh) + (R)kEps;
            Fl0 += B02 * fz; Fl1 += B12 * fz; Fl2 += B22 * fz;
            Ml0 += ry * Fl2 - rz * Fl1;
            Ml1 += rz * Fl0 - rx * Fl2;
            Ml2 += rx * Fl1 - ry * Fl0;
        }
    }
    o.F[0] = X_WN + Fl0;
    o.F[1] = thr_t + Y_VT + Fl1;
    o.F[2] = Z_HT + Z_WN + Fl2;
    o.M[0] = thr_t * P.tr_H + Y_VT * P.vt_H + Ml0;
    o.M[1] = Z_HT * P.ht_D + Ml1;
    o.M[2] = Ml2 - thr_t * P.tr_D - Y_VT * P.vt_D;
    o.power = power_tr + power_wn;
    return o;
}

// Totals and the rigid-body equations of motion (:446-470) from the two groups.
template <typename R>
HD void eom(const Params<R>& P, const R* __restrict__ s, const Frame<R>& f, const Loads<R>& A, const Loads<R>& B,
            R* __restrict__ d) {
    const R uu = s[6], vv = s[7], ww = s[8], p = s[9], q = s[10], r = s[11];
    d[0] = A.d[0];
    d[1] = B.d[0];
    d[2] = P.mr_OMEGA;
    d[3] = P.tr_OMEGA;
    d[4] = A.d[1];
    d[5] = A.d[2];
    const R Fx = (A.F[0] + B.F[0]) + P.wt * f.B02;
    const R Fy = (A.F[1] + B.F[1]) + P.wt * f.B12;
    const R Fz = (A.F[2] + B.F[2]) + P.wt * f.B22;
    const R Mx = A.M[0] + B.M[0], My = A.M[1] + B.M[1], Mz = A.M[2] + B.M[2];
    d[6] = Fx * P.inv_mass - (q * ww - r * vv);
    d[7] = Fy * P.inv_mass - (r * uu - p * ww);
    d[8] = Fz * P.inv_mass - (p * vv - q * uu);
    const R Ip0 = P.Ixx * p + P.Ixz * r, Ip1 = P.Iyy * q, Ip2 = P.Ixz * p + P.Izz * r;
    const R g0 = Mx - (q * Ip2 - r * Ip1);
    const R g1 = My - (r * Ip0 - p * Ip2);
    const R g2 = Mz - (p * Ip1 - q * Ip0);
    d[9] = P.Ji00 * g0 + P.Ji02 * g2;
    d[10] = P.Ji11 * g1;
    d[11] = P.Ji20 * g0 + P.Ji22 * g2;
    d[12] = f.phid; d[13] = f.thd; d[14] = f.psid;
    d[15] = f.n0; d[16] = f.n1; d[17] = f.n2;
}

// The observation at this stage's input state (:471-488).
template <typename R>
HD void observe(const Params<R>& P, const R* __restrict__ s, const Frame<R>& f, const Loads<R>& A,
                const Loads<R>& B, R* __restrict__ obs) {
    obs[0] = ((A.power + B.power) + P.p_loss) * (R)(1.0 / 550.0);
    obs[1] = f.ua; obs[2] = f.va; obs[3] = f.wa;
    obs[4] = f.n0; obs[5] = f.n1; obs[6] = f.n2;
    obs[7] = s[12]; obs[8] = s[13]; obs[9] = s[14];
    obs[10] = s[9]; obs[11] = s[10]; obs[12] = s[11];
    obs[13] = s[15]; obs[14] = s[16]; obs[15] = -s[17]; obs[16] = -f.zh;
}

// One evaluation of the model; with OBS also the 17 observations.
template <bool OBS, typename R>
HD void dynamics(const Params<R>& P, const R* __restrict__ s, const Controls<R>& u, const R W[3],
                 const Ground<R>& gc, const Attitude<R>& att, R* __restrict__ d, R* __restrict__ obs,
                 const R* rho_irho = nullptr) {
    const Frame<R> f = frame(P, s, W, gc, att, rho_irho);
    const Loads<R> A = main_loads(P, s, u, f);
    const Loads<R> B = tail_loads(P, s, u, f);
    eom(P, s, f, A, B, d);
    if (OBS) observe(P, s, f, A, B, obs);
}

// ------------------------------------------------------------------------------------------
// Tasks and flags

// HeliHover._calculate_reward (helicopter_with_tasks.py:27-52)
template <typename R>
HD R reward_hover(const Params<R>& P, const R s[18], const R d[18], bool* success) {
    R pf = 0, pt = 0, xf = 0, xt = 0;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        const R pn = s[9 + i] * P.n_t, pdn = d[9 + i] * P.n_t2;
        const R e = s[15 + i] * P.inv_n_x - P.tgt_n[i];
        pf -= pn * pn;
        pt -= m_sign(pn) * pdn;
        xf -= e * e;
        xt -= m_sign(e) * (d[15 + i] * P.inv_n_v);
    }
    *success = pf > (R)-1 && xf > (R)-1;
    return (m_max(pf, pt) + m_max(xf, xt)) * (R)0.5;
}

// HeliForwardFlight._calculate_reward (helicopter_with_tasks.py:78-115).  QUIRK: divides by the
// speed, so a helicopter at exactly zero velocity gets a NaN reward like the reference.
template <typename R>
HD R reward_forward(const Params<R>& P, const R s[18], const R d[18], bool* success) {
    const R vel = m_sqrt(s[6] * s[6] + s[7] * s[7] + s[8] * s[8]);
    const R vn = vel * P.inv_n_v;
    const R vdn = (s[6] * d[6] + s[7] * d[7] + s[8] * d[8]) * m_rcp(vel) * P.inv_n_a;
    const R dn = s[17] * P.inv_n_x, ddn = d[17] * P.inv_n_v;
    R pf = 0, pt = 0;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        const R pn = s[9 + i] * P.n_t, pdn = d[9 + i] * P.n_t2;
        pf -= pn * pn;
        pt -= m_sign(pn) * pdn;
    }
    const R ev = vn - P.vel_tgt_n, ed = dn - P.dwn_tgt_n;
    const R vf = -ev * ev, vt = -m_sign(ev) * vdn;
    const R df = -ed * ed, dtt = -m_sign(ed) * ddn;
    *success = pf > (R)-1 && vf > (R)-1 && df > (R)-1;
    return (m_max(pf, pt) + m_max(vf, vt) + m_max(df, dtt)) * (R)(1.0 / 3.0);
}

// Heli._is_failed (helicopter.py:226-234) on the post-step state, k4 derivatives and the ground
// height under the post-step position.
template <typename R>
HD bool is_failed(const Params<R>& P, const R s[18], const R d[18], const Ground<R>& gp) {
    const R gta = gp.h() + P.wl_cg_ft;
    const bool hit = -gp.zh(s[17]) - P.wl_cg_ft < (R)0;
    const bool c2 = d[17] > P.fail_zdot;
    const bool c3 = s[12] > P.fail_ang, c4 = s[13] > P.fail_ang;
    const bool c5 = m_fabs(s[15]) > P.ns_half || m_fabs(s[16]) > P.ew_half || -s[17] > gta + (R)10000;
    return (hit && (c2 || c3 || c4)) || c5;
}

}  // namespace hg
