/*
 * heli_oracle.c — CPU restatement of the reference heli-gym step()/reset() path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
 * leg may load this library (oracle/liboracle.so); the product path (heli-gym_amd/) never links,
 * loads or calls it.  It is the checker the HIP kernel is compared against, and the "port" CPU
 * baseline.
 *
 * Pinning: every function below is checked in tests/test_oracle_golden.py against golden vectors
 * that tools/gen_goldens.py produced by running the unmodified reference Python code
 * (/root/reference, ugurcanozalp/heli-gym v2, numpy 2.2.6) in the build container.
 *
 * Numerics: fp64, with the reference's fp32 rounding points restated where the reference packs
 * values into float32 arrays (F32() below): component force/moment vectors and their partial
 * sums, the rotor/flapping state derivatives, the DCMs and inertia inverse, the turbulence
 * derivatives and wind output.  Controls computed from fp32 actions use float32
 * arithmetic like numpy-2 weak-scalar promotion does (helicopter_dynamics.py:414-422).
 *
 * Every function cites the reference file:line it restates (paths relative to
 * /root/reference/heligym/envs/).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/heligym_amd.h"

#define F32(x) ((double)(float)(x))
#define EPS_DYN 1e-4            /* helicopter_dynamics.py:15, wind_dynamics.py:10 */
#define R2D (180.0 / M_PI)      /* helicopter_dynamics.py:16 */
#define D2R (1.0 / R2D)         /* helicopter_dynamics.py:17 */
#define SQRT_3 1.7320508075688772     /* wind_dynamics.py:12 */
#define TWO_D_PI 0.6366197723675814   /* wind_dynamics.py:13 */

typedef struct or_model {
    hg_config cfg;
    /* derived constants, helicopter_dynamics.py:107-154 */
    double mr_H, mr_D, fus_H, fus_D, wn_H, wn_D, ht_H, ht_D, vt_H, vt_D, tr_H, tr_D;
    double lg_loc[3][3];          /* fp32 arrays (:123-126) */
    double mass;                  /* :128 */
    double mr_OMEGA, mr_VTIP, mr_FR, mr_SOL, mr_ASIG, mr_GAM_DRO, mr_DL_DB1, mr_DL_DA1_DRO, mr_COEF;
    double tr_OMEGA, tr_FR, tr_VTIP, tr_SOL, tr_COEF;
    double I[3][3], IINV[3][3];   /* fp32 (:151-154) */
    /* wind, wind_dynamics.py:21-37 */
    double eta_norm, wind_dir, wind_mean[3];
    float tep[8][13];             /* LookUpTable(7,12) data, float32 (lookup.py:91) */
    /* env normalisers, helicopter.py:63-68 */
    double n_t, n_x, n_v, n_a;
    /* terrain (fp64 heights like the reference: png/65535*MAX_GR_ALT, :39-43) */
    double* hmap;
    int rows, cols;
} or_model;

typedef struct or_env {
    double heli[HG_N_HELI];
    double wind[HG_N_WIND];
    double obs[HG_N_OBS];        /* heli_dyn.observation (previous step / trim) */
    double dots[HG_N_HELI];      /* heli_dyn.state_dots (k4 / trim) */
    double time_counter;         /* helicopter.py:193 */
    double successed_time;       /* helicopter.py:205 */
    int32_t state_f32;           /* 1 right after a reset: the state array is still float32 */
    int32_t _pad;
} or_env;

typedef struct or_out {
    double obs[HG_N_OBS];
    double wind_ned[3];
    double reward_hover, reward_ff, reward;
    int32_t success_hover, success_ff, failed, successed, time_up, terminated, truncated, _pad;
} or_out;

/* ------------------------------------------------------------------ utils.py / lookup.py */

/* utils.py:3-4 — numpy floor-mod semantics. */
double or_pi_bound(double x) {
    double m = 2.0 * M_PI;
    double r = fmod(x + M_PI, m);
    if (r != 0.0 && ((r < 0) != (m < 0))) r += m;
    return r - M_PI;
}

/* lookup.py:146-183 (get_value_2D), float32 table and float32 arithmetic (weak python scalars).
 * `t` is the (nr+1)x(nc+1) table, row 0 = column keys, column 0 = row keys.  The stateful
 * last-index cache of the reference only changes where the walk starts, not the bracket. */
static double lut2d_f64(const float* t, int nr, int nc, double rowKey, double colKey);

double or_lut2d(const float* t, int nr, int nc, double rowKey, double colKey) {
#define T(i, j) t[(i) * (nc + 1) + (j)]
    int r = 2, c = 2;
    float rk = (float)rowKey, ck = (float)colKey;
    while (r > 2 && T(r - 1, 0) > rowKey) r -= 1;
    while (r < nr && T(r, 0) < rowKey) r += 1;
    while (c > 2 && T(0, c - 1) > colKey) c -= 1;
    while (c < nc && T(0, c) < colKey) c += 1;
    float rF = (rk - T(r - 1, 0)) / (T(r, 0) - T(r - 1, 0));
    float cF = (ck - T(0, c - 1)) / (T(0, c) - T(0, c - 1));
    if (rF > 1.0f) rF = 1.0f; else if (rF < 0.0f) rF = 0.0f;
    if (cF > 1.0f) cF = 1.0f; else if (cF < 0.0f) cF = 0.0f;
    float c1 = rF * (T(r, c - 1) - T(r - 1, c - 1)) + T(r - 1, c - 1);
    float c2 = rF * (T(r, c) - T(r - 1, c)) + T(r - 1, c);
    return (double)(c1 + cF * (c2 - c1));
}

/* Same walk with float64 arithmetic: what the reference computes when the keys are numpy
 * float64 scalars instead of python floats (used only by the docstring KAT). */
static double lut2d_f64(const float* t, int nr, int nc, double rowKey, double colKey) {
    int r = 2, c = 2;
    while (r > 2 && T(r - 1, 0) > rowKey) r -= 1;
    while (r < nr && T(r, 0) < rowKey) r += 1;
    while (c > 2 && T(0, c - 1) > colKey) c -= 1;
    while (c < nc && T(0, c) < colKey) c += 1;
    double rF = (rowKey - T(r - 1, 0)) / ((double)(T(r, 0) - T(r - 1, 0)));
    double cF = (colKey - T(0, c - 1)) / ((double)(T(0, c) - T(0, c - 1)));
    if (rF > 1.0) rF = 1.0; else if (rF < 0.0) rF = 0.0;
    if (cF > 1.0) cF = 1.0; else if (cF < 0.0) cF = 0.0;
    double c1 = rF * (double)(T(r, c - 1) - T(r - 1, c - 1)) + T(r - 1, c - 1);
    double c2 = rF * (double)(T(r, c) - T(r - 1, c)) + T(r - 1, c);
    return c1 + cF * (c2 - c1);
#undef T
}

double or_lut2d_f64(const float* t, int nr, int nc, double rowKey, double colKey) {
    return lut2d_f64(t, nr, nc, rowKey, colKey);
}

/* ------------------------------------------------------------------ model construction */

static const double TEP_COLS[12] = {500.0, 1750.0, 3750.0, 7500.0, 15000.0, 25000.0, 35000.0,
                                    45000.0, 55000.0, 65000.0, 75000.0, 80000.0};
/* MIL-HDBK-1797 turbulence exceedance table, wind_dynamics.py:29-37 (values are physical data). */
static const double TEP_VALS[7][12] = {
    {3.2, 2.2, 1.5, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0},
    {4.2, 3.6, 3.3, 1.6, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0},
    {6.6, 6.9, 7.4, 6.7, 4.6, 2.7, 0.4, 0.0, 0.0, 0.0, 0.0, 0.0},
    {8.6, 9.6, 10.6, 10.1, 8.0, 6.6, 5.0, 4.2, 2.7, 0.0, 0.0, 0.0},
    {11.8, 13.0, 16.0, 15.1, 11.6, 9.7, 8.1, 8.2, 7.9, 4.9, 3.2, 2.1},
    {15.6, 17.6, 23.0, 23.6, 22.1, 20.0, 16.0, 15.1, 12.1, 7.9, 6.2, 5.1},
    {18.7, 21.5, 28.4, 30.2, 30.7, 31.0, 25.2, 23.1, 17.5, 10.7, 8.4, 7.2}};

static void inv3(const double a[3][3], double o[3][3]) {
    double det = a[0][0] * (a[1][1] * a[2][2] - a[1][2] * a[2][1]) -
                 a[0][1] * (a[1][0] * a[2][2] - a[1][2] * a[2][0]) +
                 a[0][2] * (a[1][0] * a[2][1] - a[1][1] * a[2][0]);
    o[0][0] = (a[1][1] * a[2][2] - a[1][2] * a[2][1]) / det;
    o[0][1] = (a[0][2] * a[2][1] - a[0][1] * a[2][2]) / det;
    o[0][2] = (a[0][1] * a[1][2] - a[0][2] * a[1][1]) / det;
    o[1][0] = (a[1][2] * a[2][0] - a[1][0] * a[2][2]) / det;
    o[1][1] = (a[0][0] * a[2][2] - a[0][2] * a[2][0]) / det;
    o[1][2] = (a[0][2] * a[1][0] - a[0][0] * a[1][2]) / det;
    o[2][0] = (a[1][0] * a[2][1] - a[1][1] * a[2][0]) / det;
    o[2][1] = (a[0][1] * a[2][0] - a[0][0] * a[2][1]) / det;
    o[2][2] = (a[0][0] * a[1][1] - a[0][1] * a[1][0]) / det;
}

/* helicopter_dynamics.py:29-44,107-154; wind_dynamics.py:21-37; helicopter.py:63-68 */
or_model* or_create(const hg_config* cfg, const uint16_t* hmap_u16, int rows, int cols) {
    or_model* m = (or_model*)calloc(1, sizeof(or_model));
    const hg_airframe* a = &cfg->af;
    m->cfg = *cfg;
    m->mr_H = (a->mr_WL - a->WL_CG) / 12;  m->mr_D = (a->mr_FS - a->FS_CG) / 12;
    m->fus_H = (a->fus_WL - a->WL_CG) / 12; m->fus_D = (a->fus_FS - a->FS_CG) / 12;
    m->wn_H = (a->wn_WL - a->WL_CG) / 12;  m->wn_D = (a->wn_FS - a->FS_CG) / 12;
    m->ht_H = (a->ht_WL - a->WL_CG) / 12;  m->ht_D = (a->ht_FS - a->FS_CG) / 12;
    m->vt_H = (a->vt_WL - a->WL_CG) / 12;  m->vt_D = (a->vt_FS - a->FS_CG) / 12;
    m->tr_H = (a->tr_WL - a->WL_CG) / 12;  m->tr_D = (a->tr_FS - a->FS_CG) / 12;
    /* :123-126  (float32 arrays: each entry rounded after the /12) */
    double n_loc[3] = {-(a->lg_FS_N - a->FS_CG), -0.0, -(a->lg_WL - a->WL_CG)};
    double r_loc[3] = {-(a->lg_FS_MN - a->FS_CG), a->lg_BL_MN, -(a->lg_WL - a->WL_CG)};
    double l_loc[3] = {-(a->lg_FS_MN - a->FS_CG), -a->lg_BL_MN, -(a->lg_WL - a->WL_CG)};
    for (int i = 0; i < 3; i++) {
        /* np.array(..., float32) rounds the inch values first, then / 12 in float32 */
        m->lg_loc[0][i] = (double)((float)n_loc[i] / 12.0f);
        m->lg_loc[1][i] = (double)((float)r_loc[i] / 12.0f);
        m->lg_loc[2][i] = (double)((float)l_loc[i] / 12.0f);
    }
    m->mass = a->WT / a->env_GRAV;
    m->mr_OMEGA = a->mr_RPM * 2 * M_PI / 60;
    m->mr_VTIP = a->mr_R * m->mr_OMEGA;
    m->mr_FR = a->mr_CD0 * a->mr_R * a->mr_B * a->mr_C;
    m->mr_SOL = a->mr_B * a->mr_C / (a->mr_R * M_PI);
    m->mr_ASIG = a->mr_A * m->mr_SOL;
    m->mr_GAM_DRO = a->mr_A * a->mr_C * pow(a->mr_R, 4) / a->mr_IB * m->mr_OMEGA / 16 *
                    (1 + 8.0 / 3 * a->mr_E / a->mr_R);
    m->mr_DL_DB1 = a->mr_B / 2 * (1.5 * a->mr_IB * a->mr_E / a->mr_R * m->mr_OMEGA * m->mr_OMEGA);
    m->mr_DL_DA1_DRO = 0.5 * a->mr_A * a->mr_B * a->mr_C * a->mr_R * m->mr_VTIP * m->mr_VTIP * a->mr_E / 6;
    m->mr_COEF = 0.25 * m->mr_VTIP * a->mr_R * a->mr_A * a->mr_B * a->mr_C;
    m->tr_OMEGA = a->tr_RPM * 2 * M_PI / 60;
    m->tr_FR = a->tr_CD0 * a->tr_R * a->tr_B * a->tr_C;
    m->tr_VTIP = a->tr_R * m->tr_OMEGA;
    m->tr_SOL = a->tr_B * a->tr_C / (a->tr_R * M_PI);
    m->tr_COEF = 0.25 * m->tr_VTIP * a->tr_R * a->tr_A * a->tr_B * a->tr_C;
    double I[3][3] = {{a->IX, 0, -a->IXZ}, {0, a->IY, 0}, {-a->IXZ, 0, a->IZ}};
    double Ii[3][3];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) m->I[i][j] = F32(I[i][j]);
    inv3(m->I, Ii);
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) m->IINV[i][j] = F32(Ii[i][j]);
    /* wind_dynamics.py:21-37 */
    m->eta_norm = 1.0 / sqrt(cfg->dt);
    m->wind_dir = a->env_WIND_DIR_deg * D2R;
    m->wind_mean[0] = (double)((float)a->env_WIND_SPD * (float)cos(m->wind_dir));
    m->wind_mean[1] = (double)((float)a->env_WIND_SPD * (float)sin(m->wind_dir));
    m->wind_mean[2] = 0.0;
    memset(m->tep, 0, sizeof(m->tep));
    for (int j = 0; j < 12; j++) m->tep[0][j + 1] = (float)TEP_COLS[j];
    for (int i = 0; i < 7; i++) {
        m->tep[i + 1][0] = (float)(i + 1);
        for (int j = 0; j < 12; j++) m->tep[i + 1][j + 1] = (float)TEP_VALS[i][j];
    }
    m->n_t = sqrt(2 * a->mr_R / a->env_GRAV);
    m->n_x = 2 * a->mr_R;
    m->n_v = sqrt(2 * a->mr_R * a->env_GRAV);
    m->n_a = a->env_GRAV;
    m->rows = rows;
    m->cols = cols;
    m->hmap = (double*)malloc(sizeof(double) * (size_t)rows * cols);
    for (size_t i = 0; i < (size_t)rows * cols; i++)
        m->hmap[i] = ((double)hmap_u16[i] / 65535.0) * a->env_MAX_GR_ALT;
    return m;
}

void or_free(or_model* m) {
    if (!m) return;
    free(m->hmap);
    free(m);
}

/* Named derived constants for the KAT test (helicopter_dynamics.py:107-154). */
double or_const(const or_model* m, const char* n) {
#define C(s, v) if (!strcmp(n, s)) return v;
    C("MR.H", m->mr_H) C("MR.D", m->mr_D) C("MR.OMEGA", m->mr_OMEGA) C("MR.V_TIP", m->mr_VTIP)
    C("MR.FR", m->mr_FR) C("MR.SOL", m->mr_SOL) C("MR.A_SIGMA", m->mr_ASIG)
    C("MR.GAM_OM16_DRO", m->mr_GAM_DRO) C("MR.DL_DB1", m->mr_DL_DB1)
    C("MR.DL_DA1_DRO", m->mr_DL_DA1_DRO) C("MR.COEF_TH", m->mr_COEF)
    C("TR.H", m->tr_H) C("TR.D", m->tr_D) C("TR.OMEGA", m->tr_OMEGA) C("TR.V_TIP", m->tr_VTIP)
    C("TR.FR", m->tr_FR) C("TR.SOL", m->tr_SOL) C("TR.COEF_TH", m->tr_COEF)
    C("FUS.H", m->fus_H) C("FUS.D", m->fus_D) C("HT.H", m->ht_H) C("HT.D", m->ht_D)
    C("VT.H", m->vt_H) C("VT.D", m->vt_D) C("WN.H", m->wn_H) C("WN.D", m->wn_D)
    C("HELI.M", m->mass)
    C("IINV00", m->IINV[0][0]) C("IINV02", m->IINV[0][2]) C("IINV11", m->IINV[1][1])
    C("IINV20", m->IINV[2][0]) C("IINV22", m->IINV[2][2])
    C("WIND_N", m->wind_mean[0]) C("WIND_E", m->wind_mean[1])
    C("NORM_T", m->n_t) C("NORM_X", m->n_x) C("NORM_V", m->n_v) C("NORM_A", m->n_a)
#undef C
    return NAN;
}

void or_lg_loc(const or_model* m, double out[9]) {
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) out[3 * i + j] = m->lg_loc[i][j];
}

/* ------------------------------------------------------------------ terrain */

/* helicopter_dynamics.py:167-195 (x, y = the COMMITTED state position).  While the state array
 * is still float32 (trim, and the first step after a reset: dynamics.py:142-144,168) numpy-2
 * evaluates x_loc in float32 (np.float32 / python float); afterwards in float64. */
double or_ground_height_p(const or_model* m, double x, double y, int state_f32) {
    const hg_airframe* a = &m->cfg.af;
    int R = m->rows, Cc = m->cols;
    double x_ = a->env_NS_MAX / R, y_ = a->env_EW_MAX / Cc;
    double x_loc, y_loc;
    if (state_f32) {
        x_loc = (double)((float)x / (float)x_ + (float)(R / 2));
        y_loc = (double)((float)y / (float)y_ + (float)(Cc / 2));
    } else {
        x_loc = x / x_ + (R / 2);
        y_loc = y / y_ + (Cc / 2);
    }
    if (x_loc < 0) x_loc = 0; else if (x_loc > R - 1) x_loc = R - 1;
    if (y_loc < 0) y_loc = 0; else if (y_loc > R - 1) y_loc = R - 1;   /* shape[0], :182-183 */
    int xi = (int)floor(x_loc), yi = (int)floor(y_loc);
    double middle = m->hmap[(size_t)yi * Cc + xi];
    if (xi == R - 1) xi = R - 2;
    if (yi == Cc - 1) yi = Cc - 2;
    double north = m->hmap[(size_t)yi * Cc + xi + 1];
    double east = m->hmap[(size_t)(yi + 1) * Cc + xi];
    return middle + (north - middle) * (x_loc - xi) + (east - middle) * (y_loc - yi);
}

double or_ground_height(const or_model* m, double x, double y) { return or_ground_height_p(m, x, y, 0); }

/* :200-201 */
static double ground_touching_altitude(const or_model* m, double x, double y, int state_f32) {
    return or_ground_height_p(m, x, y, state_f32) + m->cfg.af.WL_CG / 12;
}

/* ------------------------------------------------------------------ Dryden wind */

/* wind_dynamics.py:54-83 -> [Lu, Lv, Lw, su, sv, sw, azimuth] */
void or_dryden_params(const or_model* m, double h_gr, const double vel_inf_ned[3], double out[7]) {
    double lvl = m->cfg.af.env_TURB_LVL;
    double w20 = lvl / 7 * 88.61;
    double Lu, Lv, Lw, su, sv, sw, az;
    if (h_gr <= 1000.0) {
        double h = h_gr > 10.0 ? h_gr : 10.0;
        Lu = h / pow(0.177 + 0.000823 * h, 1.2);
        Lv = 0.5 * Lu;
        Lw = 0.5 * h;
        sw = 0.1 * w20;
        su = sw / pow(0.177 + 0.000823 * h, 0.4);
        sv = su;
        az = m->wind_dir;
    } else if (h_gr >= 2000.0) {
        Lu = 1750.0; Lv = 0.5 * Lu; Lw = 0.5 * Lu;
        double s = or_lut2d(&m->tep[0][0], 7, 12, lvl, h_gr);
        su = sv = sw = s;
        az = atan2(vel_inf_ned[1], vel_inf_ned[0]);
    } else {
        Lu = 1000 + (h_gr - 1000.0) / 1000.0 * 750.0;
        Lv = 0.5 * Lu;
        Lw = Lu;   /* wind_dynamics.py:76 */
        /* TEP value is np.float32, so the blend runs in float32 (weak python scalars) */
        float tv = (float)or_lut2d(&m->tep[0][0], 7, 12, lvl, h_gr);
        float blend = (float)((h_gr - 1000.0) / 1000.0) * (tv - (float)(0.1 * w20));
        double s = (double)((float)(0.1 * w20) + blend);
        su = sv = sw = s;
        double r = (h_gr - 1000.0) / 1000.0;
        /* wind_mean_ned is a float32 array: its product with the python float (1 - r) is float32 */
        double m1 = (double)((float)m->wind_mean[1] * (float)(1 - r));
        double m0 = (double)((float)m->wind_mean[0] * (float)(1 - r));
        az = atan2(vel_inf_ned[1] * r + m1, vel_inf_ned[0] * r + m0);
    }
    out[0] = Lu; out[1] = Lv; out[2] = Lw; out[3] = su; out[4] = sv; out[5] = sw; out[6] = az;
}

typedef struct wind_par { double t_u, t_v, t_w, su, sv, sw, az; } wind_par;

/* wind_dynamics.py:101-109 (derivatives are float32 arrays) */
static void wind_f(const wind_par* p, const double eta[3], const double s[5], double d[5]) {
    d[0] = F32(1 / p->t_u * (eta[0] - s[0]));
    d[1] = F32(1 / (4 * p->t_v * p->t_v) * (eta[1] - s[2]) - 1 / p->t_v * s[1]);
    d[2] = F32(s[1]);
    d[3] = F32(1 / (4 * p->t_w * p->t_w) * (eta[2] - s[4]) - 1 / p->t_w * s[3]);
    d[4] = F32(s[3]);
}

/* WindDynamics.step: dynamics.py:158-171 with wind_dynamics.py:85-125.  `carry` = previous heli
 * observation [N_VEL, E_VEL, DES_RATE, GROUND_ALT] (helicopter.py:195-196).  The derivative
 * object is aliased across the four stages (wind_dynamics.py:86,107-109), so the update uses the
 * stage-4 derivative six times.  Writes the wind NED velocity (float32). */
void or_wind_step(const or_model* m, double s[5], const double carry[4], const double eta[3], double wind_out[3]) {
    double vinf[3] = {carry[0] + m->wind_mean[0], carry[1] + m->wind_mean[1], carry[2] + m->wind_mean[2]};
    double vel = sqrt(vinf[0] * vinf[0] + vinf[1] * vinf[1] + vinf[2] * vinf[2]);
    double par[7];
    or_dryden_params(m, carry[3], vinf, par);
    wind_par p = {par[0] / (vel + EPS_DYN), par[1] / (vel + EPS_DYN), par[2] / (vel + EPS_DYN),
                  par[3], par[4], par[5], par[6]};
    double dt = m->cfg.dt, k[5], st[5];
    wind_f(&p, eta, s, k);
    for (int i = 0; i < 5; i++) st[i] = s[i] + k[i] * (0.5 * dt);
    wind_f(&p, eta, st, k);
    for (int i = 0; i < 5; i++) st[i] = s[i] + k[i] * (0.5 * dt);
    wind_f(&p, eta, st, k);
    for (int i = 0; i < 5; i++) st[i] = s[i] + k[i] * dt;           /* stage-4 input */
    wind_f(&p, eta, st, k);
    /* observation at the stage-4 input (wind_dynamics.py:111-123) */
    double Ku = p.su * sqrt(TWO_D_PI * p.t_u), Kv = p.sv * sqrt(TWO_D_PI * p.t_v), Kw = p.sw * sqrt(TWO_D_PI * p.t_w);
    double ut = Ku * st[0];
    double vt = Kv * (st[2] + 2 * SQRT_3 * st[1]);
    double wt = Kw * (st[4] + 2 * SQRT_3 * st[3]);
    double c = cos(p.az), sn = sin(p.az);
    double turb[3] = {F32(c * ut - sn * vt), F32(sn * ut + c * vt), F32(wt)};
    for (int i = 0; i < 3; i++) wind_out[i] = F32(m->wind_mean[i] + turb[i]);
    for (int i = 0; i < 5; i++) s[i] = s[i] + (k[i] + k[i] * 2 + k[i] * 2 + k[i]) * (0.16666666666666666 * dt);
}

/* ------------------------------------------------------------------ helicopter dynamics */

typedef struct controls { double coll, lon, lat, ped; } controls;

/* helicopter_dynamics.py:414-422 with float32 actions: numpy-2 weak-scalar promotion keeps every
 * operation in float32. */
static controls controls_f32(const hg_airframe* a, const double act[4]) {
    controls c;
    float a0 = (float)act[0], a1 = (float)act[1], a2 = (float)act[2], a3 = (float)act[3];
    float d2r = (float)D2R;
    float t;
    t = (0.5f * a0) * (float)(a->COL_H - a->COL_L);
    t = (float)a->COL_OS + t;
    t = t + (float)(0.5 * (a->COL_H + a->COL_L));
    c.coll = d2r * t;
    t = (0.5f * a1) * (float)(a->LON_H - a->LON_L);
    t = t + (float)(0.5 * (a->LON_H + a->LON_L));
    c.lon = d2r * t;
    t = (0.5f * a2) * (float)(a->LAT_H - a->LAT_L);
    t = t + (float)(0.5 * (a->LAT_H + a->LAT_L));
    c.lat = d2r * t;
    t = (0.5f * a3) * (float)(a->PED_H - a->PED_L);
    t = (float)a->PED_OS + t;
    t = t + (float)(0.5 * (a->PED_H + a->PED_L));
    c.ped = d2r * t;
    return c;
}

/* Same, fp64 actions (the trim's Newton iterate, helicopter_dynamics.py:534,565). */
static controls controls_f64(const hg_airframe* a, const double act[4]) {
    controls c;
    c.coll = D2R * (a->COL_OS + 0.5 * act[0] * (a->COL_H - a->COL_L) + 0.5 * (a->COL_H + a->COL_L));
    c.lon = D2R * (0.5 * act[1] * (a->LON_H - a->LON_L) + 0.5 * (a->LON_H + a->LON_L));
    c.lat = D2R * (0.5 * act[2] * (a->LAT_H - a->LAT_L) + 0.5 * (a->LAT_H + a->LAT_L));
    c.ped = D2R * (a->PED_OS + 0.5 * act[3] * (a->PED_H - a->PED_L) + 0.5 * (a->PED_H + a->PED_L));
    return c;
}

static void cross(const double a[3], const double b[3], double o[3]) {   /* utils.py:6-14 */
    o[0] = a[1] * b[2] - a[2] * b[1];
    o[1] = a[2] * b[0] - a[0] * b[2];
    o[2] = a[0] * b[1] - a[1] * b[0];
}

/* Diagnostics for the parity tests: the smallest |gear clearance| seen by the landing-gear contact
 * test (helicopter_dynamics.py:393) since the last or_diag_reset().  The reference's contact force
 * jumps by K * WL_CG/12 (~96 000 lb) when a gear crosses that threshold, so a step whose clearance
 * is within rounding of 0 is ill-conditioned for any finite-precision comparison. */
static __thread double g_lg_margin = INFINITY;
void or_diag_reset(void) { g_lg_margin = INFINITY; }
double or_diag_lg_margin(void) { return g_lg_margin; }

/* HelicopterDynamics.dynamics (helicopter_dynamics.py:400-489) at stage state s, with committed
 * ground height h_c (F6).  Writes the 18 derivatives; if obs != NULL also the observation
 * (:471-488). */
void or_dynamics_c(const or_model* m, const double s[18], const controls* u, const double W[3],
                   double h_c, double d[18], double* obs) {
    const hg_airframe* a = &m->cfg.af;
    const double vi_mr = s[0], vi_tr = s[1], b0 = s[4], b1 = s[5];
    const double* uvw = s + 6; const double* pqr = s + 9; const double* eul = s + 12; const double* xyz = s + 15;
    /* kinematic.py:3-18 (fp32 DCM) and :20-29 (fp32 euler-rate matrix) */
    double s0 = sin(eul[0]), c0 = cos(eul[0]), s1 = sin(eul[1]), c1 = cos(eul[1]), s2 = sin(eul[2]), c2 = cos(eul[2]);
    /* phi_rot @ theta_rot @ psi_rot, float32 factors and float32 products (kinematic.py:17) */
    float s0f = (float)s0, c0f = (float)c0, s1f = (float)s1, c1f = (float)c1, s2f = (float)s2, c2f = (float)c2;
    float p10 = s0f * s1f, p20 = c0f * s1f, p21 = -s0f;
    double B[3][3] = {{c1f * c2f, c1f * s2f, -s1f},
                      {p10 * c2f + c0f * (-s2f), p10 * s2f + c0f * c2f, s0f * c1f},
                      {p20 * c2f + p21 * (-s2f), p20 * s2f + p21 * c2f, c0f * c1f}};
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) B[i][j] = F32(B[i][j]);
    double Tm[3][3] = {{1, F32(s0 * s1 / c1), F32(c0 * s1 / c1)}, {0, F32(c0), F32(-s0)}, {0, F32(s0 / c1), F32(c0 / c1)}};
    double eul_dot[3], ned[3], uvwa[3];
    for (int i = 0; i < 3; i++) {
        eul_dot[i] = Tm[i][0] * pqr[0] + Tm[i][1] * pqr[1] + Tm[i][2] * pqr[2];
        ned[i] = B[0][i] * uvw[0] + B[1][i] * uvw[1] + B[2][i] * uvw[2];
        /* earth2body(fp32) @ WIND_NED(fp32): float32 dot product */
        float bw = (float)B[i][0] * (float)W[0];
        bw = bw + (float)B[i][1] * (float)W[1];
        bw = bw + (float)B[i][2] * (float)W[2];
        uvwa[i] = uvw[i] - (double)bw;
    }
    double power_climb = a->WT * (-ned[2]);
    /* :160-165 ISA */
    double temp = a->env_T0 - a->env_LAPSE * (-xyz[2]);
    double rho = a->env_RO_SEA * pow(temp / a->env_T0, (a->env_GRAV / (a->env_LAPSE * a->env_R)) - 1.0);
    const double ua = uvwa[0], va = uvwa[1], wa = uvwa[2];

    /* ---- main rotor :203-270 */
    double GAM = rho * m->mr_GAM_DRO;
    double KC = (0.75 * m->mr_OMEGA * a->mr_E / a->mr_R / GAM) + a->mr_K1;
    double ITB2_OM = m->mr_OMEGA / (1 + pow(m->mr_OMEGA / GAM, 2));
    double ITB = ITB2_OM * m->mr_OMEGA / GAM;
    double DL_DB1 = m->mr_DL_DB1, DL_DA1 = rho * m->mr_DL_DA1_DRO;
    double vadv2 = ua * ua + va * va;
    double wr = wa + (b0 - a->mr_IS) * ua - b1 * va;
    double wb = wr + 0.66667 * m->mr_VTIP * (u->coll + 0.75 * a->mr_TWST) + vadv2 / m->mr_VTIP * (u->coll + 0.5 * a->mr_TWST);
    double thr = (wb - vi_mr) * rho * m->mr_COEF;
    double vi_mr_dot = F32(0.75 * M_PI / a->mr_R * (thr / (2 * M_PI * rho * a->mr_R * a->mr_R) -
                                                   vi_mr * sqrt(vadv2 + (wr - vi_mr) * (wr - vi_mr))));
    double p_ind = thr * (vi_mr - wr);
    double p_prof = 0.5 * rho * (m->mr_FR / 4) * m->mr_VTIP * (m->mr_VTIP * m->mr_VTIP + 3.0 * vadv2);
    double power_mr = p_ind + p_prof;
    double torque_mr = power_mr / m->mr_OMEGA;
    double CT = thr / (rho * M_PI * a->mr_R * a->mr_R * m->mr_VTIP * m->mr_VTIP);
    if (CT < 0.0) CT = 0.0;
    double DB1DV = 2 / m->mr_VTIP * (8 * CT / m->mr_ASIG + sqrt(0.5 * CT));
    double DA1DU = -DB1DV;
    double wake = fabs(ua) > a->VTRANS ? 1.0 : 0.0;
    double a_sum = b1 - u->lat + KC * b0 + DB1DV * va * (1 + wake);
    double b_sum = b0 + u->lon - KC * b1 + DA1DU * ua * (1 + 2 * wake);
    double b0_dot = F32(-ITB * b_sum - ITB2_OM * a_sum - pqr[1]);
    double b1_dot = F32(-ITB * a_sum + ITB2_OM * b_sum - pqr[0]);
    double X_MR = -thr * (b0 - a->mr_IS), Y_MR = thr * b1, Z_MR = -thr;
    double L_MR = Y_MR * m->mr_H + DL_DB1 * b1 + DL_DA1 * (b0 + u->lon - a->mr_K1 * b1);
    double M_MR = Z_MR * m->mr_D - X_MR * m->mr_H + DL_DB1 * b0 + DL_DA1 * (-b1 + u->lat - a->mr_K1 * b0);
    double F_mr[3] = {F32(X_MR), F32(Y_MR), F32(Z_MR)};
    double M_mr[3] = {F32(L_MR), F32(M_MR), F32(torque_mr)};

    /* ---- tail rotor :272-300 */
    double vadv2t = pow(wa + pqr[1] * m->tr_D, 2) + ua * ua;
    double vr = -(va - pqr[2] * m->tr_D + pqr[0] * m->tr_H);
    double vb = vr + 0.66667 * m->tr_VTIP * (u->ped + 0.75 * a->tr_TWST) + vadv2t / m->tr_VTIP * (u->ped + 0.5 * a->tr_TWST);
    double thr_t = (vb - vi_tr) * rho * m->tr_COEF;
    double vi_tr_dot = F32(0.75 * M_PI / a->tr_R * (thr_t / (2 * M_PI * rho * a->tr_R * a->tr_R) -
                                                   vi_tr * sqrt(vadv2t + (vr - vi_tr) * (vr - vi_tr))));
    vi_tr_dot = F32(vi_tr_dot * 0.5);
    double power_tr = thr_t * (vi_tr - vr);
    double F_tr[3] = {0.0, F32(thr_t), 0.0};
    double M_tr[3] = {F32(thr_t * m->tr_H), 0.0, F32(-thr_t * m->tr_D)};

    /* ---- fuselage :302-320 */
    double wa_f = wa - vi_mr;
    if (wa_f > 0) wa_f += EPS_DYN;
    double d_fw = (ua / (-wa_f) * (m->mr_H - m->fus_H)) - (m->fus_D - m->mr_D);
    d_fw *= a->fus_COR;
    double rh = 0.5 * rho;
    double X_F = rh * a->fus_XUU * fabs(ua) * ua, Y_F = rh * a->fus_YVV * fabs(va) * va, Z_F = rh * a->fus_ZWW * fabs(wa_f) * wa_f;
    double power_fus = -X_F * ua - Y_F * va - Z_F * wa_f;
    double F_f[3] = {F32(X_F), F32(Y_F), F32(Z_F)};
    double M_f[3] = {F32(Y_F * m->fus_H), F32(Z_F * d_fw - X_F * m->fus_H), 0.0};

    /* ---- horizontal tail :322-345 */
    double v_dw = vi_mr - wa;
    if (v_dw < EPS_DYN) v_dw = EPS_DYN;
    double d_dw = (ua / v_dw * (m->mr_H - m->ht_H)) - (m->ht_D - m->mr_D - a->mr_R);
    double eps_ht = (d_dw > 0 && d_dw < a->mr_R) ? 2 * (1 - d_dw / a->mr_R) : 0.0;
    double wa_ht = wa - eps_ht * vi_mr + m->ht_D * pqr[1];
    double Z_HT;
    if (fabs(wa_ht) > 0.3 * fabs(ua)) {
        double vta = sqrt(ua * ua + va * va + wa_ht * wa_ht);
        Z_HT = 0.5 * rho * a->ht_ZMAX * fabs(vta) * wa_ht;
    } else {
        Z_HT = 0.5 * rho * (a->ht_ZUU * fabs(ua) * ua + a->ht_ZUW * fabs(ua) * wa_ht);
    }
    double F_ht[3] = {0.0, 0.0, F32(Z_HT)};
    double M_ht[3] = {0.0, F32(Z_HT * m->ht_D), 0.0};

    /* ---- vertical tail :347-361 */
    double va_vt = va + vi_tr - m->vt_D * pqr[2];
    double Y_VT;
    if (fabs(va_vt) > 0.3 * fabs(ua)) {
        double vta = sqrt(ua * ua + va_vt * va_vt);
        Y_VT = 0.5 * rho * a->vt_YMAX * fabs(vta) * va_vt;
    } else {
        Y_VT = 0.5 * rho * (a->vt_YUU * fabs(ua) * ua + a->vt_YUV * fabs(ua) * va_vt);
    }
    double F_vt[3] = {0.0, F32(Y_VT), 0.0};
    double M_vt[3] = {F32(Y_VT * m->vt_H), 0.0, F32(-Y_VT * m->vt_D)};

    /* ---- wing :363-383 */
    double X_WN = 0.0, Z_WN = 0.0;
    if (a->wn_ZUW != 0.0) {
        double wa_w = wa - vi_mr;
        double vta = sqrt(ua * ua + wa_w * wa_w);
        if (fabs(wa_w) > 0.3 * fabs(ua)) Z_WN = 0.5 * rho * a->wn_ZMAX * fabs(vta) * wa_w;
        else Z_WN = 0.5 * rho * (a->wn_ZUU * ua * ua + a->wn_ZUW * ua * wa_w);
        double q = a->wn_ZUU * ua * ua + a->wn_ZUW * ua * wa_w;
        X_WN = -0.5 * rho / M_PI / (vta * vta) * q * q;
    }
    double power_wn = fabs(X_WN * ua);
    double F_w[3] = {F32(X_WN), 0.0, F32(Z_WN)};

    /* ---- landing gear :385-398 (moment uses the ACCUMULATED force, :397) */
    double F_lg[3] = {0, 0, 0}, M_lg[3] = {0, 0, 0};
    double h_touch = h_c + a->WL_CG / 12;
    for (int g = 0; g < 3; g++) {
        const double* r = m->lg_loc[g];
        double wxr[3], pos[3], vel[3];
        cross(pqr, r, wxr);
        for (int i = 0; i < 3; i++) {
            float br = (float)B[0][i] * (float)r[0];   /* fp32 @ fp32 */
            br = br + (float)B[1][i] * (float)r[1];
            br = br + (float)B[2][i] * (float)r[2];
            pos[i] = xyz[i] + (double)br;
            vel[i] = ned[i] + (B[0][i] * wxr[0] + B[1][i] * wxr[1] + B[2][i] * wxr[2]);
        }
        double clearance = (-pos[2]) - h_touch;
        if (fabs(clearance) < g_lg_margin) g_lg_margin = fabs(clearance);
        if (clearance < 0.0) {
            double fz = -(a->lg_C * vel[2] + a->lg_K * (pos[2] + h_c)) + EPS_DYN;
            for (int i = 0; i < 3; i++) F_lg[i] += B[i][2] * fz;
            double mm[3];
            cross(r, F_lg, mm);
            for (int i = 0; i < 3; i++) M_lg[i] += mm[i];
        }
    }

    /* ---- totals :448-459 */
    double p_extra = power_climb + power_fus;
    M_mr[2] = F32(M_mr[2] + p_extra / m->mr_OMEGA);
    double power_total = power_mr + power_tr + p_extra + power_wn + 550 * a->HP_LOSS;
    double F[3], Mo[3];
    for (int i = 0; i < 3; i++) {
        double f = F32(F_mr[i] + F_tr[i]);
        f = F32(f + F_f[i]); f = F32(f + F_ht[i]); f = F32(f + F_vt[i]); f = F32(f + F_w[i]);
        F[i] = f + B[i][2] * a->WT + F_lg[i];
        double mo = F32(M_mr[i] + M_tr[i]);
        mo = F32(mo + M_f[i]); mo = F32(mo + M_ht[i]); mo = F32(mo + M_vt[i]); mo = F32(mo + 0.0);
        Mo[i] = mo + M_lg[i];
    }
    double pxu[3], Ip[3], pxIp[3], rhs[3];
    cross(pqr, uvw, pxu);
    for (int i = 0; i < 3; i++) Ip[i] = m->I[i][0] * pqr[0] + m->I[i][1] * pqr[1] + m->I[i][2] * pqr[2];
    cross(pqr, Ip, pxIp);
    for (int i = 0; i < 3; i++) rhs[i] = Mo[i] - pxIp[i];
    d[0] = vi_mr_dot;
    d[1] = vi_tr_dot;
    d[2] = F32(m->mr_OMEGA);
    d[3] = F32(m->tr_OMEGA);
    d[4] = b0_dot;
    d[5] = b1_dot;
    for (int i = 0; i < 3; i++) {
        d[6 + i] = F[i] / m->mass - pxu[i];
        d[9 + i] = m->IINV[i][0] * rhs[0] + m->IINV[i][1] * rhs[1] + m->IINV[i][2] * rhs[2];
        d[12 + i] = eul_dot[i];
        d[15 + i] = ned[i];
    }
    if (obs) {
        obs[0] = power_total / 550;
        for (int i = 0; i < 3; i++) {
            obs[1 + i] = uvwa[i];
            obs[4 + i] = ned[i];
            obs[7 + i] = eul[i];
            obs[10 + i] = pqr[i];
        }
        obs[13] = xyz[0];
        obs[14] = xyz[1];
        obs[15] = -xyz[2];
        obs[16] = -xyz[2] - h_c;
    }
}

/* Convenience: dynamics from fp32 actions (the step path). */
void or_dynamics(const or_model* m, const double s[18], const double act[4], const double W[3],
                 double h_c, double d[18], double* obs) {
    controls u = controls_f32(&m->cfg.af, act);
    or_dynamics_c(m, s, &u, W, h_c, d, obs);
}

/* HelicopterDynamics.step: dynamics.py:158-171 + step_after (helicopter_dynamics.py:73-77).
 * s is updated in place; k4 -> dots; obs from the stage-4 input state. */
/* Diagnostic (tests only, not the reference's semantics): round every RK stage input and the
 * updated state to float32, as an fp32 implementation stores them -- the rounding the parity tests'
 * altitude-ulp term is meant to bound. */
static int g_stage_f32 = 0;
void or_set_stage_f32(int on) { g_stage_f32 = on; }
static inline double SR(double x) { return g_stage_f32 ? F32(x) : x; }

void or_heli_step(const or_model* m, double s[18], const double act[4], const double W[3],
                  double dots[18], double obs[17], int state_f32) {
    controls u = controls_f32(&m->cfg.af, act);
    double dt = m->cfg.dt;
    double h_c = or_ground_height_p(m, s[15], s[16], state_f32);   /* committed xy (F6) */
    double k1[18], k2[18], k3[18], k4[18], st[18];
    or_dynamics_c(m, s, &u, W, h_c, k1, NULL);
    for (int i = 0; i < 18; i++) st[i] = SR(s[i] + k1[i] * (0.5 * dt));
    or_dynamics_c(m, st, &u, W, h_c, k2, NULL);
    for (int i = 0; i < 18; i++) st[i] = SR(s[i] + k2[i] * (0.5 * dt));
    or_dynamics_c(m, st, &u, W, h_c, k3, NULL);
    for (int i = 0; i < 18; i++) st[i] = SR(s[i] + k3[i] * dt);
    or_dynamics_c(m, st, &u, W, h_c, k4, obs);
    for (int i = 0; i < 18; i++) {
        s[i] = SR(s[i] + (k1[i] + k2[i] * 2 + k3[i] * 2 + k4[i]) * (0.16666666666666666 * dt));
        dots[i] = k4[i];
    }
    s[2] = or_pi_bound(s[2]);
    s[3] = or_pi_bound(s[3]);
    s[4] = or_pi_bound(s[4]);
    s[5] = or_pi_bound(s[5]);
    for (int i = 12; i < 15; i++) s[i] = or_pi_bound(s[i]);
}

/* ------------------------------------------------------------------ tasks and flags */

static double sgn(double x) { return (x > 0) - (x < 0); }

/* HeliHover._calculate_reward (helicopter_with_tasks.py:27-52) */
static double reward_hover(const or_model* m, const double s[18], const double d[18], int* success) {
    const hg_target* t = &m->cfg.target;
    double tgt[3] = {F32(t->north_loc) / m->n_x, F32(t->east_loc) / m->n_x, F32(-t->sea_alt) / m->n_x};
    tgt[0] = F32(tgt[0]); tgt[1] = F32(tgt[1]); tgt[2] = F32(tgt[2]);
    double pf = 0, pt = 0, xf = 0, xt = 0;
    for (int i = 0; i < 3; i++) {
        double pn = s[9 + i] * m->n_t, pdn = d[9 + i] * m->n_t * m->n_t;
        double xn = s[15 + i] / m->n_x, xdn = d[15 + i] / m->n_v;
        pf -= pn * pn;
        pt -= sgn(pn) * pdn;
        xf -= (xn - tgt[i]) * (xn - tgt[i]);
        xt -= sgn(xn - tgt[i]) * xdn;
    }
    *success = pf > -1.0 && xf > -1.0;
    return ((pf > pt ? pf : pt) + (xf > xt ? xf : xt)) / 2.0;
}

/* HeliForwardFlight._calculate_reward (helicopter_with_tasks.py:78-115) */
static double reward_ff(const or_model* m, const double s[18], const double d[18], int* success) {
    const hg_target* t = &m->cfg.target;
    double vel = sqrt(s[6] * s[6] + s[7] * s[7] + s[8] * s[8]);
    double vn = vel / m->n_v;
    double vdn = (s[6] * d[6] + s[7] * d[7] + s[8] * d[8]) / vel / m->n_a;
    double dn = s[17] / m->n_x, ddn = d[17] / m->n_v;
    /* np.array(vel, float32) / np.float64 -> float64; np.array(-alt, float32) / int -> float32 */
    double vt = F32(t->vel) / m->n_v, dt_ = F32(F32(-t->sea_alt) / m->n_x);
    double pf = 0, pt = 0;
    for (int i = 0; i < 3; i++) {
        double pn = s[9 + i] * m->n_t, pdn = d[9 + i] * m->n_t * m->n_t;
        pf -= pn * pn;
        pt -= sgn(pn) * pdn;
    }
    double vf = -(vn - vt) * (vn - vt), vtr = -sgn(vn - vt) * vdn;
    double df = -(dn - dt_) * (dn - dt_), dtr = -sgn(dn - dt_) * ddn;
    *success = pf > -1.0 && vf > -1.0 && df > -1.0;
    double pr = pf > pt ? pf : pt, vr = vf > vtr ? vf : vtr, dr = df > dtr ? df : dtr;
    return (pr + vr + dr) / 3.0;
}

/* Heli._is_failed (helicopter.py:226-234), post-step state and k4 dots. */
int or_is_failed(const or_model* m, const double s[18], const double d[18]) {
    const hg_airframe* a = &m->cfg.af;
    double gta = ground_touching_altitude(m, s[15], s[16], 0);
    int c1 = (-s[17]) - gta < 0.0;
    int c2 = d[17] > m->mr_VTIP * 0.05;
    int c3 = s[12] > 60 * D2R;
    int c4 = s[13] > 60 * D2R;
    int c5 = fabs(s[15]) > a->env_NS_MAX / 2 || fabs(s[16]) > a->env_EW_MAX / 2 || -s[17] > gta + 10000;
    return (c1 && (c2 || c3 || c4)) || c5;
}

/* ------------------------------------------------------------------ env step / reset */

/* Heli.step (helicopter.py:192-206) for one env with injected turbulence noise eta (the value of
 * wind_dyn.eta, i.e. randn(3)/sqrt(dt)). */
void or_step(const or_model* m, or_env* e, const double act[4], const double eta[3], or_out* o) {
    e->time_counter += m->cfg.dt;
    double carry[4] = {e->obs[4], e->obs[5], e->obs[6], e->obs[16]};
    or_wind_step(m, e->wind, carry, eta, o->wind_ned);
    or_heli_step(m, e->heli, act, o->wind_ned, e->dots, e->obs, e->state_f32);
    e->state_f32 = 0;
    memcpy(o->obs, e->obs, sizeof(o->obs));
    int sh, sf;
    o->reward_hover = reward_hover(m, e->heli, e->dots, &sh);
    o->reward_ff = reward_ff(m, e->heli, e->dots, &sf);
    o->success_hover = sh;
    o->success_ff = sf;
    int task = m->cfg.task, succ;
    if (task == HG_TASK_HOVER) { o->reward = o->reward_hover; succ = sh; }
    else if (task == HG_TASK_FORWARD_FLIGHT) { o->reward = o->reward_ff; succ = sf; }
    else { o->reward = 0.0; succ = 0; }
    o->failed = or_is_failed(m, e->heli, e->dots);
    o->successed = e->successed_time >= m->cfg.max_time / 4;      /* :236-237, :89-92 */
    o->time_up = e->time_counter > m->cfg.max_time;                 /* :239-240 */
    o->terminated = o->failed || o->successed;                      /* :203 (reward==nan never true) */
    o->truncated = o->time_up;
    if (succ) e->successed_time += m->cfg.dt;                       /* :205 */
}

/* ---- trim (helicopter_dynamics.py:491-576) ---- */

static void trim_fcn(const or_model* m, const double base[18], const double x[16], const double W[3],
                     double h_c, double y[16], double* state_out, double* dots_out, double* obs) {
    double s[18];
    memcpy(s, base, sizeof(s));
    /* __trim_fcn writes into a copy of the float32 state (:558-564) */
    s[0] = F32(x[0] * m->mr_VTIP);
    s[1] = F32(x[1] * m->tr_VTIP);
    s[4] = F32(x[2]); s[5] = F32(x[3]);
    for (int i = 0; i < 3; i++) { s[6 + i] = F32(x[4 + i] * m->mr_VTIP); s[9 + i] = F32(x[7 + i] * m->mr_OMEGA); }
    s[12] = F32(x[10]); s[13] = F32(x[11]);
    controls u = controls_f64(&m->cfg.af, x + 12);
    double d[18];
    or_dynamics_c(m, s, &u, W, h_c, d, obs);
    y[0] = d[0] / m->mr_VTIP;
    y[1] = d[1] / m->tr_VTIP;
    y[2] = d[4]; y[3] = d[5];
    for (int i = 0; i < 3; i++) {
        y[4 + i] = d[6 + i] / m->mr_VTIP;
        y[7 + i] = d[9 + i] / m->mr_OMEGA;
        y[10 + i] = d[12 + i];
        y[13 + i] = d[15 + i] / m->cfg.af.mr_R;
    }
    if (state_out) memcpy(state_out, s, sizeof(s));
    if (dots_out) memcpy(dots_out, d, sizeof(d));
}

/* 16x16 Gauss-Jordan inverse with partial pivoting, then v = A^-1 r (np.linalg.inv(dydx)@r). */
static int solve16(double A[16][16], const double r[16], double v[16]) {
    double M[16][32];
    for (int i = 0; i < 16; i++)
        for (int j = 0; j < 32; j++) M[i][j] = j < 16 ? A[i][j] : (j - 16 == i);
    for (int c = 0; c < 16; c++) {
        int p = c;
        for (int i = c + 1; i < 16; i++) if (fabs(M[i][c]) > fabs(M[p][c])) p = i;
        if (M[p][c] == 0.0) return -1;
        if (p != c) for (int j = 0; j < 32; j++) { double t = M[c][j]; M[c][j] = M[p][j]; M[p][j] = t; }
        double piv = M[c][c];
        for (int j = 0; j < 32; j++) M[c][j] /= piv;
        for (int i = 0; i < 16; i++) {
            if (i == c) continue;
            double f = M[i][c];
            if (f != 0.0) for (int j = 0; j < 32; j++) M[i][j] -= f * M[c][j];
        }
    }
    for (int i = 0; i < 16; i++) {
        double acc = 0;
        for (int j = 0; j < 16; j++) acc += M[i][16 + j] * r[j];
        v[i] = acc;
    }
    return 0;
}

/* HelicopterDynamics.trim (helicopter_dynamics.py:491-555) against wind W. */
int or_trim(const or_model* m, const hg_trim_cond* tc, const double W[3], hg_trim_result* out) {
    const hg_airframe* a = &m->cfg.af;
    double base[18] = {0};
    base[14] = F32(tc->yaw);
    base[2] = F32(tc->psi_mr);
    base[3] = F32(tc->psi_tr);
    base[15] = F32(tc->xy[0]);
    base[16] = F32(tc->xy[1]);
    double cg = -ground_touching_altitude(m, base[15], base[16], 1);
    base[17] = F32(cg - tc->gr_alt);
    double h_c = or_ground_height_p(m, base[15], base[16], 1);
    double yt[16] = {0};
    yt[12] = F32(tc->yaw_rate);
    for (int i = 0; i < 3; i++) yt[13 + i] = (double)((float)tc->ned_vel[i] / (float)a->mr_R);
    double x[16] = {0.05f, 0.05f, 0, 0, 0, 0, 0, 0, 0, F32(tc->yaw_rate), -0.01f, 0.01f, 0, 0, 0, 0};
    for (int i = 0; i < 3; i++) x[4 + i] = (double)((float)tc->ned_vel[i] / (float)m->mr_VTIP);
    double y[16], tol = 0;
    trim_fcn(m, base, x, W, h_c, y, NULL, NULL, NULL);
    for (int i = 0; i < 16; i++) tol += (y[i] - yt[i]) * (y[i] - yt[i]);
    int it = 0;
    while (tol > EPS_DYN) {
        double J[16][16], yp[16], ym[16], xp[16], xm[16], r[16], dir[16];
        for (int i = 0; i < 16; i++) {
            memcpy(xp, x, sizeof(x)); memcpy(xm, x, sizeof(x));
            xp[i] += EPS_DYN; xm[i] -= EPS_DYN;
            trim_fcn(m, base, xp, W, h_c, yp, NULL, NULL, NULL);
            trim_fcn(m, base, xm, W, h_c, ym, NULL, NULL, NULL);
            for (int k = 0; k < 16; k++) J[k][i] = (yp[k] - ym[k]) / (2 * EPS_DYN);
        }
        for (int k = 0; k < 16; k++) r[k] = y[k] - yt[k];
        if (solve16(J, r, dir)) return HG_E_TRIM;
        double step = 1.0, xn[16], yn[16], tn = 0;
        int j;
        for (j = 0; j < 10; j++) {
            for (int k = 0; k < 16; k++) xn[k] = x[k] - step * dir[k];
            trim_fcn(m, base, xn, W, h_c, yn, NULL, NULL, NULL);
            tn = 0;
            for (int k = 0; k < 16; k++) tn += (yn[k] - yt[k]) * (yn[k] - yt[k]);
            step *= 0.5;
            if (tn < tol) break;
        }
        if (j >= 9) break;      /* :540 — also when the 10th candidate improved */
        memcpy(x, xn, sizeof(x)); memcpy(y, yn, sizeof(y)); tol = tn;
        if (++it > 200) return HG_E_TRIM;   /* the reference asserts after 5 s (:543-544) */
    }
    trim_fcn(m, base, x, W, h_c, y, out->state, out->state_dots, out->obs);
    for (int i = 0; i < 4; i++) out->action[i] = x[12 + i];
    out->residual = tol;
    out->iterations = it;
    out->failed = or_is_failed(m, out->state, out->state_dots);
    return HG_OK;
}

/* Heli.reset (helicopter.py:208-217) from a trim result. */
void or_reset(const or_model* m, or_env* e, const hg_trim_result* tr) {
    (void)m;
    memcpy(e->heli, tr->state, sizeof(e->heli));
    memset(e->wind, 0, sizeof(e->wind));
    memcpy(e->obs, tr->obs, sizeof(e->obs));
    memcpy(e->dots, tr->state_dots, sizeof(e->dots));
    e->time_counter = 0;
    e->successed_time = 0;
    e->state_f32 = 1;
}

size_t or_env_size(void) { return sizeof(or_env); }
size_t or_out_size(void) { return sizeof(or_out); }

/* ---- CPU baseline: n envs x n_steps, U(-1,1) actions and N(0,1)/sqrt(dt) noise from a small
 * xorshift generator (not bitwise the product's Philox stream), auto-reset to the template.
 * Returns the number of env-steps executed.  Timed by bench.py as the "port" baseline. */
static inline uint64_t xs64(uint64_t* s) { uint64_t x = *s; x ^= x << 13; x ^= x >> 7; x ^= x << 17; return *s = x; }
static inline double u01(uint64_t* s) { return ((xs64(s) >> 11) + 0.5) * (1.0 / 9007199254740992.0); }

int64_t or_rollout(const or_model* m, const hg_trim_result* tr, int64_t n_envs, int64_t n_steps,
                   uint64_t seed, double* checksum) {
    int64_t done_steps = 0;
    double acc = 0;
    or_env e;
    or_out o;
    for (int64_t i = 0; i < n_envs; i++) {
        uint64_t s = seed * 0x9E3779B97F4A7C15ull + (uint64_t)i + 1;
        or_reset(m, &e, tr);
        for (int64_t t = 0; t < n_steps; t++) {
            double act[4], eta[3];
            for (int k = 0; k < 4; k++) act[k] = (double)(float)(2 * u01(&s) - 1);
            for (int k = 0; k < 3; k++) {
                double u1 = u01(&s), u2 = u01(&s);
                eta[k] = sqrt(-2 * log(u1)) * cos(2 * M_PI * u2) * m->eta_norm;
            }
            or_step(m, &e, act, eta, &o);
            acc += o.reward;
            done_steps++;
            if (o.terminated || o.truncated) or_reset(m, &e, tr);
        }
    }
    if (checksum) *checksum = acc;
    return done_steps;
}
