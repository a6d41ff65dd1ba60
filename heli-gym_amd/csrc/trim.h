// trim.h — the reference's Newton trim (HelicopterDynamics.trim / __trim_fcn,
// heligym/envs/dynamics/helicopter_dynamics.py:491-576) as __host__ __device__ pieces.
//
// The host runs it serially for the reset template and hg_trim; the device re-trim kernel
// (exact second-episode resets) runs the same pieces with the finite-difference
// Jacobian columns and the line-search trials spread over lanes.  All arithmetic is fp64 with
// the trial point rounded to fp32, as the reference writes it into its float32 state array.
#pragma once

#include "physics.h"

namespace hg {

constexpr double kTrimEps = 1e-4;    // FD step and convergence threshold (:495, :517)
constexpr int kTrimMaxIter = 200;    // the reference gives up after 5 s of wall time (:543-544)
constexpr int kTrimLineSearch = 10;  // step-halving trials per Newton step (:530-540)

// Everything that depends only on the trim condition and the terrain, not on the wind.
struct TrimSetup {
    double base[18];     // state with the fixed entries set: psi_mr, psi_tr, yaw, x, y, z (:498-506)
    double yt[16];       // target normalised derivatives: yaw rate and ned velocity / R (:508-512)
    double x0[16];       // initial guess (:513-516)
    Ground<double> hc;   // ground under the trim position (committed xy)
    // functions of the fixed entries alone, evaluated once per trim condition (trim_precompute):
    double rho_irho[2];  // density at the trim altitude and its reciprocal
    double s_psi, c_psi; // sin / cos of the fixed yaw
    // the pivot order partial pivoting took in the host's trim of this condition at the mean wind,
    // per Newton step (the 4th for every later one): piv[k][C] = the row that pivots column C.  The
    // device trim's solve tries it first (gj_mfma.h gjs_solve; piv[0][0] < 0: no order, search).
    int8_t piv[4][16];
};

// The per-condition constants of TrimSetup, from its base state (the same functions the model
// would evaluate on every trial point).
HD void trim_precompute(const Params<double>& P, TrimSetup& t) {
    t.rho_irho[0] = atmosphere_rho(P, t.base[17]);
    t.rho_irho[1] = m_rcp(t.rho_irho[0]);
    m_sincos(t.base[14], &t.s_psi, &t.c_psi);
}

// Trial state for the unknowns x = [vi_mr/Vtip, vi_tr/Vtip_tr, b0, b1, uvw/Vtip, pqr/Omega,
// phi, theta, a0..a3] (:557-566), rounded to float like the reference's float32 state.
HD void trim_state(const Params<double>& P, const double base[18], const double x[16], double s[18]) {
    for (int i = 0; i < 18; ++i) s[i] = base[i];
    s[0] = (float)(x[0] * P.mr_VTIP);
    s[1] = (float)(x[1] * P.tr_VTIP);
    s[4] = (float)x[2];
    s[5] = (float)x[3];
    for (int i = 0; i < 3; ++i) {
        s[6 + i] = (float)(x[4 + i] * P.mr_VTIP);
        s[9 + i] = (float)(x[7 + i] * P.mr_OMEGA);
    }
    s[12] = (float)x[10];
    s[13] = (float)x[11];
}

// __trim_fcn (:557-576): normalised derivatives y(x) at the trial point; optionally the trial
// state, its derivatives and the observation (the final evaluation gives the reset state).
HD void trim_fcn(const Params<double>& P, const TrimSetup& T, const double x[16], const double W[3],
                 double y[16], double* s_out, double* d_out, double* obs) {
    double s[18], d[18], ob[17];
    trim_state(P, T.base, x, s);
    const Controls<double> u = controls(P, x[12], x[13], x[14], x[15]);
    Attitude<double> att;   // phi, theta are trial values; the yaw is fixed
    m_sincos(s[12], &att.s[0], &att.c[0]);
    m_sincos(s[13], &att.s[1], &att.c[1]);
    att.s[2] = T.s_psi;
    att.c[2] = T.c_psi;
    dynamics<true>(P, s, u, W, T.hc, att, d, ob, T.rho_irho);
    y[0] = m_div_c(d[0], P.mr_VTIP, P.mr_inv_VTIP);
    y[1] = m_div_c(d[1], P.tr_VTIP, P.tr_inv_VTIP);
    y[2] = d[4];
    y[3] = d[5];
    for (int i = 0; i < 3; ++i) {
        y[4 + i] = m_div_c(d[6 + i], P.mr_VTIP, P.mr_inv_VTIP);
        y[7 + i] = m_div_c(d[9 + i], P.mr_OMEGA, P.mr_inv_OMEGA);
        y[10 + i] = d[12 + i];
        y[13 + i] = m_div_c(d[15 + i], P.mr_R, P.mr_inv_R);
    }
    if (s_out)
        for (int i = 0; i < 18; ++i) s_out[i] = s[i];
    if (d_out)
        for (int i = 0; i < 18; ++i) d_out[i] = d[i];
    if (obs)
        for (int i = 0; i < 17; ++i) obs[i] = ob[i];
}

HD double trim_residual(const double y[16], const double yt[16]) {
    double t = 0;
    for (int i = 0; i < 16; ++i) t += (y[i] - yt[i]) * (y[i] - yt[i]);
    return t;
}

// np.linalg.inv(dydx) @ r (:524-527) via Gauss-Jordan with partial pivoting.  Returns false for a
// singular or non-finite pivot.
HD bool solve16(double A[16][16], const double r[16], double v[16], int8_t* piv = nullptr) {
    double M[16][17];
    int8_t idx[16];   // the original row now in row i (piv: the row that pivoted column i)
    for (int i = 0; i < 16; ++i) idx[i] = (int8_t)i;
    for (int i = 0; i < 16; ++i) {
        for (int j = 0; j < 16; ++j) M[i][j] = A[i][j];
        M[i][16] = r[i];
    }
    for (int c = 0; c < 16; ++c) {
        int p = c;
        for (int i = c + 1; i < 16; ++i)
            if (fabs(M[i][c]) > fabs(M[p][c])) p = i;
        if (M[p][c] == 0.0 || !isfinite(M[p][c])) return false;
        if (p != c) {
            for (int j = 0; j < 17; ++j) {
                const double t = M[c][j];
                M[c][j] = M[p][j];
                M[p][j] = t;
            }
            const int8_t t = idx[c];
            idx[c] = idx[p];
            idx[p] = t;
        }
        const double rinv = 1.0 / M[c][c];   // one division per pivot step (the device's too)
        for (int j = c; j < 17; ++j) M[c][j] *= rinv;
        for (int i = 0; i < 16; ++i) {
            if (i == c) continue;
            const double f = M[i][c];
            if (f != 0.0)
                for (int j = c; j < 17; ++j) M[i][j] -= f * M[c][j];
        }
    }
    for (int i = 0; i < 16; ++i) v[i] = M[i][16];
    if (piv)
        for (int i = 0; i < 16; ++i) piv[i] = idx[i];
    return true;
}

}  // namespace hg
