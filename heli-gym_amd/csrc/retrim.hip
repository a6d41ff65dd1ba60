// retrim.hip — the device batched Newton trim: exact second-episode resets (reset_mode RETRIM,
// SURVEY F8), hg_trim_batch and hg_trim_conds_batch.
//
// Its own translation unit, compiled with -ffp-contract=off: the reference's trim is numpy without
// fused multiply-adds and its stopping point depends on the Newton path (an ill-conditioned
// system stopped at ||y - y*||^2 <= 1e-4), so the device evaluates exactly the host's operation
// sequence (heligym_amd.hip::do_trim, which reproduces the reference's trims) instead of a fused
// one whose different roundings can change a line-search decision.
#include "../../include/heligym_amd.h"
#include "retrim.h"

namespace hgk {
namespace {

// HelicopterDynamics.trim (helicopter_dynamics.py:491-555) for many winds at once: the reset path of
// reset_mode RETRIM (F8) and hg_trim_batch.  One wave per trim, fp64 throughout, every lane holding
// the same Newton iterate:
//   * lanes 0..15 / 16..31 evaluate the +eps / -eps Jacobian columns in parallel;
//   * lane j <= 16 then holds column j of [J | r] in registers and the Gauss-Jordan elimination
//     (hg::solve16, same operation order) runs with the pivot column broadcast by readlane;
//   * lanes 0..9 evaluate the ten step-halving trials at once; the first one that lowers the
//     residual is the trial the reference's sequential search accepts.


__device__ __forceinline__ double read_lane(double v, int lane) {
    const uint64_t u = __double_as_longlong(v);
    const uint32_t lo = __builtin_amdgcn_readlane((int)(uint32_t)u, lane);
    const uint32_t hi = __builtin_amdgcn_readlane((int)(uint32_t)(u >> 32), lane);
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}
__device__ __forceinline__ double shfl_d(double v, int src) {
    const uint64_t u = __double_as_longlong(v);
    const uint32_t lo = __shfl((int)(uint32_t)u, src);
    const uint32_t hi = __shfl((int)(uint32_t)(u >> 32), src);
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}

__device__ __forceinline__ void retrim_write(const RetrimArgs& a, int64_t job, int64_t env, const double x[16],
                                             const double s[18], const double ob[17]) {
    if (a.list) {
        for (int c = 0; c < 18; ++c) a.state[(int64_t)c * a.n + env] = (float)s[c];
        const int co[4] = {4, 5, 6, 16};
        for (int c = 0; c < 4; ++c) a.state[(int64_t)(23 + c) * a.n + env] = (float)ob[co[c]];
        if (a.obs)
            for (int c = 0; c < 17; ++c) a.obs[env * 17 + c] = (float)ob[c];
    } else {
        if (a.out_state)
            for (int c = 0; c < 18; ++c) a.out_state[job * 18 + c] = (float)s[c];
        if (a.out_action)
            for (int c = 0; c < 4; ++c) a.out_action[job * 4 + c] = (float)x[12 + c];
        if (a.out_obs)
            for (int c = 0; c < 17; ++c) a.out_obs[job * 17 + c] = (float)ob[c];
    }
    if (a.out_status) a.out_status[job] = HG_OK;
}

// Lane roles per evaluation round: lanes 0..31 the Jacobian columns at the point the next Newton
// step will start from, lanes 32..41 the ten step-halving trials of the current step (trial 0,
// the full step, is that point whenever the search accepts it, which it usually does), lane 32
// alone the residual at x0 in the first round.  A round is one trim_fcn latency; a trim of three
// Newton steps takes four rounds.
__global__ __launch_bounds__(64) void retrim_kernel(const RetrimArgs a) {
    const int l = threadIdx.x;
    const hg::Params<double>& P = *a.P;
    const double eps = hg::kTrimEps;
    const int64_t jobs = a.count ? (int64_t)*a.count : a.njobs;
    for (int64_t job = blockIdx.x; job < jobs; job += gridDim.x) {   // uniform per wave
        const int64_t env = a.list ? (int64_t)a.list[job] : job;
        const hg::TrimSetup& T = a.T[a.setup_stride ? job : 0];
        double W[3] = {P.wm[0], P.wm[1], P.wm[2]};   // NULL wind: the mean wind (helicopter.py:55)
        if (a.wind) {
            const float* wr = a.wind + 3 * (a.list ? env : job);
            W[0] = (double)wr[0];
            W[1] = (double)wr[1];
            W[2] = (double)wr[2];
        }
        double x[16], y[16], dir[16];
        for (int k = 0; k < 16; ++k) { x[k] = T.x0[k]; dir[k] = 0.0; }
        double tol = 0;
        int it = 0;
        bool ok = true, done = false, first = true, have_jac = false;
        while (!done) {
            // ---- one evaluation round
            const int c = l & 15;
            const int j = l - 32;   // line-search trial of this lane (0..9), first round: base point
            double xe[16];
            if (l < 32) {   // Jacobian columns at x - dir (= x in the first round)
                for (int k = 0; k < 16; ++k) {
                    const double xs = first ? x[k] : x[k] - 1.0 * dir[k];
                    xe[k] = k == c ? (l < 16 ? xs + eps : xs - eps) : xs;
                }
            } else {
                const double step = (j >= 0 && j < hg::kTrimLineSearch) ? ldexp(1.0, -j) : 0.0;
                for (int k = 0; k < 16; ++k) xe[k] = first ? x[k] : x[k] - step * dir[k];
            }
            double ye[16], se[18], de[18], oe[17];
            hg::trim_fcn(P, T.base, xe, W, T.hc, ye, se, de, oe);
            const double te = hg::trim_residual(ye, T.yt);
            // ---- accept a trial (or take the base point)
            int src = 32;   // lane whose evaluation is the new iterate
            if (first) {
                first = false;
                have_jac = true;
            } else {
                int js = hg::kTrimLineSearch;
                for (int jj = hg::kTrimLineSearch - 1; jj >= 0; --jj)
                    if (read_lane(te, 32 + jj) < tol) js = jj;
                if (js >= hg::kTrimLineSearch - 1) {   // helicopter_dynamics.py:540: keep x
                    done = true;
                    src = -1;
                } else {
                    const double step = ldexp(1.0, -js);
                    for (int k = 0; k < 16; ++k) x[k] = x[k] - step * dir[k];
                    src = 32 + js;
                    have_jac = js == 0;   // the Jacobian lanes evaluated around trial 0
                    if (++it > hg::kTrimMaxIter) { ok = false; done = true; src = -1; }
                }
            }
            if (src >= 0) {
                for (int k = 0; k < 16; ++k) y[k] = read_lane(ye[k], src);
                tol = read_lane(te, src);
                if (!(tol > eps)) {   // converged: the accepting lane holds the final evaluation
                    done = true;
                    if (l == src) retrim_write(a, job, env, x, se, oe);
                    break;
                }
            }
            if (done) break;
            if (!have_jac) {   // the search accepted a shorter step: Jacobian at the new x
                if (l < 32) {
                    for (int k = 0; k < 16; ++k) xe[k] = k == c ? (l < 16 ? x[k] + eps : x[k] - eps) : x[k];
                    hg::trim_fcn(P, T.base, xe, W, T.hc, ye, nullptr, nullptr, nullptr);
                }
            }
            // ---- Newton direction: Gauss-Jordan (hg::solve16), lane j <= 16 owns column j of [J | r]
            double col[16];
            for (int k = 0; k < 16; ++k) {
                const double ym = shfl_d(ye[k], (l + 16) & 63);
                col[k] = l < 16 ? (ye[k] - ym) / (2 * eps) : y[k] - T.yt[k];
            }
#pragma unroll
            for (int cc = 0; cc < 16; ++cc) {
                double bc[16];   // column cc, broadcast to every lane
#pragma unroll
                for (int k = 0; k < 16; ++k) bc[k] = read_lane(col[k], cc);
                int p = cc;
#pragma unroll
                for (int i = cc + 1; i < 16; ++i)
                    if (fabs(bc[i]) > fabs(bc[p])) p = i;
                p = __builtin_amdgcn_readfirstlane(p);
                double mp = bc[cc];
#pragma unroll
                for (int i = cc + 1; i < 16; ++i)
                    if (i == p) mp = bc[i];
                if (mp == 0.0 || !isfinite(mp)) { ok = false; break; }
                if (p != cc) {
#pragma unroll
                    for (int i = cc + 1; i < 16; ++i)
                        if (i == p) {
                            double t = col[cc]; col[cc] = col[i]; col[i] = t;
                            t = bc[cc]; bc[cc] = bc[i]; bc[i] = t;
                        }
                }
                const double piv = bc[cc];
                if (l >= cc) col[cc] /= piv;
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    if (i == cc) continue;
                    const double f = bc[i];
                    if (l >= cc && f != 0.0) col[i] -= f * col[cc];
                }
            }
            if (!ok) break;
#pragma unroll
            for (int k = 0; k < 16; ++k) dir[k] = read_lane(col[k], 16);
        }
        if (ok && done && l == 0) {
            // the search stopped without converging (:540): final evaluation at the kept x
            bool written = !(tol > eps);
            if (!written) {
                double yy[16], s[18], d[18], ob[17];
                hg::trim_fcn(P, T.base, x, W, T.hc, yy, s, d, ob);
                retrim_write(a, job, env, x, s, ob);
            }
        }
        if (!ok && l == 0) {
            if (a.fail_count) atomicAdd(a.fail_count, 1);
            if (a.out_status) a.out_status[job] = HG_E_TRIM;
        }
    }
}


}  // namespace

hipError_t launch_retrim(const RetrimArgs& a, unsigned grid, hipStream_t stream) {
    hipLaunchKernelGGL(retrim_kernel, dim3(grid), dim3(64), 0, stream, a);
    return hipGetLastError();
}

}  // namespace hgk
