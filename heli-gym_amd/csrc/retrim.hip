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

#ifndef HG_TIMING
#define HG_TIMING 0
#endif
#if HG_TIMING
// diagnostic build: s_memtime at the phase boundaries of the first job's rounds (lane 0)
__device__ unsigned long long g_rt_timing[64];
#define RSTAMP(j, ...)                                                                \
    do {                                                                              \
        asm volatile("" ::__VA_ARGS__);                                               \
        const unsigned long long t_ = __builtin_amdgcn_s_memtime();                   \
        if (l == 0 && job == 0 && (j) < 64) g_rt_timing[(j)] = t_;                    \
    } while (0)
// sub-phases of the first two pivot steps of one solve (slots 40..51)
#define GJSTAMP(j, ...)                                                               \
    do {                                                                              \
        if (stamp && c < 2) {                                                         \
            asm volatile("" ::__VA_ARGS__);                                           \
            const unsigned long long t_ = __builtin_amdgcn_s_memtime();               \
            if (l == 0) g_rt_timing[40 + 6 * c + (j)] = t_;                           \
        }                                                                             \
    } while (0)
#else
#define RSTAMP(j, ...) do { } while (0)
#define GJSTAMP(j, ...) do { } while (0)
#endif

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

// hg::solve16 (np.linalg.inv(dydx) @ r, helicopter_dynamics.py:524-527) on the augmented matrix
// [J | r] (16 x 17 doubles, row-major) in LDS: Gauss-Jordan with partial pivoting in the host
// solver's operation order.  Every lane reads the pivot column (broadcast reads) and finds the
// pivot itself; lane e owns the elements e, e + 64, ... of the elimination, whose operands (the
// row's multiplier and the pivot row's element) are all read before any element is written.
constexpr int kGJElems = 16 * 17;

// The block is one wave, whose LDS operations execute in issue order: a read issued after a write
// sees it.  This only keeps the compiler from reordering LDS accesses across the point (no
// s_barrier, no wait for the LDS queue to drain).
__device__ __forceinline__ void lds_order() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}
constexpr int kGJPerLane = (kGJElems + 63) / 64;

__device__ __forceinline__ bool gauss_jordan(double* M, int l) {
    int ei[kGJPerLane], ej[kGJPerLane];   // row / column of this lane's elements
#pragma unroll
    for (int k = 0; k < kGJPerLane; ++k) {
        ei[k] = (l + 64 * k) / 17;
        ej[k] = (l + 64 * k) - 17 * ei[k];
    }
#pragma unroll
    for (int c = 0; c < 16; ++c) {
        int p = c;   // first row of maximal |M[i][c]| among rows c..15 (strict >, as the host)
        double mp = M[c * 17 + c];
#pragma unroll
        for (int i = c + 1; i < 16; ++i) {
            const double v = M[i * 17 + c];
            if (fabs(v) > fabs(mp)) { p = i; mp = v; }
        }
        if (mp == 0.0 || !isfinite(mp)) return false;
        if (p != c) {   // wave-uniform
            lds_order();
            if (l < 17) {
                const double t = M[c * 17 + l];
                M[c * 17 + l] = M[p * 17 + l];
                M[p * 17 + l] = t;
            }
        }
        lds_order();
        if (l >= c && l < 17) M[c * 17 + l] /= mp;   // the pivot row, j >= c
        lds_order();
        double f[kGJPerLane], pr[kGJPerLane];
#pragma unroll
        for (int k = 0; k < kGJPerLane; ++k) {
            const bool in = l + 64 * k < kGJElems;
            f[k] = in ? M[ei[k] * 17 + c] : 0.0;
            pr[k] = in ? M[c * 17 + ej[k]] : 0.0;
        }
        lds_order();
#pragma unroll
        for (int k = 0; k < kGJPerLane; ++k) {
            const int e = l + 64 * k;
            if (e < kGJElems && ei[k] != c && ej[k] >= c && f[k] != 0.0) M[e] -= f[k] * pr[k];
        }
        lds_order();
    }
    return true;
}

// The same elimination with the augmented matrix in registers: lane j (0..16) holds column j of
// [J | r] (m[i] = M[i][j]).  One pivot step C (a template parameter: every other array index is a
// compile-time constant): lane c's column goes to LDS while every lane searches its own column for
// the pivot (lane c's search is the step's; the others are discarded), the multipliers M[i][c] are
// read back with rows c and p already exchanged in the addressing while each lane swaps the two
// rows of its own column (a register-indexed move), and then each lane divides and eliminates its
// own column -- the LDS round trip hides behind the search and the swap.  Same operations in the same order as hg::solve16 (and as
// the LDS elimination above); an update the host skips (f == 0) is computed and discarded here.
template <int C>
__device__ __forceinline__ bool gj_step(double (&m)[16], double* colbuf, int l, bool stamp) {
    constexpr int c = C;
    (void)stamp;
    GJSTAMP(0, "v"(m[0]));
    if (l == c) {
#pragma unroll
        for (int i = 0; i < 16; ++i) colbuf[i] = m[i];
    }
    int pl = c;    // first row of maximal |M[i][c]| among rows c..15 (strict >, as the host)
    double mxl = m[c];
#pragma unroll
    for (int i = c + 1; i < 16; ++i)
        if (fabs(m[i]) > fabs(mxl)) { pl = i; mxl = m[i]; }
    const int p = __builtin_amdgcn_readlane(pl, c);
    const double mp = read_lane(mxl, c);        // the pivot M[p][c]
    GJSTAMP(1, "s"(p));
    if (__builtin_amdgcn_readfirstlane((int)(mp == 0.0 || !isfinite(mp)))) return false;
    lds_order();
    double f[16];                                // M[i][c] after the row exchange (f[c] unused)
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        if (i == c) continue;
        f[i] = i < c ? colbuf[i] : colbuf[i == p ? c : i];
    }
    lds_order();   // read before the next step's column is written
    GJSTAMP(2, "s"(p));
    {   // rows c and p exchange in every column: p is uniform, so this is a register-indexed move
        // (s_set_gpr_idx), not the 15 scalar branches of a test per row (one branch per row cost
        // 5 % more; a binary tree of branches put the arrays in scratch memory)
        const double t = m[p];
        m[p] = m[c];
        m[c] = t;
    }
    GJSTAMP(3, "v"(m[c]));
    const bool upd = l < 17 && l >= c;   // columns j >= c
    const double piv = m[c] / mp;
    m[c] = upd ? piv : m[c];
    GJSTAMP(4, "v"(m[c]));
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        if (i == c) continue;
        const double t = m[i] - f[i] * m[c];
        m[i] = (upd && f[i] != 0.0) ? t : m[i];
    }
    GJSTAMP(5, "v"(m[0]), "v"(m[15]));
    return true;
}
template <int C>
__device__ __forceinline__ bool gj_steps(double (&m)[16], double* colbuf, int l, bool stamp) {
    if (!gj_step<C>(m, colbuf, l, stamp)) return false;
    if constexpr (C < 15) return gj_steps<C + 1>(m, colbuf, l, stamp);
    return true;
}

// The 16 pivot steps of the register elimination.
__device__ __forceinline__ bool gauss_jordan_cols(double (&m)[16], double* colbuf, int l, bool stamp) {
    return gj_steps<0>(m, colbuf, l, stamp);
}

#ifndef HG_GJ_LDS
#define HG_GJ_LDS 0   // 1: the LDS elimination (A/B)
#endif

__device__ __forceinline__ void retrim_write(const RetrimArgs& a, int64_t job, int64_t env, const double x[16],
                                             const double s[18], const double ob[17]) {
    if (a.list) {
        for (int c = 0; c < 18; ++c) a.state[tix(env, c)] = (float)s[c];
        const int co[4] = {4, 5, 6, 16};
        for (int c = 0; c < 4; ++c) a.state[tix(env, 23 + c)] = (float)ob[co[c]];
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
#if HG_GJ_LDS
    __shared__ double M[kGJElems];   // [J | r] of the current Newton step
#else
    __shared__ double colbuf[16];    // the pivot column of the current elimination step
#endif
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
        int round = 0;
        RSTAMP(0, "v"(l));
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
            RSTAMP(1 + 4 * round, "v"(xe[0]));
            hg::trim_fcn(P, T.base, xe, W, T.hc, ye, se, de, oe);
            const double te = hg::trim_residual(ye, T.yt);
            RSTAMP(2 + 4 * round, "v"(te));
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
            // ---- Newton direction: lane j <= 16 holds column j of [J | r], then Gauss-Jordan
            double mcol[16];
#pragma unroll
            for (int k = 0; k < 16; ++k) {
                const double ym = shfl_d(ye[k], (l + 16) & 63);
                mcol[k] = l < 16 ? (ye[k] - ym) / (2 * eps) : y[k] - T.yt[k];
            }
#if HG_GJ_LDS
#pragma unroll
            for (int k = 0; k < 16; ++k)
                if (l < 17) M[k * 17 + l] = mcol[k];
            __syncthreads();
            RSTAMP(3 + 4 * round, "v"(ye[0]));
            ok = gauss_jordan(M, l);
            if (!ok) break;
#pragma unroll
            for (int k = 0; k < 16; ++k) dir[k] = M[k * 17 + 16];
            __syncthreads();   // dir read before the next round's matrix is written
#else
            RSTAMP(3 + 4 * round, "v"(mcol[0]));
            ok = gauss_jordan_cols(mcol, colbuf, l, job == 0 && round == 0);
            if (!ok) break;
#pragma unroll
            for (int k = 0; k < 16; ++k) dir[k] = read_lane(mcol[k], 16);
#endif
            RSTAMP(4 + 4 * round, "v"(dir[0]));
            ++round;
        }
        RSTAMP(63, "v"(l));
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

#if HG_TIMING
extern "C" int hg_debug_retrim_timing(void* dst, int64_t bytes) {
    return hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_rt_timing), (size_t)bytes) == hipSuccess ? 0 : -1;
}
#endif

hipError_t launch_retrim(const RetrimArgs& a, unsigned grid, hipStream_t stream) {
    hipLaunchKernelGGL(retrim_kernel, dim3(grid), dim3(64), 0, stream, a);
    return hipGetLastError();
}

}  // namespace hgk
