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
#ifndef HG_GJ_FLOW   // Gauss-Jordan pivot steps without per-step early exits (see gj_step)
#define HG_GJ_FLOW 1
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
//   * the Gauss-Jordan elimination of [J | r] (hg::solve16, same operation order) runs over the
//     whole wave, four lanes per row (gauss_jordan_wave);
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

// hg::solve16 (np.linalg.inv(dydx) @ r, helicopter_dynamics.py:524-527): Gauss-Jordan with partial
// pivoting on the augmented matrix [J | r] spread over the whole wave.  Lane l = 16 q + i holds row i
// of columns 4q .. 4q+3 and of the right-hand side (a[0..3], a[4]; the right-hand side is kept by all
// four lanes of a row, which compute it identically), so a DPP row of 16 lanes is one column
// quarter.  Per pivot step C:
//   * the pivot search is a 4-level DPP rotation max over the 16 rows of column C (in the row of
//     lanes that holds it) instead of a serial scan, and a ballot of the rows attaining it;
//   * rows are never moved: every row carries its position in the host's row order (`pos`, the
//     same in its four lanes), exchanged by the pivot step as the host exchanges the rows, and the
//     search breaks ties by that position, so the pivot is the host's (first row of maximal |M[i][C]|
//     among positions C..15, strict >);
//   * the multiplier M[i][C] (from the lane of this row that holds column C) and the pivot row's
//     elements (from the lane of the pivot row that holds this lane's columns) are two ds_bpermute
//     reads; the first is issued before the search, as it does not depend on the pivot;
//   * each lane scales the pivot row by 1/pivot and eliminates its own five elements.
// The values of columns >= C and of the right-hand side are the host's bit for bit (hg::solve16 in
// the same operation order, unfused); columns < C, which the host leaves alone and never reads
// again, are updated here too and ignored.  The solution is the right-hand side in host order.
// The block is one wave, whose LDS operations execute in issue order: a read issued after a write
// sees it.  This only keeps the compiler from reordering LDS accesses across the point (no
// s_barrier, no wait for the LDS queue to drain).
__device__ __forceinline__ void lds_order() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

// Rotate a double within each row of 16 lanes (DPP row_ror: every lane has a source, so no
// "old" operand is needed); n is a compile-time constant after inlining.
__device__ __forceinline__ double ror16_d(double v, int n) {
    const uint64_t u = __double_as_longlong(v);
    int lo = (int)(uint32_t)u, hi = (int)(uint32_t)(u >> 32);
    switch (n) {
        case 8: lo = __builtin_amdgcn_mov_dpp(lo, 0x128, 0xF, 0xF, true); hi = __builtin_amdgcn_mov_dpp(hi, 0x128, 0xF, 0xF, true); break;
        case 4: lo = __builtin_amdgcn_mov_dpp(lo, 0x124, 0xF, 0xF, true); hi = __builtin_amdgcn_mov_dpp(hi, 0x124, 0xF, 0xF, true); break;
        case 2: lo = __builtin_amdgcn_mov_dpp(lo, 0x122, 0xF, 0xF, true); hi = __builtin_amdgcn_mov_dpp(hi, 0x122, 0xF, 0xF, true); break;
        default: lo = __builtin_amdgcn_mov_dpp(lo, 0x121, 0xF, 0xF, true); hi = __builtin_amdgcn_mov_dpp(hi, 0x121, 0xF, 0xF, true); break;
    }
    return __longlong_as_double((long long)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo));
}
// v_max_f64 without the canonicalising maxes fmax() adds (the operands here are never NaN)
__device__ __forceinline__ double vmax_d(double a, double b) {
    double r;
    asm("v_max_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}

template <int C>
__device__ __forceinline__ bool gj_step(double (&a)[5], int& pos, int l, bool stamp) {
    constexpr int c = C, qc = C >> 2, tc = C & 3;
    (void)stamp;
    (void)c;
    const int i = l & 15, q = l >> 4;
    GJSTAMP(0, "v"(a[0]));
    const double f = shfl_d(a[tc], 16 * qc + i);   // M[i][C] of this lane's row
    const double v = a[tc];                         // M[i][4q + tc]; row of lanes qc: column C
    const bool nan_v = v != v;
    const bool cand = pos >= C && !nan_v;
    const double key = cand ? fabs(v) : -1.0;
    double mx = key;                                // max |M[i][C]| over the candidate rows
#pragma unroll
    for (int sh = 8; sh >= 1; sh >>= 1) mx = vmax_d(mx, ror16_d(mx, sh));
    // the rows that attain it (usually one); ties go to the smallest host position
    const uint32_t hit = (uint32_t)(__ballot(cand && key == mx) >> (16 * qc)) & 0xFFFFu;
    int P = hit ? __builtin_ctz(hit) : 0;
    int ppos = __builtin_amdgcn_readlane(pos, 16 * qc + P);
    if (hit & (hit - 1)) {   // wave-uniform, rare
        for (uint32_t m = hit & (hit - 1); m; m &= m - 1) {
            const int b = __builtin_ctz(m);
            const int pb = __builtin_amdgcn_readlane(pos, 16 * qc + b);
            if (pb < ppos) { ppos = pb; P = b; }
        }
    }
    const double mp = read_lane(v, 16 * qc + P);    // the pivot M[P][C]
    double pr[5];
#pragma unroll
    for (int t = 0; t < 5; ++t) pr[t] = shfl_d(a[t], 16 * q + P);   // the pivot row
    // the host's first candidate M[C][C] being NaN keeps it as the (non-finite) pivot
    const bool c_nan = __ballot(q == qc && pos == C && nan_v) != 0;
    GJSTAMP(1, "s"(P));
    const bool bad = !hit || c_nan || mp == 0.0 || !isfinite(mp);
#if HG_GJ_FLOW
    // No branch on a failed pivot step: it is reported after the last step (the steps in between
    // compute values nobody reads), so a step's remaining eliminations and the next step's pivot
    // search share a basic block and the scheduler overlaps them.
#else
    if (bad) return false;
    __builtin_amdgcn_sched_barrier(0);   // the pivot-row reads are in flight during the division
#endif
    const double rinv = 1.0 / mp;
#pragma unroll
    for (int t = 0; t < 5; ++t) pr[t] *= rinv;
    GJSTAMP(2, "v"(pr[0]), "v"(pr[4]));
    const bool is_piv = i == P;
#pragma unroll
    for (int t = 0; t < 5; ++t) {
        const double u = a[t] - f * pr[t];
        a[t] = is_piv ? pr[t] : (f != 0.0 ? u : a[t]);
    }
    pos = pos == ppos ? C : (pos == C ? ppos : pos);
    GJSTAMP(3, "v"(a[0]), "v"(a[4]));
    return !bad;
}
template <int C>
__device__ __forceinline__ bool gj_steps(double (&a)[5], int& pos, int l, bool stamp) {
#if HG_GJ_FLOW
    const bool ok = gj_step<C>(a, pos, l, stamp);
    if constexpr (C < 15) {
        const bool rest = gj_steps<C + 1>(a, pos, l, stamp);
        return ok && rest;
    }
    return ok;
#else
    if (!gj_step<C>(a, pos, l, stamp)) return false;
    if constexpr (C < 15) return gj_steps<C + 1>(a, pos, l, stamp);
    return true;
#endif
}

// The Newton system arrives in LDS as the raw evaluations: E[j][k] = y_k at x + eps e_j (j < 16) and
// at x - eps e_{j-16} (16 <= j < 32), R[k] = y_k - y*_k.  Each lane forms its own four Jacobian
// elements (J[i][j] = (E[j][i] - E[j+16][i]) / (2 eps), helicopter_dynamics.py:521-523, the host's
// operation) and right-hand side, so the 256 divisions are spread over the wave (4 per lane); the
// solution leaves through `sol` in host row order.
__device__ __forceinline__ bool gauss_jordan_wave(const double* E, const double* R, double* sol, int l, bool stamp,
                                                  double (&dir)[16]) {
    const int i = l & 15, q = l >> 4;
    const double eps = hg::kTrimEps;
    double a[5];
#pragma unroll
    for (int t = 0; t < 4; ++t) a[t] = (E[(4 * q + t) * 16 + i] - E[(4 * q + t + 16) * 16 + i]) / (2 * eps);
    a[4] = R[i];
    int pos = i;
    if (!gj_steps<0>(a, pos, l, stamp)) return false;
    if (l < 16) sol[pos] = a[4];
    lds_order();
#pragma unroll
    for (int k = 0; k < 16; ++k) dir[k] = sol[k];
    return true;
}

__device__ __forceinline__ void retrim_write(const RetrimArgs& a, int64_t job, int64_t env, const double x[16],
                                             const double s[18], const double ob[17]) {
    if (a.list) {
        for (int c = 0; c < 18; ++c)
            if (has_slot(c)) a.state[tix(env, c)] = (float)s[c];
        const int32_t epi = reinterpret_cast<const int32_t*>(a.state)[tix(env, kCtrCol0 + 2)];
        a.az[env] = AzRec{(float)s[kAzCol0], (float)s[kAzCol0 + 1], 0, epi};   // the reset's step 0
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
    __shared__ double gjE[32 * 16];   // the +-eps evaluations of the current Newton step
    __shared__ double gjR[16];        // its right-hand side y - y*
    __shared__ double gjS[16];        // its solution
    const int l = threadIdx.x;
    const hg::Params<double>& P = *a.P;
    const double eps = hg::kTrimEps;
    int64_t jobs = a.count ? (int64_t)*a.count : a.njobs;
    if (a.count && jobs > a.n) jobs = a.n;   // a queue holds at most one job per env
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
        double x[16], dir[16];
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
            hg::trim_fcn(P, T, xe, W, ye, se, de, oe);
            const double te = hg::trim_residual(ye, T.yt);
            RSTAMP(2 + 4 * round, "v"(te));
            // ---- accept a trial (or take the base point)
            int src = 32;   // lane whose evaluation is the new iterate
            if (first) {
                first = false;
                have_jac = true;
            } else {
                // the first trial (lanes 32 + j) whose residual is below tol: one ballot instead of a
                // readlane per trial (the reference's sequential search, helicopter_dynamics.py:532-541)
                const unsigned long long lower = __ballot(j >= 0 && j < hg::kTrimLineSearch && te < tol) >> 32;
                const int js = lower ? __builtin_ctzll(lower) : hg::kTrimLineSearch;
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
                    hg::trim_fcn(P, T, xe, W, ye, nullptr, nullptr, nullptr);
                }
            }
            // ---- Newton direction: the evaluations and the residual (lane src holds y) into LDS,
            // then Gauss-Jordan over the wave
            lds_order();   // the previous solve's reads are done
            if (l < 32) {
#pragma unroll
                for (int k = 0; k < 16; ++k) gjE[l * 16 + k] = ye[k];
            }
            if (l == src) {
#pragma unroll
                for (int k = 0; k < 16; ++k) gjR[k] = ye[k] - T.yt[k];
            }
            lds_order();
            RSTAMP(3 + 4 * round, "v"(ye[0]));
            ok = gauss_jordan_wave(gjE, gjR, gjS, l, job == 0 && round == 0, dir);
            if (!ok) break;
            RSTAMP(4 + 4 * round, "v"(dir[0]));
            ++round;
        }
        RSTAMP(63, "v"(l));
        if (ok && done && l == 0) {
            // the search stopped without converging (:540): final evaluation at the kept x
            bool written = !(tol > eps);
            if (!written) {
                double yy[16], s[18], d[18], ob[17];
                hg::trim_fcn(P, T, x, W, yy, s, d, ob);
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
