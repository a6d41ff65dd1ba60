// retrim_body.h -- the device batched Newton trim's per-job body (HelicopterDynamics.trim,
// helicopter_dynamics.py:491-555), shared by retrim.hip's retrim_kernel and the overlapped next-step
// re-trim kernel of heligym_amd.hip.  Both translation units build it with -ffp-contract=on (fused
// multiply-adds per source expression, decided by the front end), so the two kernels round every
// trim identically.
#pragma once

#include "retrim.h"
#include "gj_mfma.h"

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
#else
#define RSTAMP(j, ...) do { } while (0)
#endif
#if HG_TIMING
// diagnostic build: a fused launch's trim waves, per job (< 1024): s_memrealtime at the claim, at the
// record's arrival and at the write-out
__device__ unsigned long long g_fused_probe[1024][4];
#define FSTAMP(k) do { if (FUSED && l == 0 && job < 1024) g_fused_probe[job][(k)] = __builtin_amdgcn_s_memrealtime(); } while (0)
#else
#define FSTAMP(k) do { } while (0)
#endif

__device__ __forceinline__ double read_lane(double v, int lane) {
    const uint64_t u = __double_as_longlong(v);
    const uint32_t lo = __builtin_amdgcn_readlane((int)(uint32_t)u, lane);
    const uint32_t hi = __builtin_amdgcn_readlane((int)(uint32_t)(u >> 32), lane);
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}

// The wave is the block: its LDS operations execute in issue order, so a read issued after a write
// sees it.  This only keeps the compiler from reordering LDS accesses across the point.
__device__ __forceinline__ void lds_order() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

// 1 / x for a finite non-zero x: v_rcp_f64 and two Newton steps (fused), within an ulp
__device__ __forceinline__ double rcp_f64(double x) {
    double r = __builtin_amdgcn_rcp(x);
    r = fma(r, fma(-x, r, 1.0), r);
    return fma(r, fma(-x, r, 1.0), r);
}

// max of a 32-bit key over each row of 16 lanes (DPP row rotations; every lane has a source)
__device__ __forceinline__ uint32_t row16_max(uint32_t k) {
    k = max(k, (uint32_t)__builtin_amdgcn_mov_dpp((int)k, 0x128, 0xF, 0xF, true));
    k = max(k, (uint32_t)__builtin_amdgcn_mov_dpp((int)k, 0x124, 0xF, 0xF, true));
    k = max(k, (uint32_t)__builtin_amdgcn_mov_dpp((int)k, 0x122, 0xF, 0xF, true));
    k = max(k, (uint32_t)__builtin_amdgcn_mov_dpp((int)k, 0x121, 0xF, 0xF, true));
    return k;
}

// np.linalg.inv(dydx) @ r (helicopter_dynamics.py:524-527) as Gauss-Jordan with partial pivoting,
// one row per lane: lane l holds row i = l & 15 of [J | r] (the four rows of 16 lanes are identical
// copies).  Per pivot step C (unrolled, so every column index is a register):
//   * the pivot is the unused row with the largest |J[i][C]|, found with a DPP max over the 16 rows
//     on the high word of |J[i][C]| (monotonic in |x|; rows within 2^-20 of the maximum tie and the
//     lowest row wins: any of them is as good a pivot, partial pivoting only needs a large one);
//   * the pivot row is read with readlanes (its row index is uniform), each row subtracts
//     (J[i][C] / pivot) x the pivot row with one fused multiply-add per element, and the pivot row
//     is scaled by 1 / pivot;
//   * rows never move: each remembers the column it was the pivot of, and the solution is the
//     right-hand side in that order.
// Columns < C are neither read nor updated after step C (the host's solve16 updates them and never
// reads them again).  Fused arithmetic and a different tie rule make this a different rounding of
// the same solve (the trims are compared with the host's to fp32 resolution, not bitwise).
// A zero or non-finite pivot (a singular or non-finite system) makes its reciprocal, and with it the
// solution, non-finite: the caller checks the solution once instead of every pivot.
#ifndef HG_GJ_NOSCALE   // 1: the pivot rows stay unscaled, each row's solution divided at the end
#define HG_GJ_NOSCALE 0
#endif
#ifndef HG_GJ_LDS       // 1: the pivot row reaches the other rows through LDS (broadcast reads)
#define HG_GJ_LDS 0
#endif
constexpr int kRowStride = 18;   // doubles per LDS row (16-byte aligned pairs)
#ifndef HG_E_STRIDE
#define HG_E_STRIDE 17
#endif
constexpr int kEStride = HG_E_STRIDE;   // doubles per evaluation row of sE

template <int C>
__device__ __forceinline__ void gj_step(double (&A)[16], double& b, uint32_t& live, int& mycol, int i,
                                        double& myinv, double* sRow, int l) {
    (void)myinv; (void)sRow; (void)l;
    const double v = A[C];
    // |v|'s high word with the top bit set (so that a zero candidate still beats a used row); 0 once used
    const uint32_t key = ((uint32_t)(__double_as_longlong(v) >> 32) | 0x80000000u) & live;
    const double own_inv = rcp_f64(v);   // every row's reciprocal while the search runs (off its chain)
    const uint32_t mx = row16_max(key);
    const uint32_t hit = (uint32_t)__ballot(key == mx) & 0xFFFFu;   // rows of the first 16 lanes
    const int P = __builtin_ctz(hit | 0x10000u);
    const double rinv = read_lane(own_inv, P);
    const bool piv = i == P;
#if HG_GJ_LDS
    // every row's live part to its LDS row, then the pivot row read back by all (broadcast)
    constexpr int k0 = (C + 1) >> 1;
    double* mine = sRow + l * kRowStride;
#pragma unroll
    for (int k = k0; k < 8; ++k) {
        typedef double d2 __attribute__((ext_vector_type(2)));
        *reinterpret_cast<d2*>(mine + 2 * k) = d2{A[2 * k], A[2 * k + 1]};
    }
    mine[16] = b;
    lds_order();
    double pr[17];
    const double* prow = sRow + P * kRowStride;
#pragma unroll
    for (int k = k0; k < 8; ++k) {
        typedef double d2 __attribute__((ext_vector_type(2)));
        const d2 t = *reinterpret_cast<const d2*>(prow + 2 * k);
        pr[2 * k] = t.x;
        pr[2 * k + 1] = t.y;
    }
    pr[16] = prow[16];
#define HG_PJ(j) pr[j]
#define HG_PB pr[16]
#else
#define HG_PJ(j) read_lane(A[j], P)
#define HG_PB read_lane(b, P)
#endif
#if HG_GJ_NOSCALE
    // rows are never scaled: other rows subtract (v / pivot) x the pivot row, the pivot row keeps its
    // values (the fused add of -0 is exact) and its reciprocal divides its right-hand side at the end
    const double g = piv ? 0.0 : v * rinv;
#pragma unroll
    for (int j = C + 1; j < 16; ++j) A[j] = fma(-g, HG_PJ(j), A[j]);
    b = fma(-g, HG_PB, b);
    myinv = piv ? rinv : myinv;
#else
    // other rows: A - (v / pivot) pj; the pivot row: A / pivot -- one form for both, A * m - g pj with
    // (m, g) = (1, v / pivot) or (1 / pivot, 0): the product by 1 and the fused add of -0 are exact
    const double g = piv ? 0.0 : v * rinv;
    const double m = piv ? rinv : 1.0;
#pragma unroll
    for (int j = C + 1; j < 16; ++j) A[j] = fma(-g, HG_PJ(j), A[j] * m);
    b = fma(-g, HG_PB, b * m);
#endif
#undef HG_PJ
#undef HG_PB
    live = piv ? 0u : live;
    mycol = piv ? C : mycol;
}
template <int C>
__device__ __forceinline__ void gj_steps(double (&A)[16], double& b, uint32_t& live, int& mycol, int i,
                                         double& myinv, double* sRow, int l) {
    gj_step<C>(A, b, live, mycol, i, myinv, sRow, l);
    if constexpr (C < 15) gj_steps<C + 1>(A, b, live, mycol, i, myinv, sRow, l);
}

// HG_GJ_SPLIT: the same solve with the four copies of a row splitting its columns.  Lane l holds row
// i = l & 15 and, in quarter q = l >> 4, the columns 4 jj + q (jj = 0..3) plus the right-hand side
// (identical in every quarter).  Pivot step C reads column C in quarter C & 3 (each quarter is one DPP
// row, so the 16-lane max is per quarter and the ballot takes that quarter's 16 bits); the row's
// multiplier goes to its four quarters and each quarter fetches its own columns of the pivot row with
// one lane shuffle per column.  Same pivots, same fused operations, so the same results bit for bit,
// with a quarter of the elementwise work and of the LDS reads per lane.
#ifndef HG_GJ_SPLIT
#define HG_GJ_SPLIT 2
#endif
// HG_GJ_MFMA (default): the blocked solve of gj_mfma.h (four panels, one v_mfma_f64_16x16x4_f64 each)
// instead of the unblocked one below (HG_GJ_MFMA=0 for A/B).  HG_GJ_STATIC (default): first with the
// pivot order of the host's trim of the same condition (gjs_solve, no pivot search), accepted when its
// residual is that of a backward-stable solve, else searched (gjm_solve).
#ifndef HG_GJ_MFMA
#define HG_GJ_MFMA 1
#endif
#ifndef HG_GJ_STATIC
#define HG_GJ_STATIC 1
#endif
template <int C>
__device__ __forceinline__ void gjs_step(double (&A4)[4], double& b, uint32_t& live, int& mycol, int i, int l) {
    constexpr int qc = C & 3, jc = C >> 2;
    const double v = A4[jc];   // column C in quarter qc
    const uint32_t key = ((uint32_t)(__double_as_longlong(v) >> 32) | 0x80000000u) & live;
    const double own_inv = rcp_f64(v);
    const uint32_t mx = row16_max(key);
    const uint32_t hit = (uint32_t)(__ballot(key == mx) >> (16 * qc)) & 0xFFFFu;
    const int P = __builtin_ctz(hit | 0x10000u);
    const double rinv = read_lane(own_inv, 16 * qc + P);
    const bool piv = i == P;
    const double g = __shfl(piv ? 0.0 : v * rinv, 16 * qc + i);   // row i's multiplier, from quarter qc
    const double m = piv ? rinv : 1.0;
    const int src = (l & 48) + P;   // this quarter's lane of the pivot row
#pragma unroll
    for (int jj = jc; jj < 4; ++jj) A4[jj] = fma(-g, __shfl(A4[jj], src), A4[jj] * m);
    b = fma(-g, read_lane(b, P), b * m);
    live = piv ? 0u : live;
    mycol = piv ? C : mycol;
}
template <int C>
__device__ __forceinline__ void gjs_steps(double (&A4)[4], double& b, uint32_t& live, int& mycol, int i, int l) {
    gjs_step<C>(A4, b, live, mycol, i, l);
    if constexpr (C < 15) gjs_steps<C + 1>(A4, b, live, mycol, i, l);
}

// HG_GJ_SPLIT 2: as 1, and the next three pivot columns (C, C+1, C+2) also replicated in every quarter
// (rep, nx1, nx2), so that a pivot step's chain -- search, reciprocal, multiplier, the update of
// the next pivot column -- has no lane shuffle in it: the multiplier is formed in every quarter and
// the next column is updated with a readlane of the pivot row's value.  The owners keep their columns
// from C+3 on current (one shuffle per column, off that chain), and column C+3 is broadcast to the
// quarters at the end of step C.  The same values in the same operations: bitwise the solve above.
template <int C>
__device__ __forceinline__ void gjr_step(double (&A4)[4], double& b, double& rep, double& nx1, double& nx2,
                                         uint32_t& live, int& mycol, int i, int l) {
    const uint32_t key = ((uint32_t)(__double_as_longlong(rep) >> 32) | 0x80000000u) & live;
    const double own_inv = rcp_f64(rep);
    const uint32_t mx = row16_max(key);
    const uint32_t hit = (uint32_t)__ballot(key == mx) & 0xFFFFu;
    const int P = __builtin_ctz(hit | 0x10000u);
    const double rinv = read_lane(own_inv, P);
    const bool piv = i == P;
    const double g = piv ? 0.0 : rep * rinv;
    const double m = piv ? rinv : 1.0;
    if constexpr (C + 1 < 16) nx1 = fma(-g, read_lane(nx1, P), nx1 * m);
    if constexpr (C + 2 < 16) nx2 = fma(-g, read_lane(nx2, P), nx2 * m);
    const int src = (l & 48) + P;
#pragma unroll
    for (int jj = (C + 3) >> 2; jj < 4; ++jj) A4[jj] = fma(-g, __shfl(A4[jj], src), A4[jj] * m);
    b = fma(-g, read_lane(b, P), b * m);
    live = piv ? 0u : live;
    mycol = piv ? C : mycol;
    rep = nx1;
    nx1 = nx2;
    if constexpr (C + 3 < 16) nx2 = __shfl(A4[(C + 3) >> 2], 16 * ((C + 3) & 3) + i);
}
template <int C>
__device__ __forceinline__ void gjr_steps(double (&A4)[4], double& b, double& rep, double& nx1, double& nx2,
                                          uint32_t& live, int& mycol, int i, int l) {
    gjr_step<C>(A4, b, rep, nx1, nx2, live, mycol, i, l);
    if constexpr (C < 15) gjr_steps<C + 1>(A4, b, rep, nx1, nx2, live, mycol, i, l);
}

// What the observation needs from one evaluation beyond the state: power, uvw_air, ned velocity
// (observe(), helicopter_dynamics.py:471-488).
struct EvalExt {
    double o[7];
};

// __trim_fcn (helicopter_dynamics.py:557-576, trim.h trim_fcn): the normalised derivatives y(x) at
// one trial point, and the observation's non-state terms.
__device__ __forceinline__ void trim_eval(const hg::Params<double>& P, const hg::TrimSetup& T, const double x[16],
                                          const double W[3], double y[16], EvalExt& e) {
    double s[18], d[18];
    hg::trim_state(P, T.base, x, s);
    const hg::Controls<double> u = hg::controls(P, x[12], x[13], x[14], x[15]);
    hg::Attitude<double> att;
    hg::m_sincos(s[12], &att.s[0], &att.c[0]);
    hg::m_sincos(s[13], &att.s[1], &att.c[1]);
    att.s[2] = T.s_psi;
    att.c[2] = T.c_psi;
    const hg::Frame<double> f = hg::frame(P, s, W, T.hc, att, T.rho_irho);
    const hg::Loads<double> A = hg::main_loads(P, s, u, f);
    const hg::Loads<double> B = hg::tail_loads(P, s, u, f);
    hg::eom(P, s, f, A, B, d);
    y[0] = hg::m_div_c(d[0], P.mr_VTIP, P.mr_inv_VTIP);
    y[1] = hg::m_div_c(d[1], P.tr_VTIP, P.tr_inv_VTIP);
    y[2] = d[4];
    y[3] = d[5];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        y[4 + k] = hg::m_div_c(d[6 + k], P.mr_VTIP, P.mr_inv_VTIP);
        y[7 + k] = hg::m_div_c(d[9 + k], P.mr_OMEGA, P.mr_inv_OMEGA);
        y[10 + k] = d[12 + k];
        y[13 + k] = hg::m_div_c(d[15 + k], P.mr_R, P.mr_inv_R);
    }
    e.o[0] = ((A.power + B.power) + P.p_loss) * (1.0 / 550.0);
    e.o[1] = f.ua; e.o[2] = f.va; e.o[3] = f.wa;
    e.o[4] = f.n0; e.o[5] = f.n1; e.o[6] = f.n2;
}

__device__ __forceinline__ void retrim_write(const RetrimArgs& a, const hg::Params<double>& P, const hg::TrimSetup& T,
                                             int64_t job, int64_t env, const double x[16], const double* ext) {
    double s[18], ob[17];
    hg::trim_state(P, T.base, x, s);
#pragma unroll
    for (int c = 0; c < 7; ++c) ob[c] = ext[c];
    ob[7] = s[12]; ob[8] = s[13]; ob[9] = s[14];
    ob[10] = s[9]; ob[11] = s[10]; ob[12] = s[11];
    ob[13] = s[15]; ob[14] = s[16]; ob[15] = -s[17]; ob[16] = -T.hc.zh(s[17]);
    if (a.list || a.recs) {
        for (int c = 0; c < 18; ++c)
            if (has_slot(c)) a.state[tix(env, c)] = (float)s[c];
        int32_t* ctr = reinterpret_cast<int32_t*>(a.state);
        int32_t epi = ctr[tix(env, kCtrCol0 + 2)];
        if (a.ov) {   // the rest of the reset (the concurrent step stored the step counter)
            epi += 1;
            for (int c = 18; c < 23; ++c) a.state[tix(env, c)] = 0.f;
            ctr[tix(env, kCtrCol0 + 1)] = 0;
            ctr[tix(env, kCtrCol0 + 2)] = epi;
        }
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

// ov mode, a failed trim: the env takes the template reset the step would have stored (the
// reference raises instead, helicopter_dynamics.py:543-544; the failure is counted)
__device__ __forceinline__ void retrim_write_template(const RetrimArgs& a, int64_t env) {
    const float* tr = a.tmpl_env ? a.tmpl_env + env * 39 : a.tmpl;
    for (int c = 0; c < 18; ++c)
        if (has_slot(c)) a.state[tix(env, c)] = tr[c];
    for (int c = 18; c < 23; ++c) a.state[tix(env, c)] = 0.f;
    for (int c = 0; c < 4; ++c) a.state[tix(env, 23 + c)] = tr[18 + c];
    int32_t* ctr = reinterpret_cast<int32_t*>(a.state);
    const int32_t epi = ctr[tix(env, kCtrCol0 + 2)] + 1;
    ctr[tix(env, kCtrCol0 + 1)] = 0;
    ctr[tix(env, kCtrCol0 + 2)] = epi;
    // an episode begun from the template: the azimuth record anchors the template's azimuths
    a.az[env] = AzRec{tr[kAzCol0], tr[kAzCol0 + 1], 0, epi};
    if (a.obs)
        for (int c = 0; c < 17; ++c) a.obs[env * 17 + c] = tr[22 + c];
}

// One wave per trim.  Each evaluation round evaluates 42 points at once: lanes 0..31 the +-eps
// Jacobian columns around the point the next Newton step starts from, lanes 32..41 the ten
// step-halving trials of the current step (trial 0, the full step, is that point whenever the
// search accepts it, which it usually does; the first round: lane 32 the residual at x0).  The first
// trial that lowers the residual is the one the reference's sequential search accepts
// (helicopter_dynamics.py:530-541).  When the search accepts a shorter step, a round of Jacobian
// lanes alone re-evaluates around it (the trial lanes keep their values).  Then the evaluations go
// through LDS to the Gauss-Jordan solve.  A trim of three Newton steps takes four rounds and three
// solves.
enum : int { kRoundFirst = 0, kRoundNormal = 1, kRoundJacobian = 2 };

// Model constants and trim setup through the constant address space: scalar loads (the kernel's
// stores cannot alias them), re-issued each round (opaque pointers) instead of hoisted out of the
// Newton loop, where ~180 fp64 values would stay live in registers.
typedef __attribute__((address_space(4))) const hg::Params<double> ConstP;
typedef __attribute__((address_space(4))) const hg::TrimSetup ConstT;
template <typename Q, typename T>
__device__ __forceinline__ const T& opaque_const(const T* p) {
    Q* c = (Q*)p;
    asm volatile("" : "+s"(c));
    return *(const T*)c;
}

// HG_RT_XLDS: the Newton iterate x and direction dir (uniform over the wave) live in LDS instead of
// 64 VGPRs, which leaves the solve's schedule room to keep its lane shuffles in flight
#ifndef HG_RT_XLDS
#define HG_RT_XLDS 1
#endif
#if HG_RT_XLDS
#define HG_X(k) sXc[k]
#define HG_DIR(k) sX[k]
#else
#define HG_X(k) x[k]
#define HG_DIR(k) dir[k]
#endif
#ifndef HG_RT_VLOAD
#define HG_RT_VLOAD 1
#endif
#ifndef HG_RETRIM_WAVES
#define HG_RETRIM_WAVES 2
#endif
#if HG_RT_DEBUG
__device__ long long g_rt_dbg[4096][4];
__device__ unsigned g_rt_dbg_n;
#endif
// The jobs first, first + stride, ... of a batch, one wave (this block) per trim: retrim_kernel and the
// trim blocks of the overlapped next-step re-trim (heligym_amd.hip step_ov_kernel).
// count_p / recs_p / T_p / P_p: a.count / a.recs / a.T / a.P, passed again as leading kernel
// arguments, which the kernels have preloaded into SGPRs at wave launch (-amdgpu-kernarg-preload-count),
// and Tstride_p = a.setup_stride: the job count, the first record, the first job's setup and a
// prefetch of the model constants are all requested at once, before the kernel-argument segment has
// arrived (round 6: each was a dependent memory round trip of the trim's start-up).
#ifndef HG_FUSED_MAX_POLLS   // a fused trim wave waits at most this many polls for a record (never reached)
#define HG_FUSED_MAX_POLLS (1 << 20)
#endif
#ifndef HG_FUSED_SLEEP       // s_sleep between a fused trim wave's polls (units of 64 clocks)
#define HG_FUSED_SLEEP 4
#endif
// FUSED (step_fused_kernel): jobs are claimed one at a time (a.claim) and each record waited for until
// its step wave publishes it, or until every step wave has reserved and the claim is past the queue.
template <bool FUSED = false>
__device__ __forceinline__ void retrim_jobs(const RetrimArgs& a, int64_t first, int64_t stride, const int32_t* count_p,
                                            const int4* recs_p, const hg::TrimSetup* T_p, const hg::Params<double>* P_p,
                                            int32_t Tstride_p) {
    // the trim is the launch's long pole: its wave issues first wherever it shares a SIMD (the
    // overlapped launch's step waves, one per SIMD, have time to spare)
    __builtin_amdgcn_s_setprio(3);
    // the +-eps evaluations E[j][k] of the current Newton step, row j (the evaluating lane) at a stride
    // of kEStride doubles: lane j's 16 writes of a 16-double stride all hit the same two banks
    __shared__ double sE[42 * kEStride];   // rows 32..41: the line-search trials' evaluations
    __shared__ double sYt[16];       // the trim's target derivatives y* (its right-hand side is y(src) - y*)
    __shared__ double sX[16];        // the solution (Newton direction), by column
    __shared__ double sXc[16];       // HG_RT_XLDS: the current iterate (else the first job's x0)
    __shared__ double sExt[7];       // observation terms of the current iterate
    __shared__ double sRow[HG_GJ_LDS ? 64 * kRowStride : 2];   // HG_GJ_LDS: the rows of the solve
    __shared__ double sImg[HG_GJ_MFMA ? 16 * kImgStride : 2];  // HG_GJ_MFMA: the system's image per panel
    __shared__ int8_t sPiv[64];      // HG_GJ_STATIC: the setup's pivot order per Newton step
    const int l = threadIdx.x;
    const hg::Params<double>& P = *a.P;
    const double eps = hg::kTrimEps;
#if HG_TIMING
    if (l == 0 && first == 0) g_rt_timing[62] = __builtin_amdgcn_s_memtime();   // entry (start-up latency)
#endif
    const int c = l & 15;            // Jacobian column of lanes 0..31
    const int j = l - 32;            // line-search trial of lanes 32..41
    // the first job record is requested with the job count, so the start waits for one load, not two
    // dependent ones; the records hold n entries, and a block past them (a grid of more blocks than
    // envs) reads none
#if HG_RT_VLOAD
    // the job count and the first record as vector loads (a uniform address made opaque to the
    // compiler), both requested before either is waited for: as scalar loads each was waited for at
    // once (its result spills to VGPR lanes), two memory latencies in a row.  A block with nothing to
    // read reads the model constants instead (any readable address) and discards them.
    int zero_v;
    asm volatile("v_mov_b32 %0, 0" : "=v"(zero_v));
    // (a launch has at most one block per env, so recs_p[first] is a record; with no queue, no load)
    int4 rec0_v = make_int4(-1, 0, 0, 0);
    int32_t count_v = 0;
    if (!FUSED && (recs_p || count_p)) {
        const int32_t* any = count_p ? count_p : reinterpret_cast<const int32_t*>(recs_p);
        rec0_v = (recs_p ? recs_p + first : reinterpret_cast<const int4*>(any))[zero_v];
        count_v = any[zero_v];
    }
    const bool has_rec0 = a.recs && first < a.n;
#endif
    // the first job's setup (initial guess, targets, pivot order), and one lane per 64-byte line of the
    // model constants (into the L2 for the first round's scalar loads; the value is only kept alive)
    const hg::TrimSetup* T0 = T_p + (Tstride_p ? first : 0);
    const double x0_l = T0->x0[l & 15];
    const double yt_l = T0->yt[l & 15];
    const int8_t piv_l = T0->piv[l >> 4][l & 15];
    constexpr int kPWords = (int)(sizeof(hg::Params<double>) / 4);
    const uint32_t pf = reinterpret_cast<const uint32_t*>(P_p)[min(16 * l, kPWords - 1)];
#ifndef HG_RT_SETUP_LDS   // (retrim.hip sets it; the overlapped launch is 0.2 us faster without)
#define HG_RT_SETUP_LDS 0
#endif
#if HG_GJ_MFMA && HG_GJ_STATIC && HG_RT_SETUP_LDS
    // the first job's setup goes straight to LDS (the loop skips it for that job) and the prefetch is
    // consumed here, all in one wait with the job count and record: held in registers into the Newton
    // loop they were spilled to scratch, and each spill waited for its load in turn (2 us of the
    // start-up, scripts/retrim_startup.py)
    if (l < 16) {
        sYt[l] = yt_l;
        sXc[l] = x0_l;
    }
    sPiv[l] = piv_l;
    const bool use_piv0 = __builtin_amdgcn_readfirstlane(piv_l) >= 0;   // (lane 0: piv[0][0])
    asm volatile("" ::"v"(pf));
    constexpr bool kSetupInLds = true;
#else
    constexpr bool kSetupInLds = false;
    constexpr bool use_piv0 = false;   // (unused)
#endif
#if HG_RT_VLOAD
    const int4 rec0 = has_rec0 ? make_int4(__builtin_amdgcn_readfirstlane(rec0_v.x), __builtin_amdgcn_readfirstlane(rec0_v.y),
                                           __builtin_amdgcn_readfirstlane(rec0_v.z), __builtin_amdgcn_readfirstlane(rec0_v.w))
                               : make_int4(-1, 0, 0, 0);
    int64_t jobs = a.count ? (int64_t)__builtin_amdgcn_readfirstlane(count_v) : a.njobs;
#else
    const int4 rec0 = (a.recs && first < a.n) ? a.recs[first] : make_int4(-1, 0, 0, 0);
    int64_t jobs = a.count ? (int64_t)*a.count : a.njobs;
#endif
#if HG_RT_DEBUG
    if (l == 0 && first == 0) {   // diagnostic build: one record per launch (count address, jobs, mode, first record)
        const unsigned k = atomicAdd(&g_rt_dbg_n, 1u);
        if (k < 4096) {
            g_rt_dbg[k][0] = (long long)(uintptr_t)a.count;
            g_rt_dbg[k][1] = jobs;
            g_rt_dbg[k][2] = a.ov + (a.list ? 2 : 0) + (a.recs ? 4 : 0);
            g_rt_dbg[k][3] = rec0.x;
        }
    }
#endif
#if HG_TIMING
    if (first == 0) {   // the job count and first record have arrived
        asm volatile("" ::"s"((int)jobs), "s"(rec0.x));
        if (l == 0) g_rt_timing[60] = __builtin_amdgcn_s_memtime();
    }
#endif
    if (a.count && jobs > a.n) {   // a queue holds at most one job per env
        if (first == 0 && l == 0 && a.bad_jobs) atomicAdd(a.bad_jobs, 1);
        jobs = a.n;
    }
    for (int64_t job = first; FUSED || job < jobs; job += stride) {   // uniform per wave
        int4 rec;
        if constexpr (FUSED) {
            // claim the next job, then wait for its record (env >= 0, stored last) or for the end: every
            // step wave reserved and the claim past the queue.  Device-coherent loads only (no acquire,
            // whose L2 invalidate per poll would evict the step waves' data); the wind is read after
            // env, as the step wave stored it before env.
            int claimed = 0;
            if (l == 0) claimed = atomicAdd(a.claim, 1);
            job = __builtin_amdgcn_readfirstlane(claimed);
            if (job >= a.n) break;
            FSTAMP(0);
            int* rp = reinterpret_cast<int*>(const_cast<int4*>(a.recs) + job);
            int x = -1;
            bool end = false;
            for (int polls = 0; x < 0 && !end; ++polls) {
                x = __builtin_amdgcn_readfirstlane(__hip_atomic_load(rp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
                if (x < 0) {
                    // {queued jobs, waves with jobs}, and lanes 0..15 the counts of waves without
                    const unsigned long long q =
                        __hip_atomic_load(const_cast<unsigned long long*>(a.ctr), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    int wl = 0;
                    if (l < kFusedWaveCtrs)
                        wl = __hip_atomic_load(reinterpret_cast<const int32_t*>(a.ctr) + kFusedLine * (1 + l), __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT);
                    const int qn = __builtin_amdgcn_readfirstlane((int)(uint32_t)q);
                    int wn = __builtin_amdgcn_readfirstlane((int)(uint32_t)(q >> 32));
#pragma unroll
                    for (int k = 0; k < kFusedWaveCtrs; ++k) wn += __builtin_amdgcn_readlane(wl, k);
                    // (each count is bounded by its own waves, so the parts read at different times
                    // reach the wave count only once every wave with jobs has reserved: qn is final)
                    end = wn >= a.nwaves && job >= qn;
                    if (!end && polls >= HG_FUSED_MAX_POLLS) {   // (a step wave that never reserved)
                        if (l == 0 && a.bad_jobs) atomicAdd(a.bad_jobs, 1);
                        end = true;
                    }
                    if (!end) __builtin_amdgcn_s_sleep(HG_FUSED_SLEEP);
                }
            }
            if (x < 0) break;
            FSTAMP(1);
            asm volatile("" ::: "memory");
            rec = make_int4(x, __builtin_amdgcn_readfirstlane(__hip_atomic_load(rp + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)),
                            __builtin_amdgcn_readfirstlane(__hip_atomic_load(rp + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)),
                            __builtin_amdgcn_readfirstlane(__hip_atomic_load(rp + 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)));
            if (l == 0) rp[0] = -1;   // the slot free for the next launch's queue
        } else {
            rec = a.recs ? (job == first ? rec0 : a.recs[job]) : make_int4(0, 0, 0, 0);
            // every consumed record goes back to env -1, so that a fused launch (which waits for env >= 0)
            // never takes a record an earlier launch of the other paths left behind
            if (a.recs && l == 0) const_cast<int4*>(a.recs)[job].x = -1;
        }
        const int64_t env = a.recs ? (int64_t)rec.x : (a.list ? (int64_t)a.list[job] : job);
        if ((a.recs || a.list) && (uint64_t)env >= (uint64_t)a.n) {   // never index the state with a bad record
            if (l == 0 && a.bad_jobs) atomicAdd(a.bad_jobs, 1);
            continue;
        }
        const hg::TrimSetup& T = a.T[a.setup_stride ? job : 0];
        const bool j0 = job == first || !Tstride_p;   // (its setup requested at entry: every job's, with one setup)
#if HG_GJ_MFMA && HG_GJ_STATIC
        bool use_piv;
        if (kSetupInLds && j0) {   // (the entry's: this job's setup is the first job's)
            use_piv = use_piv0;
        } else {
            const int8_t piv_v = j0 ? piv_l : T.piv[l >> 4][l & 15];
            sPiv[l] = piv_v;
            use_piv = __builtin_amdgcn_readfirstlane(piv_v) >= 0;   // (lane 0: piv[0][0])
        }
#endif
        if (l < 16 && !(kSetupInLds && j0)) sYt[l] = j0 ? yt_l : T.yt[l];   // (read after the first round's lds_order)
#if HG_TIMING
        if (job == 0) {   // the setup has arrived
            asm volatile("" ::"v"(yt_l), "v"(x0_l));
            if (l == 0) g_rt_timing[59] = __builtin_amdgcn_s_memtime();
        }
#endif
        double W[3] = {P.wm[0], P.wm[1], P.wm[2]};   // NULL wind: the mean wind (helicopter.py:55)
        if (a.recs) {
            W[0] = (double)__int_as_float(rec.y);
            W[1] = (double)__int_as_float(rec.z);
            W[2] = (double)__int_as_float(rec.w);
        } else if (a.wind && a.wind_soa) {
            W[0] = (double)a.wind[env];
            W[1] = (double)a.wind[a.n + env];
            W[2] = (double)a.wind[2 * a.n + env];
        } else if (a.wind) {
            const float* wr = a.wind + 3 * (a.list ? env : job);
            W[0] = (double)wr[0];
            W[1] = (double)wr[1];
            W[2] = (double)wr[2];
        }
        double ye[16], te = 0.0;
        EvalExt ext;
#pragma unroll
        for (int k = 0; k < 16; ++k) ye[k] = 0.0;
#if HG_RT_XLDS
        if (l < 16) {
            // (the iterate: only the first job's is the entry's, a later job starts from its setup again)
            if (!(kSetupInLds && job == first)) sXc[l] = kSetupInLds ? T.x0[l] : (j0 ? x0_l : T.x0[l]);
            sX[l] = 0.0;
        }
        lds_order();
#else
        double x[16], dir[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            x[k] = kSetupInLds ? (job == first ? sXc[k] : T.x0[k]) : (j0 ? read_lane(x0_l, k) : T.x0[k]);
            dir[k] = 0.0;
        }
#endif
        double tol = 0;
        int it = 0, kind = kRoundFirst, src = 32, round = 0;
        bool ok = true, converged = false;
        RSTAMP(0, "v"(l));
        while (true) {
            const hg::Params<double>& P = opaque_const<ConstP>(a.P);
            const hg::TrimSetup& T = opaque_const<ConstT>(a.T + (a.setup_stride ? job : 0));
            // ---- one evaluation round (every x - s dir is the same fused operation wherever formed)
            // every lane forms x - s dir with its own s (a Jacobian lane: the full step of a normal
            // round, else 0; a trial lane: 2^-j; the fused form with s = 0 is x itself), and a
            // Jacobian lane adds its +-eps to its own column: the same operations as branching per
            // lane class, with one select per component instead of three
            const double sl = l < 32 ? (kind == kRoundNormal ? 1.0 : 0.0)
                                     : ((kind == kRoundNormal && j < hg::kTrimLineSearch) ? ldexp(1.0, -j) : 0.0);
            const double pe = l < 16 ? eps : -eps;
#ifndef HG_RT_OPAQUE_COL
#define HG_RT_OPAQUE_COL 0
#endif
            // (HG_RT_OPAQUE_COL: the column re-materialised each round; hoisted out of the Newton loop,
            // the 16 selects' masks and addends take 32 VGPRs and push the loop's scalars into a long
            // spill prologue)
            int cr = c;
            if (HG_RT_OPAQUE_COL) asm volatile("" : "+v"(cr));
            double xe[16];
#pragma unroll
            for (int k = 0; k < 16; ++k) {
                const double b = fma(-sl, HG_DIR(k), HG_X(k));
                xe[k] = (l < 32 && cr == k) ? b + pe : b;
            }
            RSTAMP(1 + 4 * round, "v"(xe[0]));
            if (kind != kRoundJacobian || l < 32) {
#ifdef HG_ISA_MARK
                asm volatile("; EVAL_BEGIN");
#endif
                trim_eval(P, T, xe, W, ye, ext);
#ifdef HG_ISA_MARK
                asm volatile("; EVAL_END");
#endif
                double t = 0.0;
#pragma unroll
                for (int k = 0; k < 16; ++k) t = fma(ye[k] - T.yt[k], ye[k] - T.yt[k], t);
                te = t;
            }
            RSTAMP(2 + 4 * round, "v"(te));
#ifdef HG_ISA_MARK
            asm volatile("; ACC_BEGIN");
#endif
            if (kind != kRoundJacobian) {
                // ---- accept a trial (or take the base point)
                bool have_jac = true;
                if (kind == kRoundNormal) {
                    const unsigned long long lower = __ballot(j >= 0 && j < hg::kTrimLineSearch && te < tol) >> 32;
                    const int js = lower ? __builtin_ctzll(lower) : hg::kTrimLineSearch;
                    if (js >= hg::kTrimLineSearch - 1) break;   // helicopter_dynamics.py:540: keep x
                    const double step = ldexp(1.0, -js);
#if HG_RT_XLDS
                    if (l < 16) sXc[l] = fma(-step, sX[l], sXc[l]);
                    lds_order();
#else
#pragma unroll
                    for (int k = 0; k < 16; ++k) x[k] = fma(-step, dir[k], x[k]);
#endif
                    src = 32 + js;
                    have_jac = js == 0;   // the Jacobian lanes evaluated around trial 0
                    if (++it > hg::kTrimMaxIter) { ok = false; break; }
                }
                tol = read_lane(te, src);
                if (!(tol > eps)) { converged = true; break; }   // the accepting lane holds the final evaluation
                if (l == src) {
#pragma unroll
                    for (int k = 0; k < 7; ++k) sExt[k] = ext.o[k];
                }
                if (!have_jac) {   // the search accepted a shorter step: Jacobian at the new x first
                    kind = kRoundJacobian;
                    ++round;
                    continue;
                }
            }
            // ---- Newton direction: the evaluations and the residual (lane src holds y) into LDS,
            // then the solve, one row per lane
            lds_order();   // the previous solve's reads are done
            if (l < 42) {   // the Jacobian lanes and the trials: the residual is row src's y - y*
#pragma unroll
                for (int k = 0; k < 16; ++k) sE[l * kEStride + k] = ye[k];
            }
            lds_order();
#ifdef HG_ISA_MARK
            asm volatile("; ACC_END");
#endif
            RSTAMP(3 + 4 * round, "v"(ye[0]));
#if HG_GJ_MFMA
            {
                bool solved = false;
#if HG_GJ_STATIC
                if (use_piv) {
                    solved = gjs_solve(sE, kEStride, 0.5 / eps, src, sYt, sPiv + 16 * (it < 3 ? it : 3), sImg, sX, l);
                    if (l == 0 && a.solve_stats) {
                        atomicAdd(a.solve_stats, 1);
                        if (!solved) atomicAdd(a.solve_stats + 1, 1);
                    }
                    lds_order();   // (the searched solve rewrites the image and x the residual test read)
                }
#endif
                if (!solved) gjm_solve(sE, kEStride, 0.5 / eps, src, sYt, sImg, sX, l);
                lds_order();
                bool fin = true;
#pragma unroll
                for (int k = 0; k < 16; ++k) {
#if HG_RT_XLDS
                    fin = fin && (solved || isfinite(sX[k]));   // (a passed residual test implies finite)
#else
                    dir[k] = sX[k];
                    fin = fin && isfinite(dir[k]);
#endif
                }
                if (!fin) { ok = false; break; }
            }
#elif HG_GJ_SPLIT
            {
                const int i = l & 15, q = l >> 4;
                double A4[4], Em4[4];
#pragma unroll
                for (int jj = 0; jj < 4; ++jj) {   // all 9 reads issued before the first use
                    A4[jj] = sE[(4 * jj + q) * kEStride + i];
                    Em4[jj] = sE[(4 * jj + q + 16) * kEStride + i];
                }
                double b = sE[src * kEStride + i] - sYt[i];
#pragma unroll
                for (int jj = 0; jj < 4; ++jj) A4[jj] = (A4[jj] - Em4[jj]) * (0.5 / eps);
                uint32_t live = 0xFFFFFFFFu;
                int mycol = 0;
#if HG_GJ_SPLIT == 2
                double rep = (sE[i] - sE[16 * kEStride + i]) * (0.5 / eps);
                double nx1 = (sE[kEStride + i] - sE[17 * kEStride + i]) * (0.5 / eps);
                double nx2 = (sE[2 * kEStride + i] - sE[18 * kEStride + i]) * (0.5 / eps);
                gjr_steps<0>(A4, b, rep, nx1, nx2, live, mycol, i, l);
#else
                gjs_steps<0>(A4, b, live, mycol, i, l);
#endif
                if (l < 16) sX[mycol] = b;
                lds_order();
                bool fin = true;
#pragma unroll
                for (int k = 0; k < 16; ++k) {
#if HG_RT_XLDS
                    fin = fin && isfinite(sX[k]);
#else
                    dir[k] = sX[k];
                    fin = fin && isfinite(dir[k]);
#endif
                }
                if (!fin) { ok = false; break; }
            }
#else
            {
                const int i = l & 15;
                double A[16], Em[16];
#pragma unroll
                for (int q = 0; q < 16; ++q) {   // all 33 reads issued before the first use
                    A[q] = sE[q * kEStride + i];
                    Em[q] = sE[(q + 16) * kEStride + i];
                }
                double b = sE[src * kEStride + i] - sYt[i];
#pragma unroll
                for (int q = 0; q < 16; ++q) A[q] = (A[q] - Em[q]) * (0.5 / eps);
                uint32_t live = 0xFFFFFFFFu;   // the key mask of a row not yet used as a pivot
                int mycol = 0;
                double myinv = 1.0;
                gj_steps<0>(A, b, live, mycol, i, myinv, sRow, l);
                if (l < 16) sX[mycol] = HG_GJ_NOSCALE ? b * myinv : b;
                lds_order();
                bool fin = true;
#pragma unroll
                for (int k = 0; k < 16; ++k) {
#if HG_RT_XLDS
                    fin = fin && isfinite(sX[k]);
#else
                    dir[k] = sX[k];
                    fin = fin && isfinite(dir[k]);
#endif
                }
                if (!fin) { ok = false; break; }
            }
#endif
            RSTAMP(4 + 4 * round, "v"(HG_DIR(0)));
            kind = kRoundNormal;
            ++round;
        }
        RSTAMP(63, "v"(l));
#if HG_RT_XLDS
        double x[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) x[k] = sXc[k];
#endif
        if (ok) {
            if (converged) {
                if (l == src) retrim_write(a, P, T, job, env, x, ext.o);
            } else if (l == 0) {
                // the search stopped without converging (:540): the kept x and its evaluation
                double e[7];
                lds_order();
#pragma unroll
                for (int k = 0; k < 7; ++k) e[k] = sExt[k];
                retrim_write(a, P, T, job, env, x, e);
            }
        } else if (l == 0) {
            if (a.ov) retrim_write_template(a, env);
            if (a.fail_count) atomicAdd(a.fail_count, 1);
            if (a.out_status) a.out_status[job] = HG_E_TRIM;
        }
        RSTAMP(61, "v"(l));   // the write-out issued
        FSTAMP(2);
        lds_order();   // the next job's writes come after this job's reads
    }
    if (!kSetupInLds && pf == 0x7FC00001u && jobs == -12345 && a.bad_jobs) atomicAdd(a.bad_jobs, 0);   // (keeps the prefetch)
}

}  // namespace
}  // namespace hgk
