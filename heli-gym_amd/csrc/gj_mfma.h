// gj_mfma.h -- the device trim's Newton solve  np.linalg.inv(dydx) @ (y - y*)  (helicopter_dynamics.py:
// 524-527) as a blocked Gauss-Jordan elimination with partial pivoting: four panels of four columns,
// each factored on the VALU with its rows replicated in every quarter of the wave, and the panel's
// whole row transformation applied to the rest of the system by ONE v_mfma_f64_16x16x4_f64.
//
// Why blocked (round 6): the unblocked solve (retrim_body.h gjr_step) spends each of its 16 pivot
// steps on lane shuffles (ds_bpermute, LDS latency on the step's chain) to bring the pivot row's
// columns to the quarters that own them.  Here the panel is replicated, so a pivot row's values are
// uniform (v_readlane), and the trailing columns are touched once per panel, by the matrix core.
//
// Layout: lane l, i = l & 15 (a row of the system), q = l >> 4.  The system lives in the f64 MFMA's
// C/D layout of J^T: register v of lane (i, q) holds J[i][4 v + q] ("slot" 4 v + q).  Slot 0 holds the
// right-hand side b instead of column 0 (column 0 belongs to panel 0, which is read from the
// evaluations directly and is dead after it), so the MFMAs carry b along with the trailing columns.
//
// Panel p (columns C = 4p .. 4p+3):
//   * its columns are gathered to every lane (permlane16/32 swaps of register p; panel 0 from LDS);
//   * four pivot steps on the replicated panel, unscaled (rows are never divided; each row keeps
//     1 / its pivot for the end): the pivot is the unused row with the largest |J[i][C]| (DPP max over
//     16 rows on the high word, as gjr_step), every other row adds g_i = -J[i][C] / pivot times the
//     pivot row, and the step's row operation is recorded in an augmented column a_k = g (0 at the
//     pivot row).  After the panel, E = I + A' S^T, with A' = [a_0..a_3] (16 x 4) and S^T the pivot-row
//     selector, is the panel's whole row transformation (E is the identity outside the pivot-row
//     columns; the lazily injected identity column of each pivot row makes A' = E[:, P] - S exact);
//   * the rest of the system: J^T <- J^T + J[P, :]^T A'^T, one MFMA with A = the pivot rows at panel
//     start (read from an LDS image of the system written at panel start) and B = A'^T (lane (i, q)
//     holds a_q[i]), C = D = the system.  Columns already eliminated and the panel's own come out as
//     garbage and are never read again.
// At the end slot 0 holds the unscaled right-hand side, and x[col of row i] = b[i] / pivot[i].
//
// Any stable partial-pivot solver is within fp64 rounding x cond (~3 000) of the reference's
// inv(J) @ r; the trims are compared with the host's serial trim at fp32 resolution.  A zero or
// non-finite pivot (a singular or non-finite system) makes its reciprocal, and with it the solution,
// non-finite: the caller checks the solution once.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace hgk {
namespace {

typedef double gjm_d4 __attribute__((ext_vector_type(4)));

#ifndef GJM_STAMP   // diagnostic builds (scripts/ubench/gj_solve.hip) time the phases
#define GJM_STAMP(k, x) do { } while (0)
#endif

constexpr int kImgStride = 17;   // doubles per row of the LDS image of the system (bank spread)

__device__ __forceinline__ double gjm_readlane(double v, int lane) {
    const uint64_t u = __double_as_longlong(v);
    const uint32_t lo = __builtin_amdgcn_readlane((int)(uint32_t)u, lane);
    const uint32_t hi = __builtin_amdgcn_readlane((int)(uint32_t)(u >> 32), lane);
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}

#ifndef GJM_RCP_NR   // Newton steps after v_rcp_f64 (A/B: scripts/gj_solve_check.py)
#define GJM_RCP_NR 2
#endif
__device__ __forceinline__ double gjm_rcp(double x) {   // v_rcp_f64 and GJM_RCP_NR fused Newton steps
    double r = __builtin_amdgcn_rcp(x);
#pragma unroll
    for (int k = 0; k < GJM_RCP_NR; ++k) r = fma(r, fma(-x, r, 1.0), r);
    return r;
}

__device__ __forceinline__ uint32_t gjm_row16_max(uint32_t k) {   // max over each 16-lane row (DPP)
    k = max(k, (uint32_t)__builtin_amdgcn_mov_dpp((int)k, 0x128, 0xF, 0xF, true));
    k = max(k, (uint32_t)__builtin_amdgcn_mov_dpp((int)k, 0x124, 0xF, 0xF, true));
    k = max(k, (uint32_t)__builtin_amdgcn_mov_dpp((int)k, 0x122, 0xF, 0xF, true));
    k = max(k, (uint32_t)__builtin_amdgcn_mov_dpp((int)k, 0x121, 0xF, 0xF, true));
    return k;
}

__device__ __forceinline__ double gjm_mk(uint32_t lo, uint32_t hi) {
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}

// o[k] = x of lane (l & 15) + 16 k, at every lane: permlane16_swap(x, x) gives the rows (x0 x0 x2 x2)
// and (x1 x1 x3 x3), a permlane32_swap of each with itself the four broadcasts
__device__ __forceinline__ void gjm_quarter_gather(double x, double (&o)[4]) {
    const uint64_t u = __double_as_longlong(x);
    const uint32_t lo = (uint32_t)u, hi = (uint32_t)(u >> 32);
    const auto l16 = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
    const auto h16 = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
    const auto l02 = __builtin_amdgcn_permlane32_swap(l16[0], l16[0], false, false);
    const auto h02 = __builtin_amdgcn_permlane32_swap(h16[0], h16[0], false, false);
    const auto l13 = __builtin_amdgcn_permlane32_swap(l16[1], l16[1], false, false);
    const auto h13 = __builtin_amdgcn_permlane32_swap(h16[1], h16[1], false, false);
    o[0] = gjm_mk(l02[0], h02[0]);
    o[2] = gjm_mk(l02[1], h02[1]);
    o[1] = gjm_mk(l13[0], h13[0]);
    o[3] = gjm_mk(l13[1], h13[1]);
}

struct GjmRow {   // per-lane bookkeeping of row i across the solve
    bool live;      // not yet a pivot row
    int mycol;      // the column this row was the pivot of
    double myinv;   // 1 / its pivot
};

// pivot step k of panel p (column C = 4 p + k) on the replicated panel c[] and augmented columns a[]
template <int PN, int K>
__device__ __forceinline__ void gjm_step(double (&c)[4], double (&a)[4], GjmRow& r, int& pq, int i, int q) {
    constexpr int C = 4 * PN + K;
    const double v = c[K];
    // |v|'s high word with the top bit set (so that a zero candidate still beats a used row); 0 once used
    const uint32_t key = r.live ? ((uint32_t)(__double_as_longlong(v) >> 32) | 0x80000000u) : 0u;
    const double own_inv = gjm_rcp(v);   // every row's reciprocal while the search runs (off its chain)
    const uint32_t mx = gjm_row16_max(key);
    // every quarter holds the same rows: the first hit is a lane of quarter 0, i.e. the row itself;
    // a live row always exists, so some lane hits
    const int P = __builtin_ctzll(__ballot(key == mx));
    const double rinv = gjm_readlane(own_inv, P);
    const bool piv = i == P;
    double g = v * -rinv;
    g = piv ? 0.0 : g;
#pragma unroll
    for (int j = K + 1; j < 4; ++j) c[j] = fma(g, gjm_readlane(c[j], P), c[j]);
#pragma unroll
    for (int j = 0; j < K; ++j) a[j] = fma(g, gjm_readlane(a[j], P), a[j]);
    a[K] = g;
    r.live = r.live && !piv;
    r.mycol = piv ? C : r.mycol;
    r.myinv = piv ? own_inv : r.myinv;
    pq = q == K ? P : pq;
    GJM_STAMP(8 * PN + 2 + K, c[K < 3 ? K + 1 : 3]);
}

// panel p: pivot steps on its replicated columns c[], then the MFMA update of the system R
template <int PN>
__device__ __forceinline__ void gjm_panel(gjm_d4& R, double (&c)[4], GjmRow& r, double* sImg, int i, int q) {
    // the LDS image of the system at panel start: the pivot rows' values for the MFMA's A operand
    double* row = sImg + i * kImgStride + q;
    row[0] = R[0];
    row[4] = R[1];
    row[8] = R[2];
    row[12] = R[3];
    GJM_STAMP(8 * PN, R[0]);
    if constexpr (PN > 0) gjm_quarter_gather(R[PN], c);
    GJM_STAMP(8 * PN + 1, c[0]);
    double a[4];
    int pq = 0;   // the pivot row of pivot step q of this panel (lane (i, q))
    gjm_step<PN, 0>(c, a, r, pq, i, q);
    gjm_step<PN, 1>(c, a, r, pq, i, q);
    gjm_step<PN, 2>(c, a, r, pq, i, q);
    gjm_step<PN, 3>(c, a, r, pq, i, q);
    // A[row i][k = q] = J[P_q][slot i] at panel start; B[k = q][col i] = a_q[i]
    const double aop = sImg[pq * kImgStride + i];
    double bop = a[0];   // selects, not a branch on q
    bop = q == 1 ? a[1] : bop;
    bop = q == 2 ? a[2] : bop;
    bop = q == 3 ? a[3] : bop;
    GJM_STAMP(8 * PN + 6, aop);
    R = __builtin_amdgcn_mfma_f64_16x16x4f64(aop, bop, R, 0, 0, 0);
}

// Solve J x = b for one 16 x 16 system, one wave.  J[i][c] = (sE[c * es + i] - sE[(c + 16) * es + i]) * s
// (central differences of the evaluations, retrim_body.h), b[i] = sE[src * es + i] - sYt[i].  sImg:
// 16 * kImgStride doubles of LDS scratch.  Lanes 0..15 write x to sX (by column); the caller orders
// LDS and checks x for finiteness.
__device__ __forceinline__ void gjm_solve(const double* sE, int es, double s, int src, const double* sYt,
                                          double* sImg, double* sX, int l) {
    const int i = l & 15, q = l >> 4;
    double c[4];
    gjm_d4 R;
#pragma unroll
    for (int k = 0; k < 4; ++k) c[k] = sE[k * es + i];
    double e1 = sE[(q + 4) * es + i], e2 = sE[(q + 8) * es + i], e3 = sE[(q + 12) * es + i];
    double m[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) m[k] = sE[(k + 16) * es + i];
    const double m1 = sE[(q + 20) * es + i], m2 = sE[(q + 24) * es + i], m3 = sE[(q + 28) * es + i];
    const double b = sE[src * es + i] - sYt[i];
#pragma unroll
    for (int k = 0; k < 4; ++k) c[k] = (c[k] - m[k]) * s;
    R[0] = b;
    R[1] = (e1 - m1) * s;
    R[2] = (e2 - m2) * s;
    R[3] = (e3 - m3) * s;
    GjmRow r{true, 0, 0.0};
    gjm_panel<0>(R, c, r, sImg, i, q);
    gjm_panel<1>(R, c, r, sImg, i, q);
    gjm_panel<2>(R, c, r, sImg, i, q);
    gjm_panel<3>(R, c, r, sImg, i, q);
    GJM_STAMP(32, R[0]);
    if (l < 16) sX[r.mycol] = R[0] * r.myinv;
}


// ---------------------------------------------------------------------------------------------------
// The same blocked solve with the pivot order given (round 6): the rows are loaded permuted so that
// pivot step C pivots lane C (row perm[C] of the system) on column C, the order partial pivoting took
// on the host's trim of the same condition (hg::TrimSetup::piv, that Newton step's own order).  With
// the pivot lane known at compile time there is no search, and the pivot row reaches the other rows
// with a DPP row_newbcast inside the instruction that uses it (v_rcp_f64_dpp, v_fmac_f64_dpp): a step
// is the pivot's reciprocal (one Newton step), the multipliers, and one fused update per element.
// Its dependent chain is five instructions.
//   * Rows stay unscaled (the pivot row's multiplier is 0); x[C] = b[C] / pivot at the end.
//   * The augmented columns are one register: quarter q carries column q of Aug - S, Aug = E[:, P]
//     (the lazily injected identity column e_{4p+q} from the panel's start) less that identity column,
//     and one v_fmac_f64_dpp per step updates all four quarters -- the broadcast from lane C of each
//     quarter is the pivot row's entry of that quarter's column -- plus the identity's share in
//     quarter K.  The MFMAs then take the system itself as C: J + (Aug - S) S^T J = E J (no selects
//     zeroing the pivot rows on the chain).
//   * The next panel's columns come out of a second MFMA already replicated over the quarters (the
//     rows of its A operand repeat each pivot row's entry of those columns), and every LDS address a
//     panel needs is known before its pivots are: no lane shuffle and no LDS wait on the step chain.
//
// A given pivot order is not partial pivoting for this Jacobian, so the solution is accepted only if
// its residual is that of a backward-stable solve: |J x - b|_i <= kGjsTol (sum_c |J_ic| |x_c| + |b_i|)
// for every row (the pivoted solves' residuals are orders of magnitude below that scale,
// profiles/r06_gj_solve.txt); otherwise the caller runs the searched solve (gjm_solve).
constexpr double kGjsTol = 1e-13;
#ifndef GJS_RCP_DPP
#define GJS_RCP_DPP 0
#endif

// Hazards: the compiler pads only around the instructions it generates.  Each asm below starts with
// the 2 wait states a DPP read needs after a VALU write of its source; the other hazards around them
// are kept out by construction -- no asm reads an MFMA result (a panel's first broadcast of the
// MFMA's columns is the builtin form, which the compiler pads, and the chain after it outlasts the
// MFMA's latency before any asm reads the other columns), and the MFMA's B operand gets its last
// update from the builtin form too.
template <int C>
__device__ __forceinline__ double gjs_bcast(double v) {   // v of lane C of each 16-lane row
    double r;
    asm("s_nop 1\n\tv_mov_b64_dpp %0, %1 row_newbcast:%2 row_mask:0xf bank_mask:0xf" : "=v"(r) : "v"(v), "n"(C & 15));
    return r;
}
template <int C>
__device__ __forceinline__ double gjs_bcast_c(double v) {   // the same, compiler-generated (hazards padded)
    return __builtin_amdgcn_update_dpp(v, v, 0x150 + (C & 15), 0xF, 0xF, true);
}
template <int C>
__device__ __forceinline__ double gjs_rcp_bcast(double v) {   // v_rcp_f64 of lane C's v
    double r;
    asm("s_nop 1\n\tv_rcp_f64_dpp %0, %1 row_newbcast:%2 row_mask:0xf bank_mask:0xf" : "=v"(r) : "v"(v), "n"(C & 15));
    return r;
}
template <int C>
__device__ __forceinline__ void gjs_fmac_bcast(double& acc, double g) {   // acc += acc[lane C] * g
    asm("s_nop 1\n\tv_fmac_f64_dpp %0, %0, %1 row_newbcast:%2 row_mask:0xf bank_mask:0xf" : "+v"(acc) : "v"(g), "n"(C & 15));
}

__device__ __forceinline__ double gjs_quarter_sum(double x) {   // sum over the four quarters, at every lane
    uint64_t u = __double_as_longlong(x);
    auto lo = __builtin_amdgcn_permlane16_swap((uint32_t)u, (uint32_t)u, false, false);
    auto hi = __builtin_amdgcn_permlane16_swap((uint32_t)(u >> 32), (uint32_t)(u >> 32), false, false);
    const double t = gjm_mk(lo[0], hi[0]) + gjm_mk(lo[1], hi[1]);   // (x0+x1, x0+x1, x2+x3, x2+x3)
    u = __double_as_longlong(t);
    lo = __builtin_amdgcn_permlane32_swap((uint32_t)u, (uint32_t)u, false, false);
    hi = __builtin_amdgcn_permlane32_swap((uint32_t)(u >> 32), (uint32_t)(u >> 32), false, false);
    return gjm_mk(lo[0], hi[0]) + gjm_mk(lo[1], hi[1]);
}

template <int PN, int K>
__device__ __forceinline__ void gjs_step(double (&c)[4], double& bop, double& myinv, int i, int q) {
    constexpr int C = 4 * PN + K;
    const double cz = c[K] * (i == C ? 0.0 : 1.0);   // (off the chain) the pivot row is not updated
    const double p = K == 0 ? gjs_bcast_c<C>(c[K]) : gjs_bcast<C>(c[K]);   // the pivot J[C][C]
#if GJS_RCP_DPP
    double r = gjs_rcp_bcast<C>(c[K]);
#else
    double r = __builtin_amdgcn_rcp(p);
#endif
    r = fma(r, fma(-p, r, 1.0), r);                  // one Newton step: within 1e-14 (the residual test guards)
    const double g = -cz * r;                        // -J[i][C] / pivot
#pragma unroll
    for (int j = K + 1; j < 4; ++j) gjs_fmac_bcast<C>(c[j], g);
    // bop = Aug - S (quarter q: column q of Aug less the identity column e_{4 PN + q}), whose pivot-row
    // entry is Aug's less 1 in quarter K: Aug += Aug[C] g is bop += bop[C] g + [q == K] g
    const double dk = q == K ? 1.0 : 0.0;
    if constexpr (K < 3) {
        gjs_fmac_bcast<C>(bop, g);
        bop = fma(dk, g, bop);
    } else {
        bop = fma(gjs_bcast_c<C>(bop) + dk, g, bop);  // (the MFMA's B operand: a padded write)
    }
    myinv = i == C ? r : myinv;
    GJM_STAMP(8 * PN + 2 + K, c[K < 3 ? K + 1 : 3]);
}

// the LDS image of the system for panel PN's MFMA operands, written at its start
__device__ __forceinline__ void gjs_image(const gjm_d4& R, double* sImg, int i, int q) {
    double* row = sImg + i * kImgStride + q;
    row[0] = R[0];
    row[4] = R[1];
    row[8] = R[2];
    row[12] = R[3];
}
template <int PN>
struct GjsOps {   // panel PN's MFMA operands, read from its image as soon as it is written
    double aop, a2op;
    double c2[4];
    __device__ __forceinline__ void read(const double* sImg, int i, int q) {
        aop = sImg[(4 * PN + q) * kImgStride + i];   // A[slot i][k = q] = J[4 PN + q][slot i]
        if constexpr (PN < 3) {
            // next panel's columns, replicated: A2[r][k] = J[4 PN + k][4 (PN + 1) + (r >> 2)], C2 = its rows
            a2op = sImg[(4 * PN + q) * kImgStride + 4 * (PN + 1) + (i >> 2)];
#pragma unroll
            for (int v = 0; v < 4; ++v) c2[v] = sImg[i * kImgStride + 4 * (PN + 1) + v];
        }
    }
};

template <int PN>
__device__ __forceinline__ void gjs_panel(gjm_d4& R, double (&c)[4], GjsOps<PN>& ops, double& myinv, double* sImg,
                                          int i, int q) {
    GJM_STAMP(8 * PN, c[0]);
    double bop = 0.0;   // Aug - S before the panel (Aug's columns: the identity's)
    gjs_step<PN, 0>(c, bop, myinv, i, q);
    gjs_step<PN, 1>(c, bop, myinv, i, q);
    if constexpr (PN > 0) {   // this panel's image (the previous MFMA's system), off the step chain
        // (the write waits for that MFMA: kept after step 1, where it has long completed)
        __builtin_amdgcn_sched_barrier(0);
        gjs_image(R, sImg, i, q);
        ops.read(sImg, i, q);
        // (a scheduling barrier: the image and the operand reads stay here, their LDS latency under
        // steps 2 and 3, instead of being sunk to the MFMAs on the chain)
        __builtin_amdgcn_sched_barrier(0);
    }
    gjs_step<PN, 2>(c, bop, myinv, i, q);
    gjs_step<PN, 3>(c, bop, myinv, i, q);
    GJM_STAMP(8 * PN + 6, bop);
    // E J = J + (Aug - S) S^T J: C is the system itself (no pivot-row zeroing)
    if constexpr (PN < 3) {   // the next panel's columns first: the step chain waits for them only
        const gjm_d4 c2 = {ops.c2[0], ops.c2[1], ops.c2[2], ops.c2[3]};
        const gjm_d4 nx = __builtin_amdgcn_mfma_f64_16x16x4f64(ops.a2op, bop, c2, 0, 0, 0);
        c[0] = nx[0];
        c[1] = nx[1];
        c[2] = nx[2];
        c[3] = nx[3];
    }
    R = __builtin_amdgcn_mfma_f64_16x16x4f64(ops.aop, bop, R, 0, 0, 0);
    // (both MFMAs issue here: the system's is not deferred past the next panel's steps, whose image
    // write would then wait for it on the chain)
    __builtin_amdgcn_sched_barrier(0);
}

// GJS_BLOCK_INV: the panel's four pivot steps replaced by the inverse of its 4 x 4 pivot block D (rows
// 4 PN .. 4 PN + 3 of the panel's columns, broadcast to every lane).  Quarter q solves D y = e_q by
// elimination in the given order (the pivots are the four steps' own), so the lanes of quarter q hold
// column q of D^-1, and the panel's transformation is E = I + A S^T with A = (S - M) D^-1 (M: the
// panel's columns; the pivot rows come out scaled to the identity, so x needs no division at the
// end).  Four dependent reciprocals and the eliminations between them instead of four steps with a
// broadcast, a reciprocal and an update chain each.
#ifndef GJS_BLOCK_INV
#define GJS_BLOCK_INV 1
#endif
__device__ __forceinline__ double gjs_rcp1(double p) {   // v_rcp_f64 and one Newton step
    const double r = __builtin_amdgcn_rcp(p);
    return fma(r, fma(-p, r, 1.0), r);
}
template <int PN>
__device__ __forceinline__ void gjs_panel_blk(gjm_d4& R, double (&c)[4], GjsOps<PN>& ops, double* sImg, int i, int q) {
    constexpr int C0 = 4 * PN;
    GJM_STAMP(8 * PN, c[0]);
    double d[4][4];   // D[k][v] = c[v] of lane C0 + k (every quarter holds the same rows)
#pragma unroll
    for (int v = 0; v < 4; ++v) {
        d[0][v] = gjs_bcast_c<C0>(c[v]);
        d[1][v] = gjs_bcast_c<C0 + 1>(c[v]);
        d[2][v] = gjs_bcast_c<C0 + 2>(c[v]);
        d[3][v] = gjs_bcast_c<C0 + 3>(c[v]);
    }
    double e0 = q == 0 ? 1.0 : 0.0, e1 = q == 1 ? 1.0 : 0.0, e2 = q == 2 ? 1.0 : 0.0, e3 = q == 3 ? 1.0 : 0.0;
    double w[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) w[k] = (i == C0 + k ? 1.0 : 0.0) - c[k];
    // elimination in the given order (the pivots are D's leading diagonal as it is reduced)
    const double r0 = gjs_rcp1(d[0][0]);
    {
        const double l1 = d[1][0] * r0, l2 = d[2][0] * r0, l3 = d[3][0] * r0;
#pragma unroll
        for (int v = 1; v < 4; ++v) {
            d[1][v] = fma(-l1, d[0][v], d[1][v]);
            d[2][v] = fma(-l2, d[0][v], d[2][v]);
            d[3][v] = fma(-l3, d[0][v], d[3][v]);
        }
        e1 = fma(-l1, e0, e1);
        e2 = fma(-l2, e0, e2);
        e3 = fma(-l3, e0, e3);
    }
    GJM_STAMP(8 * PN + 2, d[1][1]);
    if constexpr (PN > 0) {   // this panel's image (the previous MFMA's system), off the chain
        __builtin_amdgcn_sched_barrier(0);
        gjs_image(R, sImg, i, q);
        ops.read(sImg, i, q);
        __builtin_amdgcn_sched_barrier(0);
    }
    const double r1 = gjs_rcp1(d[1][1]);
    {
        const double l2 = d[2][1] * r1, l3 = d[3][1] * r1;
#pragma unroll
        for (int v = 2; v < 4; ++v) {
            d[2][v] = fma(-l2, d[1][v], d[2][v]);
            d[3][v] = fma(-l3, d[1][v], d[3][v]);
        }
        e2 = fma(-l2, e1, e2);
        e3 = fma(-l3, e1, e3);
    }
    GJM_STAMP(8 * PN + 3, d[2][2]);
    const double r2 = gjs_rcp1(d[2][2]);
    {
        const double l3 = d[3][2] * r2;
        d[3][3] = fma(-l3, d[2][3], d[3][3]);
        e3 = fma(-l3, e2, e3);
    }
    const double r3 = gjs_rcp1(d[3][3]);
    // back substitution: y = column q of D^-1
    const double y3 = e3 * r3;
    const double y2 = fma(-d[2][3], y3, e2) * r2;
    const double y1 = fma(-d[1][2], y2, fma(-d[1][3], y3, e1)) * r1;
    const double y0 = fma(-d[0][1], y1, fma(-d[0][2], y2, fma(-d[0][3], y3, e0))) * r0;
    GJM_STAMP(8 * PN + 4, y0);
    // bop = A[i][q] = sum_k W[i][k] y_k with W = S - M (formed off the chain, as soon as c is)
    const double bop = fma(w[0], y0, fma(w[1], y1, fma(w[2], y2, w[3] * y3)));
    GJM_STAMP(8 * PN + 6, bop);
    if constexpr (PN < 3) {   // the next panel's columns first: the chain waits for them only
        const gjm_d4 c2 = {ops.c2[0], ops.c2[1], ops.c2[2], ops.c2[3]};
        const gjm_d4 nx = __builtin_amdgcn_mfma_f64_16x16x4f64(ops.a2op, bop, c2, 0, 0, 0);
        c[0] = nx[0];
        c[1] = nx[1];
        c[2] = nx[2];
        c[3] = nx[3];
    }
    R = __builtin_amdgcn_mfma_f64_16x16x4f64(ops.aop, bop, R, 0, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
}

// Solve with the pivot order perm (perm[C] = the row that pivots column C).  Returns whether the
// solution passed the residual test (wave-uniform; a pass implies every component is finite); x is in
// sX either way.
__device__ __forceinline__ bool gjs_solve(const double* sE, int es, double s, int src, const double* sYt,
                                          const int8_t* perm, double* sImg, double* sX, int l) {
    const int i = l & 15, q = l >> 4;
    const int pi = perm[i];
    double c[4], m[4], e[3], me[3];
    gjm_d4 R;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        c[k] = sE[k * es + pi];
        m[k] = sE[(k + 16) * es + pi];
    }
#pragma unroll
    for (int v = 1; v < 4; ++v) {
        e[v - 1] = sE[(q + 4 * v) * es + pi];
        me[v - 1] = sE[(q + 4 * v + 16) * es + pi];
    }
    const double b = sE[src * es + pi] - sYt[pi];
#pragma unroll
    for (int k = 0; k < 4; ++k) c[k] = (c[k] - m[k]) * s;
    R[0] = b;
#pragma unroll
    for (int v = 1; v < 4; ++v) R[v] = (e[v - 1] - me[v - 1]) * s;
    const double j0[4] = {c[0], c[1], c[2], c[3]};   // the system as given, for the residual test
    const double j1[3] = {R[1], R[2], R[3]};
    gjs_image(R, sImg, i, q);
    GjsOps<0> o0;
    o0.read(sImg, i, q);
    GjsOps<1> o1;
    GjsOps<2> o2;
    GjsOps<3> o3;
#if GJS_BLOCK_INV
    gjs_panel_blk<0>(R, c, o0, sImg, i, q);
    gjs_panel_blk<1>(R, c, o1, sImg, i, q);
    gjs_panel_blk<2>(R, c, o2, sImg, i, q);
    gjs_panel_blk<3>(R, c, o3, sImg, i, q);
    GJM_STAMP(32, R[0]);
    if (l < 16) sX[i] = R[0];   // (the pivot rows scaled to the identity)
#else
    double myinv = 0.0;
    gjs_panel<0>(R, c, o0, myinv, sImg, i, q);
    gjs_panel<1>(R, c, o1, myinv, sImg, i, q);
    gjs_panel<2>(R, c, o2, myinv, sImg, i, q);
    gjs_panel<3>(R, c, o3, myinv, sImg, i, q);
    GJM_STAMP(32, R[0]);
    if (l < 16) sX[i] = R[0] * myinv;
#endif
    // the residual of the permuted system: J x - b from the system as given
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    double x0[4], xs[3];
#pragma unroll
    for (int k = 0; k < 4; ++k) x0[k] = sX[k];
#pragma unroll
    for (int v = 1; v < 4; ++v) xs[v - 1] = sX[q + 4 * v];
    double dot = 0.0, mag = 0.0, dot0 = 0.0, mag0 = 0.0;
#pragma unroll
    for (int v = 0; v < 3; ++v) {
        dot = fma(j1[v], xs[v], dot);
        mag = fma(fabs(j1[v]), fabs(xs[v]), mag);
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {   // columns 0..3: every quarter holds the whole row part
        dot0 = fma(j0[k], x0[k], dot0);
        mag0 = fma(fabs(j0[k]), fabs(x0[k]), mag0);
    }
    const double r = (gjs_quarter_sum(dot) + dot0) - b;
    const double scale = (gjs_quarter_sum(mag) + mag0) + fabs(b);
    // (a non-finite x fails: a NaN compares false, and an infinite one makes the scale infinite; the
    // lanes together hold every component, so the caller need not check x again)
    const bool good = fabs(r) <= kGjsTol * scale && scale < INFINITY;
    GJM_STAMP(33, r);
    return __ballot(!good) == 0;
}

}  // namespace
}  // namespace hgk
