// Diagnostic (not part of the library): the device trim's 16 x 16 Newton solve on its own, one wave per
// system -- the blocked Gauss-Jordan on v_mfma_f64_16x16x4_f64 (csrc/gj_mfma.h) against the unblocked
// split-row solve (csrc/retrim_body.h gjr_steps) -- with s_memtime around each.  Built as a shared
// library and driven by scripts/gj_solve_check.py, which compares both with numpy.linalg.solve.
#include <hip/hip_runtime.h>
#include <stdint.h>

__device__ unsigned long long g_gjm_t[40];
#ifndef GJ_NO_STAMPS
#define GJM_STAMP(k, val)                                                            \
    do {                                                                             \
        asm volatile("" ::"v"(val));                                                 \
        const unsigned long long t_ = __builtin_amdgcn_s_memtime();                  \
        if (threadIdx.x == 0 && blockIdx.x == 0) g_gjm_t[(k)] = t_;                 \
    } while (0)
#endif
#include "../../heli-gym_amd/csrc/gj_mfma.h"
#include "../../heli-gym_amd/csrc/retrim_body.h"

namespace {
constexpr int ES = hgk::kEStride;

template <int which>
__global__ __launch_bounds__(64) void solve_kernel(const double* J, const double* b, const int8_t* perms, int n,
                                                   double* x, unsigned long long* cyc, int* fell_back) {
    __shared__ int8_t sPerm[16];
    __shared__ double sE[42 * ES];
    __shared__ double sYt[16];
    __shared__ double sX[16];
    __shared__ double sImg[16 * hgk::kImgStride];
    const int l = threadIdx.x;
    for (int job = blockIdx.x; job < n; job += gridDim.x) {
        const double* Jj = J + job * 256;
        if (l < 16) {
            for (int c = 0; c < 16; ++c) {
                sE[c * ES + l] = Jj[l * 16 + c];
                sE[(c + 16) * ES + l] = 0.0;
            }
            sE[32 * ES + l] = b[job * 16 + l];
            sYt[l] = 0.0;
            sPerm[l] = perms ? perms[job * 16 + l] : (int8_t)l;
        }
        __syncthreads();
        unsigned long long t0 = __builtin_amdgcn_s_memtime();
        if constexpr (which == 0) {
            hgk::gjm_solve(sE, ES, 1.0, 32, sYt, sImg, sX, l);
        } else if constexpr (which == 2) {
            const bool ok = hgk::gjs_solve(sE, ES, 1.0, 32, sYt, sPerm, sImg, sX, l);
            if (!ok) {
                __syncthreads();
                hgk::gjm_solve(sE, ES, 1.0, 32, sYt, sImg, sX, l);
            }
            if (l == 0) fell_back[job] = ok ? 0 : 1;
        } else {
            const int i = l & 15, q = l >> 4;
            double A4[4], Em4[4];
            for (int jj = 0; jj < 4; ++jj) {
                A4[jj] = sE[(4 * jj + q) * ES + i];
                Em4[jj] = sE[(4 * jj + q + 16) * ES + i];
            }
            double bb = sE[32 * ES + i] - sYt[i];
            for (int jj = 0; jj < 4; ++jj) A4[jj] = (A4[jj] - Em4[jj]) * 1.0;
            uint32_t live = 0xFFFFFFFFu;
            int mycol = 0;
            double rep = (sE[i] - sE[16 * ES + i]) * 1.0;
            double nx1 = (sE[ES + i] - sE[17 * ES + i]) * 1.0;
            double nx2 = (sE[2 * ES + i] - sE[18 * ES + i]) * 1.0;
            hgk::gjr_steps<0>(A4, bb, rep, nx1, nx2, live, mycol, i, l);
            if (l < 16) sX[mycol] = bb;
        }
        __syncthreads();
        unsigned long long t1 = __builtin_amdgcn_s_memtime();
        if (l < 16) x[job * 16 + l] = sX[l];
        if (l == 0) cyc[job] = t1 - t0;
        __syncthreads();
    }
}
}  // namespace

// the accuracy of v_rcp_f64 and of 1 / 2 Newton steps after it, on n values (out: 3 relative errors each)
__global__ void rcp_kernel(const double* x, double* err, int n) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    const double v = x[k];
    double r = __builtin_amdgcn_rcp(v);
    err[3 * k] = fabs(r * v - 1.0);
    r = fma(r, fma(-v, r, 1.0), r);
    err[3 * k + 1] = fabs(fma(r, v, -1.0));
    r = fma(r, fma(-v, r, 1.0), r);
    err[3 * k + 2] = fabs(fma(r, v, -1.0));
}
extern "C" int gj_rcp_check(const double* x, double* err, int n) {
    double *dx, *de;
    if (hipMalloc(&dx, 8 * n) || hipMalloc(&de, 24 * n)) return -1;
    (void)hipMemcpy(dx, x, 8 * n, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(rcp_kernel, dim3((n + 255) / 256), dim3(256), 0, 0, dx, de, n);
    if (hipDeviceSynchronize() != hipSuccess) return -2;
    (void)hipMemcpy(err, de, 24 * n, hipMemcpyDeviceToHost);
    (void)hipFree(dx);
    (void)hipFree(de);
    return 0;
}

// DPP semantics check: out[l] = {v_mov_b64_dpp row_newbcast:3 of in, v_rcp_f64_dpp row_newbcast:3 of in,
// v_fmac_f64_dpp acc=in, g=2 row_newbcast:3} for one wave
__global__ void dpp_kernel(const double* in, double* out) {
    const int l = threadIdx.x;
    const double v = in[l];
    const double b = hgk::gjs_bcast<3>(v);
    const double r = hgk::gjs_rcp_bcast<3>(v);
    double acc = v;
    hgk::gjs_fmac_bcast<3>(acc, 2.0);
    out[3 * l] = b;
    out[3 * l + 1] = r;
    out[3 * l + 2] = acc;
}
extern "C" int gj_dpp_check(const double* in, double* out) {
    double *di, *dout;
    if (hipMalloc(&di, 8 * 64) || hipMalloc(&dout, 8 * 192)) return -1;
    (void)hipMemcpy(di, in, 8 * 64, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(dpp_kernel, dim3(1), dim3(64), 0, 0, di, dout);
    if (hipDeviceSynchronize() != hipSuccess) return -2;
    (void)hipMemcpy(out, dout, 8 * 192, hipMemcpyDeviceToHost);
    (void)hipFree(di);
    (void)hipFree(dout);
    return 0;
}

extern "C" int gj_solve_stamps(unsigned long long* dst) {
    return hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_gjm_t), sizeof(unsigned long long) * 40) == hipSuccess ? 0 : -1;
}

extern "C" int gj_solve_run(const double* J, const double* b, const int8_t* perms, int n, int which, double* x,
                            unsigned long long* cyc, int* fell_back, int grid) {
    double *dJ, *db, *dx;
    unsigned long long* dc;
    int8_t* dp = nullptr;
    int* df;
    if (hipMalloc(&dJ, sizeof(double) * 256 * n) || hipMalloc(&db, sizeof(double) * 16 * n) ||
        hipMalloc(&dx, sizeof(double) * 16 * n) || hipMalloc(&dc, sizeof(unsigned long long) * n) ||
        hipMalloc(&df, sizeof(int) * n) || (perms && hipMalloc(&dp, 16 * n)))
        return -1;
    (void)hipMemcpy(dJ, J, sizeof(double) * 256 * n, hipMemcpyHostToDevice);
    (void)hipMemcpy(db, b, sizeof(double) * 16 * n, hipMemcpyHostToDevice);
    (void)hipMemset(df, 0, sizeof(int) * n);
    if (perms) (void)hipMemcpy(dp, perms, 16 * n, hipMemcpyHostToDevice);
    for (int rep = 0; rep < 2; ++rep) {
        if (which == 0) hipLaunchKernelGGL(solve_kernel<0>, dim3(grid), dim3(64), 0, 0, dJ, db, dp, n, dx, dc, df);
        else if (which == 2) hipLaunchKernelGGL(solve_kernel<2>, dim3(grid), dim3(64), 0, 0, dJ, db, dp, n, dx, dc, df);
        else hipLaunchKernelGGL(solve_kernel<1>, dim3(grid), dim3(64), 0, 0, dJ, db, dp, n, dx, dc, df);
    }
    if (hipDeviceSynchronize() != hipSuccess) return -2;
    (void)hipMemcpy(x, dx, sizeof(double) * 16 * n, hipMemcpyDeviceToHost);
    (void)hipMemcpy(cyc, dc, sizeof(unsigned long long) * n, hipMemcpyDeviceToHost);
    (void)hipMemcpy(fell_back, df, sizeof(int) * n, hipMemcpyDeviceToHost);
    (void)hipFree(df);
    if (dp) (void)hipFree(dp);
    (void)hipFree(dJ);
    (void)hipFree(db);
    (void)hipFree(dx);
    (void)hipFree(dc);
    return 0;
}
