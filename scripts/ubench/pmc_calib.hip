// Calibration of rocprofv3's FETCH_SIZE / WRITE_SIZE on gfx950 for the step kernel's own access
// widths: kernels that move a known byte count with 4-B-per-lane (the state columns) and
// 16-B-per-lane (the actions, the observation write-back) coalesced loads and stores, at an
// Infinity-Cache-resident size (21 MB, the step's working set at 65 536 envs) and past the 256 MB
// MALL (1.34 GB).  scripts/pmc_calib.sh runs it under separate --pmc passes and
// scripts/summarize_calib.py divides the counters by the known bytes.  Diagnostic only.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

// every lane reads `cols` dwords, one per column of a [cols][n] array (the state tiles' pattern)
__global__ __launch_bounds__(256) void rd_dword(const float* __restrict__ src, float* __restrict__ sink, int64_t n,
                                                int cols) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    float acc = 0.f;
    for (int c = 0; c < cols; ++c) acc += src[(int64_t)c * n + i];
    if (acc == 1234.5f) sink[0] = acc;   // never true for the zero-filled input: no writes
}

__global__ __launch_bounds__(256) void rd_x4(const float4* __restrict__ src, float* __restrict__ sink, int64_t n4) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const float4 v = src[i];
    if (v.x + v.y + v.z + v.w == 1234.5f) sink[0] = v.x;
}

__global__ __launch_bounds__(256) void wr_dword(float* __restrict__ dst, int64_t n, int cols) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    for (int c = 0; c < cols; ++c) dst[(int64_t)c * n + i] = (float)c;
}

__global__ __launch_bounds__(256) void wr_x4(float4* __restrict__ dst, int64_t n4) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    dst[i] = make_float4(1.f, 2.f, 3.f, 4.f);
}

int main() {
    const int cols = 30;
    float* sink;
    CK(hipMalloc(&sink, 256));
    // n envs x 30 dwords: 65 536 -> 7.9 MB per direction (in cache); 11 184 810 -> 1.34 GB (past the MALL)
    for (int64_t n : {(int64_t)65536 * 3, (int64_t)11184640}) {
        const int64_t bytes = n * cols * 4;
        float* buf;
        CK(hipMalloc(&buf, bytes));
        CK(hipMemset(buf, 0, bytes));
        const unsigned g1 = (unsigned)(n / 256), g4 = (unsigned)(bytes / 16 / 256);
        for (int rep = 0; rep < 3; ++rep) {
            hipLaunchKernelGGL(rd_dword, dim3(g1), dim3(256), 0, 0, buf, sink, n, cols);
            hipLaunchKernelGGL(rd_x4, dim3(g4), dim3(256), 0, 0, (const float4*)buf, sink, bytes / 16);
            hipLaunchKernelGGL(wr_dword, dim3(g1), dim3(256), 0, 0, buf, n, cols);
            hipLaunchKernelGGL(wr_x4, dim3(g4), dim3(256), 0, 0, (float4*)buf, bytes / 16);
            CK(hipMemset(buf, 0, bytes));
        }
        CK(hipDeviceSynchronize());
        printf("n=%lld bytes per kernel %lld\n", (long long)n, (long long)bytes);
        CK(hipFree(buf));
    }
    return 0;
}
