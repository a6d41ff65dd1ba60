// mover.hip — the step kernel's memory traffic with the arithmetic taken out (diagnostic, round 5).
//
// One launch moves exactly what step_kernel's bulk variant moves per env (315 B: reads 128 -- the
// 7 x 16-byte groups of the state tile, 112 B, and the float4 action; writes 187 -- the tile, the
// 68-byte observation row, the reward and the three flag bytes), with its access pattern:
//   * 64-thread blocks, one wave = one state tile [7][64][4] words, each group one dwordx4 per lane
//     from one uniform base (heligym_amd.hip ld_lane / st_lane, retrim.h tix),
//   * the action as one float4 per lane,
//   * the observations staged per wave in LDS (stride 17) and stored as 272 + 16 contiguous float4,
//   * reward a dword, terminated / truncated / info a byte each per lane, plain stores.
// BURN adds that many dependent-free VALU instructions per lane (4 independent fma chains) between
// the loads and the stores -- the step's own count is ~1 700 per wave on an aged population -- and
// LDS_PAD caps the resident waves per CU (the step's bulk variant runs three waves per SIMD, 12 per
// CU) by giving each one-wave block that much dynamic LDS.
// Usage: mover [N] -> per launch time (100 launches per hipGraph, HIP events) and achieved GB/s of the
// 315 bytes per env, for BURN in {0, 400, 800, 1200, 1700} x {unrestricted, 12, 8, 16 waves per CU}.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)
#define G1 __attribute__((address_space(1)))
typedef float f4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f4 ld4(const f4* base, uint32_t lane) { return *(const G1 f4*)((const G1 char*)base + lane * 16u); }
__device__ __forceinline__ void st4(f4* base, uint32_t lane, f4 v) { *(G1 f4*)((G1 char*)base + lane * 16u) = v; }

template <int BURN>
__global__ __launch_bounds__(64) void mover(float* state, const float* act, float* obs, float* rew, uint8_t* term,
                                            uint8_t* trunc, uint8_t* info, int64_t n) {
    __shared__ float s_obs[64 * 17];
    const int lane = threadIdx.x;
    const int64_t tile = blockIdx.x;
    const int64_t i = tile * 64 + lane;
    f4* tb = reinterpret_cast<f4*>(state + tile * 7 * 64 * 4);
    f4 g[7];
#pragma unroll
    for (int k = 0; k < 7; ++k) g[k] = ld4(tb + k * 64, lane);
    const f4 a = ld4(reinterpret_cast<const f4*>(act) + tile * 64, lane);
    // the loaded values feed the "work", the work feeds every store
    float c0 = g[0].x + a.x, c1 = g[1].y + a.y, c2 = g[2].z + a.z, c3 = g[3].w + a.w;
#pragma unroll
    for (int k = 0; k < BURN / 4; ++k) {
        asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(c0) : "v"(g[4].x), "v"(g[5].x));
        asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(c1) : "v"(g[4].y), "v"(g[5].y));
        asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(c2) : "v"(g[4].z), "v"(g[5].z));
        asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(c3) : "v"(g[4].w), "v"(g[5].w));
    }
    const float d = (c0 + c1) + (c2 + c3);
    float o[17];
#pragma unroll
    for (int k = 0; k < 17; ++k) o[k] = g[k % 7][k & 3] + d;
    if (i < n) {
        rew[i] = d;
        term[i] = (uint8_t)(d > 1e30f);
        trunc[i] = (uint8_t)(d < -1e30f);
        info[i] = (uint8_t)(d != d);
    }
#pragma unroll
    for (int k = 0; k < 17; ++k) s_obs[lane * 17 + k] = o[k];
    __builtin_amdgcn_wave_barrier();
    f4* out = reinterpret_cast<f4*>(obs + tile * 64 * 17);
    f4 v[5];
#pragma unroll
    for (int t = 0; t < 4; ++t) v[t] = *reinterpret_cast<const f4*>(s_obs + 4 * (lane + 64 * t));
    if (lane < 16) v[4] = *reinterpret_cast<const f4*>(s_obs + 4 * (lane + 256));
#pragma unroll
    for (int t = 0; t < 4; ++t) st4(out + 64 * t, lane, v[t]);
    if (lane < 16) st4(out + 256, lane, v[4]);
#pragma unroll
    for (int k = 0; k < 7; ++k) st4(tb + k * 64, lane, g[k] + d);
}

template <int BURN>
static int run(hipStream_t st, int64_t n, size_t lds_pad, float* state, float* act, float* obs, float* rew, uint8_t* fl,
               double* us_out) {
    const unsigned grid = (unsigned)(n / 64);
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
    for (int k = 0; k < 100; ++k)
        hipLaunchKernelGGL(mover<BURN>, dim3(grid), dim3(64), lds_pad, st, state, act, obs, rew, fl, fl + n, fl + 2 * n, n);
    CK(hipStreamEndCapture(st, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    for (int w = 0; w < 2; ++w) CK(hipGraphLaunch(ge, st));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0, st));
    for (int r = 0; r < 5; ++r) CK(hipGraphLaunch(ge, st));
    CK(hipEventRecord(e1, st));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    *us_out = ms * 1e3 / 500.0;
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
    return 0;
}

int main(int argc, char** argv) {
    const int64_t n = argc > 1 ? atoll(argv[1]) : 4194304;
    const int only = argc > 2 ? atoi(argv[2]) : -1;   // rocprofv3 passes: one (burn, pad) case
    if (n % 64) { printf("N must be a multiple of 64\n"); return 1; }
    hipStream_t st;
    CK(hipStreamCreate(&st));
    float *state, *act, *obs, *rew;
    uint8_t* fl;
    CK(hipMalloc(&state, 112 * n)); CK(hipMalloc(&act, 16 * n)); CK(hipMalloc(&obs, 68 * n));
    CK(hipMalloc(&rew, 4 * n)); CK(hipMalloc(&fl, 3 * n));
    CK(hipMemset(state, 0, 112 * n)); CK(hipMemset(act, 0, 16 * n));
    // W one-wave blocks per CU: 160 KB / W of LDS each (the kernel's static 4 352 B included); the
    // cases keep their round-5 indices (unrestricted 0-4, 12 per CU 5-9), 8 and 16 per CU follow
    auto pad_for = [](int w) { return (size_t)(160 * 1024 / w - 64 * 17 * 4); };
    int idx = 0;
    const int wpc[4] = {0, 12, 8, 16};
    for (int wi = 0; wi < 4; ++wi) {
        const size_t pad = wpc[wi] ? pad_for(wpc[wi]) : 0;
        double us[5];
        int rc = 0;
        const int burns[5] = {0, 400, 800, 1200, 1700};
        for (int b = 0; b < 5; ++b, ++idx) {
            if (only >= 0 && idx != only) { us[b] = 0; continue; }
            switch (b) {
                case 0: rc = run<0>(st, n, pad, state, act, obs, rew, fl, &us[b]); break;
                case 1: rc = run<400>(st, n, pad, state, act, obs, rew, fl, &us[b]); break;
                case 2: rc = run<800>(st, n, pad, state, act, obs, rew, fl, &us[b]); break;
                case 3: rc = run<1200>(st, n, pad, state, act, obs, rew, fl, &us[b]); break;
                default: rc = run<1700>(st, n, pad, state, act, obs, rew, fl, &us[b]); break;
            }
            if (rc) return rc;
            char wl[8];
            snprintf(wl, sizeof wl, "%d", wpc[wi]);
            printf("N=%lld waves/CU %-5s VALU/lane %4d: %8.2f us/launch  %7.1f GB/s (315 B/env)  %7.1f GB/s (318 B/env)\n",
                   (long long)n, wpc[wi] ? wl : "max", burns[b], us[b], 315.0 * n / us[b] * 1e-3, 318.0 * n / us[b] * 1e-3);
            fflush(stdout);
        }
    }
    return 0;
}
