// Floor of one env-step launch at N envs: (a) an empty kernel, (b) a kernel that moves exactly the
// step's algorithmic bytes (state 27 + counters 3 + action 4 dwords read; state, counters, obs 17,
// reward and 3 flag bytes written; same SoA / [N,17] layouts) and computes nothing.  100 launches
// per hipGraph, HIP-event timed.  Diagnostic only (not part of the library).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__global__ void empty_kernel(float* p) {
    if (p == nullptr) p[threadIdx.x] = 0.f;
}

template <bool NT>
__global__ __launch_bounds__(256) void move_kernel(float* state, int32_t* ctr, const float4* act, float* obs, float* rew,
                                                   uint8_t* flags, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    float s[27];
    int32_t c[3];
#pragma unroll
    for (int k = 0; k < 27; ++k) s[k] = state[k * n + i];
#pragma unroll
    for (int k = 0; k < 3; ++k) c[k] = ctr[k * n + i];
    const float4 a = act[i];
    float acc = a.x + a.y + a.z + a.w;
#pragma unroll
    for (int k = 0; k < 27; ++k) { s[k] += acc; acc = acc * 0.5f; }
#pragma unroll
    for (int k = 0; k < 27; ++k) {
        if (NT) __builtin_nontemporal_store(s[k], state + k * n + i); else state[k * n + i] = s[k];
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) ctr[k * n + i] = c[k] + 1;
#pragma unroll
    for (int k = 0; k < 17; ++k) obs[i * 17 + k] = s[k];   // uncoalesced-by-lane but contiguous per wave
    rew[i] = acc;
    flags[i] = 1; flags[n + i] = 0; flags[2 * n + i] = 0;
}

int main(int argc, char** argv) {
    hipStream_t st;
    CK(hipStreamCreate(&st));
    for (int64_t n : {65536LL, 262144LL, 1048576LL}) {
        float *state, *obs, *rew, *act;
        int32_t* ctr;
        uint8_t* flags;
        CK(hipMalloc(&state, 27 * n * 4)); CK(hipMalloc(&ctr, 3 * n * 4)); CK(hipMalloc(&act, 16 * n));
        CK(hipMalloc(&obs, 68 * n)); CK(hipMalloc(&rew, 4 * n)); CK(hipMalloc(&flags, 3 * n));
        CK(hipMemset(state, 0, 27 * n * 4)); CK(hipMemset(ctr, 0, 12 * n)); CK(hipMemset(act, 0, 16 * n));
        const unsigned grid = (unsigned)((n + 255) / 256);
        for (int kind = 0; kind < 3; ++kind) {
            hipGraph_t g;
            hipGraphExec_t ge;
            CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
            for (int k = 0; k < 100; ++k) {
                if (kind == 0) hipLaunchKernelGGL(empty_kernel, dim3(grid), dim3(256), 0, st, state);
                else if (kind == 1) hipLaunchKernelGGL(move_kernel<false>, dim3(grid), dim3(256), 0, st, state, ctr, (const float4*)act, obs, rew, flags, n);
                else hipLaunchKernelGGL(move_kernel<true>, dim3(grid), dim3(256), 0, st, state, ctr, (const float4*)act, obs, rew, flags, n);
            }
            CK(hipStreamEndCapture(st, &g));
            CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
            for (int w = 0; w < 3; ++w) CK(hipGraphLaunch(ge, st));
            hipEvent_t e0, e1;
            CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
            CK(hipEventRecord(e0, st));
            for (int r = 0; r < 20; ++r) CK(hipGraphLaunch(ge, st));
            CK(hipEventRecord(e1, st));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            const double us = ms * 1e3 / 2000.0;
            const char* name = kind == 0 ? "empty" : (kind == 1 ? "move 331 B/env" : "move 331 B/env (nt state)");
            printf("N=%8lld %-26s %7.2f us/launch  %7.1f GB/s\n", (long long)n, name, us, kind ? 331.0 * n / us * 1e-3 : 0.0);
            CK(hipGraphExecDestroy(ge)); CK(hipGraphDestroy(g));
        }
        hipFree(state); hipFree(ctr); hipFree(act); hipFree(obs); hipFree(rew); hipFree(flags);
    }
    return 0;
}
