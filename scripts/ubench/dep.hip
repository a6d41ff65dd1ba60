// Microbenchmark (diagnostic, not part of the library): what one wave alone on its SIMD pays per
// instruction on gfx950 -- dependent chains of v_fma_f32 / v_pk_fma_f32 / transcendentals, 1-4
// interleaved chains, and VALU interleaved with SALU / s_nop (does a scalar instruction cost the
// lone wave an issue slot?).  Each asm block is 16 copies of a short sequence (no compiler-inserted
// hazard nops inside).  Grid: one 64-lane block per SIMD (256 CUs x 4).
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef float f2 __attribute__((ext_vector_type(2)));
#define S4(x) x x x x
#define S16(x) S4(x) S4(x) S4(x) S4(x)

template <int K>
__global__ void __launch_bounds__(64) k(float* out, unsigned long long* cyc, int iters) {
    float a = threadIdx.x * 1e-3f + 1.f, b = a + 1, c = a + 2, d = a + 3;
    f2 p = {a, b}, q = {c, d}, r = {a, c}, s = {b, d};
    const float m = 0.999f, n = 0.001f;
    const f2 mm = {m, m}, nn = {n, n};
    int si = blockIdx.x;
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; ++i) {
        if (K == 0) asm volatile(S16("v_fma_f32 %0, %0, %1, %2\n") : "+v"(a) : "v"(m), "v"(n));
        if (K == 1) asm volatile(S16("v_fma_f32 %0, %0, %2, %3\n v_fma_f32 %1, %1, %2, %3\n") : "+v"(a), "+v"(b) : "v"(m), "v"(n));
        if (K == 2) asm volatile(S16("v_fma_f32 %0, %0, %4, %5\n v_fma_f32 %1, %1, %4, %5\n v_fma_f32 %2, %2, %4, %5\n v_fma_f32 %3, %3, %4, %5\n") : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(m), "v"(n));
        if (K == 3) asm volatile(S16("v_pk_fma_f32 %0, %0, %1, %2\n") : "+v"(p) : "v"(mm), "v"(nn));
        if (K == 4) asm volatile(S16("v_pk_fma_f32 %0, %0, %2, %3\n v_pk_fma_f32 %1, %1, %2, %3\n") : "+v"(p), "+v"(q) : "v"(mm), "v"(nn));
        if (K == 5) asm volatile(S16("v_pk_fma_f32 %0, %0, %4, %5\n v_pk_fma_f32 %1, %1, %4, %5\n v_pk_fma_f32 %2, %2, %4, %5\n v_pk_fma_f32 %3, %3, %4, %5\n") : "+v"(p), "+v"(q), "+v"(r), "+v"(s) : "v"(mm), "v"(nn));
        if (K == 6) asm volatile(S16("v_sqrt_f32 %0, %0\n") : "+v"(a));
        if (K == 7) asm volatile(S16("v_rcp_f32 %0, %0\n") : "+v"(a));
        if (K == 8) asm volatile(S16("v_sqrt_f32 %0, %0\n v_sqrt_f32 %1, %1\n v_sqrt_f32 %2, %2\n v_sqrt_f32 %3, %3\n") : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
        if (K == 9) asm volatile(S16("v_sqrt_f32 %0, %0\n v_fma_f32 %0, %0, %1, %2\n") : "+v"(a) : "v"(m), "v"(n));
        if (K == 10) asm volatile(S16("v_fma_f32 %0, %0, %5, %6\n s_add_u32 %4, %4, 1\n v_fma_f32 %1, %1, %5, %6\n s_add_u32 %4, %4, 3\n v_fma_f32 %2, %2, %5, %6\n s_add_u32 %4, %4, 5\n v_fma_f32 %3, %3, %5, %6\n s_add_u32 %4, %4, 7\n") : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+s"(si) : "v"(m), "v"(n) : "scc");
        if (K == 11) asm volatile(S16("v_fma_f32 %0, %0, %4, %5\n s_nop 0\n v_fma_f32 %1, %1, %4, %5\n s_nop 0\n v_fma_f32 %2, %2, %4, %5\n s_nop 0\n v_fma_f32 %3, %3, %4, %5\n s_nop 0\n") : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(m), "v"(n));
        if (K == 12) asm volatile(S16("v_mov_b32 %1, %0\n v_fma_f32 %0, %1, %2, %3\n") : "+v"(a), "=&v"(b) : "v"(m), "v"(n));
        if (K == 14) asm volatile(S16("v_fma_f32 %0, %0, %8, %9\n v_fma_f32 %1, %1, %8, %9\n v_fma_f32 %2, %2, %8, %9\n v_fma_f32 %3, %3, %8, %9\n v_pk_fma_f32 %4, %4, %10, %11\n v_pk_fma_f32 %5, %5, %10, %11\n v_pk_fma_f32 %6, %6, %10, %11\n v_pk_fma_f32 %7, %7, %10, %11\n") : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(p), "+v"(q), "+v"(r), "+v"(s) : "v"(m), "v"(n), "v"(mm), "v"(nn));
        if (K == 15) asm volatile(S16("v_fma_f32 %0, %0, %4, %5\n v_fma_f32 %1, %1, %4, %5\n v_fma_f32 %2, %2, %4, %5\n v_fma_f32 %3, %3, %4, %5\n v_fma_f32 %0, %0, %4, %5\n v_fma_f32 %1, %1, %4, %5\n v_fma_f32 %2, %2, %4, %5\n v_fma_f32 %3, %3, %4, %5\n") : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(m), "v"(n));
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * 64 + threadIdx.x] = a + b + c + d + p.x + p.y + q.x + q.y + r.x + s.y + (float)si;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int K>
void run(const char* name, int instr_per_copy) {
    const int grid = 1024, iters = 100;
    float* out; unsigned long long* cyc;
    hipMalloc(&out, sizeof(float) * 64 * grid);
    hipMalloc(&cyc, sizeof(unsigned long long) * grid);
    for (int w = 0; w < 2; ++w) hipLaunchKernelGGL(k<K>, dim3(grid), dim3(64), 0, 0, out, cyc, iters);
    hipDeviceSynchronize();
    unsigned long long h[1024];
    hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
    double sum = 0;
    for (int i = 0; i < grid; ++i) sum += h[i];
    printf("%-52s %6.2f cycles per instruction (one wave per SIMD)\n", name, sum / grid / ((double)iters * 16 * instr_per_copy));
    hipFree(out); hipFree(cyc);
}

int main() {
    run<0>("v_fma_f32, 1 dependent chain", 1);
    run<1>("v_fma_f32, 2 chains interleaved", 2);
    run<2>("v_fma_f32, 4 chains interleaved", 4);
    run<15>("v_fma_f32, 4 chains, 8 per copy", 8);
    run<3>("v_pk_fma_f32, 1 chain", 1);
    run<4>("v_pk_fma_f32, 2 chains", 2);
    run<5>("v_pk_fma_f32, 4 chains", 4);
    run<14>("4 fma + 4 pk_fma chains interleaved", 8);
    run<6>("v_sqrt_f32, 1 chain", 1);
    run<7>("v_rcp_f32, 1 chain", 1);
    run<8>("v_sqrt_f32, 4 independent", 4);
    run<9>("v_sqrt_f32 -> dependent v_fma_f32 (per instr)", 2);
    run<10>("4 fma chains + 4 s_add_u32 (per instr)", 8);
    run<11>("4 fma chains + 4 s_nop 0 (per instr)", 8);
    run<12>("v_mov -> dependent v_fma (per instr)", 2);
    return 0;
}
