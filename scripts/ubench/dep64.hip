// Microbenchmark (diagnostic, not part of the library): fp64 and cross-lane costs for one wave alone
// on its SIMD on gfx950 -- the instruction mix of the device trim's model evaluation and its
// Gauss-Jordan solve (v_fma_f64 chains, v_readlane into an SGPR feeding a v_fma_f64, DPP maxes).
// Each asm block is 16 copies of a short sequence.  Grid: one 64-lane block per SIMD.
#include <hip/hip_runtime.h>
#include <stdio.h>

#define S4(x) x x x x
#define S16(x) S4(x) S4(x) S4(x) S4(x)

template <int K>
__global__ void __launch_bounds__(64) k(double* out, unsigned long long* cyc, int iters) {
    double a = threadIdx.x * 1e-3 + 1.0, b = a + 1, c = a + 2, d = a + 3;
    const double m = 0.999, n = 0.001;
    unsigned u = threadIdx.x, v = threadIdx.x * 3u, w = threadIdx.x + 5u, x = threadIdx.x ^ 9u, y = 7u;
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; ++i) {
        if (K == 0) asm volatile(S16("v_fma_f64 %0, %0, %1, %2\n") : "+v"(a) : "v"(m), "v"(n));
        if (K == 1) asm volatile(S16("v_fma_f64 %0, %0, %4, %5\n v_fma_f64 %1, %1, %4, %5\n v_fma_f64 %2, %2, %4, %5\n v_fma_f64 %3, %3, %4, %5\n") : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(m), "v"(n));
        if (K == 2) asm volatile(S16("v_mul_f64 %0, %0, %4\n v_mul_f64 %1, %1, %4\n v_mul_f64 %2, %2, %4\n v_mul_f64 %3, %3, %4\n") : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(m));
        if (K == 3) {   // readlane pair -> fma using the SGPR pair (the GJ element update), 4 independent
            asm volatile(S16("v_readlane_b32 s20, %1, 5\n v_readlane_b32 s21, %2, 5\n v_fma_f64 %0, s[20:21], %3, %0\n") : "+v"(a) : "v"(u), "v"(v), "v"(m) : "s20", "s21");
        }
        if (K == 4) asm volatile(S16("v_readlane_b32 s20, %0, 5\n v_readlane_b32 s21, %1, 7\n v_readlane_b32 s22, %0, 9\n v_readlane_b32 s23, %1, 11\n") : : "v"(u), "v"(v) : "s20", "s21", "s22", "s23");
        if (K == 5) asm volatile(S16("v_max_u32_dpp %0, %0, %0 row_ror:8 row_mask:0xf bank_mask:0xf bound_ctrl:1\n s_nop 1\n") : "+v"(u));
        if (K == 6) asm volatile(S16("v_fma_f64 %0, %0, %4, %5\n v_fma_f64 %1, %1, %4, %5\n v_fma_f64 %2, %2, %4, %5\n v_fma_f64 %3, %3, %4, %5\n v_fma_f64 %0, %0, %4, %5\n v_fma_f64 %1, %1, %4, %5\n v_fma_f64 %2, %2, %4, %5\n v_fma_f64 %3, %3, %4, %5\n") : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(m), "v"(n));
        if (K == 7) asm volatile(S16("v_add_f64 %0, %0, %4\n v_add_f64 %1, %1, %4\n v_add_f64 %2, %2, %4\n v_add_f64 %3, %3, %4\n") : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(m));
        if (K == 8) asm volatile(S16("v_cndmask_b32 %0, %0, %1, vcc\n v_cndmask_b32 %1, %1, %0, vcc\n") : "+v"(u), "+v"(v));
        if (K == 9) asm volatile(S16("v_cndmask_b32 %0, %0, %4, vcc\n v_cndmask_b32 %1, %1, %4, vcc\n v_cndmask_b32 %2, %2, %4, vcc\n v_cndmask_b32 %3, %3, %4, vcc\n") : "+v"(u), "+v"(v), "+v"(w), "+v"(x) : "v"(y));
        if (K == 10) asm volatile(S16("v_cndmask_b32_e64 %0, %0, %4, s[20:21]\n v_cndmask_b32_e64 %1, %1, %4, s[20:21]\n v_cndmask_b32_e64 %2, %2, %4, s[20:21]\n v_cndmask_b32_e64 %3, %3, %4, s[20:21]\n") : "+v"(u), "+v"(v), "+v"(w), "+v"(x) : "v"(y) : "s20", "s21");
        if (K == 11) asm volatile(S16("v_add_u32 %0, %0, %4\n v_add_u32 %1, %1, %4\n v_add_u32 %2, %2, %4\n v_add_u32 %3, %3, %4\n") : "+v"(u), "+v"(v), "+v"(w), "+v"(x) : "v"(y));
        if (K == 12) asm volatile(S16("v_add_u32 %0, %0, %1\n") : "+v"(u) : "v"(y));
        if (K == 13) asm volatile(S16("v_cmp_gt_u32 vcc, %1, %0\n v_cndmask_b32 %0, %0, %1, vcc\n") : "+v"(u) : "v"(y));
        if (K == 14) asm volatile(S16("v_cmp_gt_f64 vcc, %0, %1\n s_nop 0\n") : : "v"(a), "v"(m));
        if (K == 15) {   // f64 MFMA 16x16x4, one dependent accumulator chain
            typedef double d4 __attribute__((ext_vector_type(4)));
            d4 acc = {a, b, c, d};
            for (int r = 0; r < 16; ++r) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(m, n, acc, 0, 0, 0);
            a = acc[0]; b = acc[1]; c = acc[2]; d = acc[3];
        }
        if (K == 16) {   // f64 MFMA 16x16x4, 4 independent accumulators
            typedef double d4 __attribute__((ext_vector_type(4)));
            d4 x0 = {a, b, c, d}, x1 = x0 + 1.0, x2 = x0 + 2.0, x3 = x0 + 3.0;
            for (int r = 0; r < 4; ++r) {
                x0 = __builtin_amdgcn_mfma_f64_16x16x4f64(m, n, x0, 0, 0, 0);
                x1 = __builtin_amdgcn_mfma_f64_16x16x4f64(m, n, x1, 0, 0, 0);
                x2 = __builtin_amdgcn_mfma_f64_16x16x4f64(m, n, x2, 0, 0, 0);
                x3 = __builtin_amdgcn_mfma_f64_16x16x4f64(m, n, x3, 0, 0, 0);
            }
            a = x0[0] + x1[1]; b = x2[2] + x3[3];
        }
        if (K == 17)   // v_fma_f64 -> 2 v_readlane -> next v_fma_f64 reads the SGPR pair (a loop-carried chain)
            asm volatile(S16("v_fma_f64 v[40:41], s[20:21], %0, %1\n v_readlane_b32 s20, v40, 5\n v_readlane_b32 s21, v41, 5\n")
                         : : "v"(m), "v"(n) : "s20", "s21", "v40", "v41");
        if (K == 18)   // v_cmp -> s_ff1 -> v_readlane with that lane -> v_mov (the pivot search's tail), chained
            asm volatile(S16("v_cmp_eq_u32 s[22:23], %0, %1\n s_ff1_i32_b64 s24, s[22:23]\n v_readlane_b32 s25, %0, s24\n v_add_u32 %0, s25, %0\n")
                         : "+v"(u) : "v"(y) : "s22", "s23", "s24", "s25");
        if (K == 19) asm volatile(S16("v_mul_f64 %0, %0, %1\n") : "+v"(a) : "v"(m));
        if (K == 20) {   // permlane16 swap chain
            for (int r = 0; r < 16; ++r) { auto t = __builtin_amdgcn_permlane16_swap(u, v, false, false); u = t[0] + 1; v = t[1]; }
        }
        if (K == 22) asm volatile(S16("s_nop 1\n v_mov_b64_dpp %0, %0 row_newbcast:3 row_mask:0xf bank_mask:0xf\n") : "+v"(a));
        if (K == 23) asm volatile(S16("v_rcp_f64 %0, %0\n") : "+v"(a));
        if (K == 24) asm volatile(S16("s_nop 1\n v_fmac_f64_dpp %0, %0, %1 row_newbcast:3 row_mask:0xf bank_mask:0xf\n") : "+v"(a) : "v"(m));
        if (K == 25) asm volatile(S16("s_nop 1\n v_fma_f64 %0, %0, %1, %2\n") : "+v"(a) : "v"(m), "v"(n));
        if (K == 26) asm volatile(S16("v_fmac_f64 %0, %0, %1\n") : "+v"(a) : "v"(m));
        if (K == 21) asm volatile(S16("ds_bpermute_b32 %0, %1, %0\n s_waitcnt lgkmcnt(0)\n") : "+v"(u) : "v"(w));
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * 64 + threadIdx.x] = a + b + c + d + u + v + w + x;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int K>
void run(const char* name, int instr_per_copy) {
    const int grid = 1024, iters = 100;
    double* out; unsigned long long* cyc;
    hipMalloc(&out, sizeof(double) * 64 * grid);
    hipMalloc(&cyc, sizeof(unsigned long long) * grid);
    for (int w = 0; w < 2; ++w) hipLaunchKernelGGL(k<K>, dim3(grid), dim3(64), 0, 0, out, cyc, iters);
    hipDeviceSynchronize();
    unsigned long long h[1024];
    hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
    double sum = 0;
    for (int i = 0; i < grid; ++i) sum += h[i];
    printf("%-56s %6.2f memtime ticks per instruction\n", name, sum / grid / ((double)iters * 16 * instr_per_copy));
    hipFree(out); hipFree(cyc);
}

int main() {
    run<0>("v_fma_f64, 1 dependent chain", 1);
    run<1>("v_fma_f64, 4 chains interleaved", 4);
    run<6>("v_fma_f64, 4 chains, 8 per copy", 8);
    run<2>("v_mul_f64, 4 chains", 4);
    run<7>("v_add_f64, 4 chains", 4);
    run<3>("2 v_readlane_b32 -> v_fma_f64 (per instr)", 3);
    run<4>("v_readlane_b32, independent", 4);
    run<5>("v_max_u32_dpp chain + s_nop 1 (per pair)", 1);
    run<8>("v_cndmask_b32, 2 chains (vcc)", 2);
    run<9>("v_cndmask_b32, 4 independent (vcc)", 4);
    run<10>("v_cndmask_b32_e64, 4 independent (SGPR pair)", 4);
    run<11>("v_add_u32, 4 independent", 4);
    run<12>("v_add_u32, 1 dependent chain", 1);
    run<13>("v_cmp -> v_cndmask on vcc (per instr)", 2);
    run<14>("v_cmp_gt_f64 + s_nop 0 (per pair)", 1);
    run<15>("v_mfma_f64_16x16x4, 1 dependent chain", 1);
    run<16>("v_mfma_f64_16x16x4, 4 chains", 1);
    run<17>("fma_f64 -> 2 readlane -> fma (per group)", 1);
    run<18>("cmp -> s_ff1 -> readlane(lane s) -> add (per group)", 1);
    run<19>("v_mul_f64, 1 dependent chain", 1);
    run<20>("permlane16_swap chain (+add) (per swap)", 1);
    run<21>("ds_bpermute + wait (per round trip)", 1);
    run<22>("s_nop 1 + v_mov_b64_dpp row_newbcast, dependent (per pair)", 1);
    run<23>("v_rcp_f64, dependent chain", 1);
    run<24>("s_nop 1 + v_fmac_f64_dpp row_newbcast, dependent (per pair)", 1);
    run<25>("s_nop 1 + v_fma_f64, dependent (per pair)", 1);
    run<26>("v_fmac_f64 (e32), dependent chain", 1);
    return 0;
}
