// Microbenchmark: VALU issue cost per wave on gfx950 for scalar vs packed fp32 and a few other
// instruction kinds, with 1 or 2 waves per SIMD.  Diagnostic only (not part of the library).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define REP8(x) x x x x x x x x
template <int K>
__global__ void k(float* out, unsigned long long* cyc, int iters) {
    float a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    typedef float f2 __attribute__((ext_vector_type(2)));
    f2 p0 = {a0, a1}, p1 = {a2, a3}, p2 = {a4, a5}, p3 = {a6, a7}, p4 = {a1, a0}, p5 = {a3, a2}, p6 = {a5, a4}, p7 = {a7, a6};
    const float b = 0.999f, c = 0.001f;
    f2 bb = {b, b}, cc = {c, c};
    uint32_t u0 = threadIdx.x, u1 = u0 * 3, u2 = u0 * 5, u3 = u0 * 7, u4 = u0 + 11, u5 = u0 + 13, u6 = u0 + 17, u7 = u0 + 19;
    __syncthreads();
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; ++i) {
        if (K == 0) {   // v_fma_f32, 8 independent chains
            REP8(asm volatile("v_fma_f32 %0, %0, %8, %9\n v_fma_f32 %1, %1, %8, %9\n v_fma_f32 %2, %2, %8, %9\n v_fma_f32 %3, %3, %8, %9\n v_fma_f32 %4, %4, %8, %9\n v_fma_f32 %5, %5, %8, %9\n v_fma_f32 %6, %6, %8, %9\n v_fma_f32 %7, %7, %8, %9"
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b), "v"(c));)
        } else if (K == 1) {   // v_pk_fma_f32
            REP8(asm volatile("v_pk_fma_f32 %0, %0, %8, %9\n v_pk_fma_f32 %1, %1, %8, %9\n v_pk_fma_f32 %2, %2, %8, %9\n v_pk_fma_f32 %3, %3, %8, %9\n v_pk_fma_f32 %4, %4, %8, %9\n v_pk_fma_f32 %5, %5, %8, %9\n v_pk_fma_f32 %6, %6, %8, %9\n v_pk_fma_f32 %7, %7, %8, %9"
                         : "+v"(p0), "+v"(p1), "+v"(p2), "+v"(p3), "+v"(p4), "+v"(p5), "+v"(p6), "+v"(p7) : "v"(bb), "v"(cc));)
        } else if (K == 2) {   // v_mul_f32 with an SGPR operand
            REP8(asm volatile("v_mul_f32 %0, %8, %0\n v_mul_f32 %1, %8, %1\n v_mul_f32 %2, %8, %2\n v_mul_f32 %3, %8, %3\n v_mul_f32 %4, %8, %4\n v_mul_f32 %5, %8, %5\n v_mul_f32 %6, %8, %6\n v_mul_f32 %7, %8, %7"
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "s"(b));)
        } else if (K == 3) {   // v_mul_hi_u32 (integer multiply)
            REP8(asm volatile("v_mul_hi_u32 %0, %0, %8\n v_mul_hi_u32 %1, %1, %8\n v_mul_hi_u32 %2, %2, %8\n v_mul_hi_u32 %3, %3, %8\n v_mul_hi_u32 %4, %4, %8\n v_mul_hi_u32 %5, %5, %8\n v_mul_hi_u32 %6, %6, %8\n v_mul_hi_u32 %7, %7, %8"
                         : "+v"(u0), "+v"(u1), "+v"(u2), "+v"(u3), "+v"(u4), "+v"(u5), "+v"(u6), "+v"(u7) : "s"(0xD2511F53u));)
        } else if (K == 4) {   // v_sqrt_f32 (transcendental)
            REP8(asm volatile("v_sqrt_f32 %0, %0\n v_sqrt_f32 %1, %1\n v_sqrt_f32 %2, %2\n v_sqrt_f32 %3, %3\n v_sqrt_f32 %4, %4\n v_sqrt_f32 %5, %5\n v_sqrt_f32 %6, %6\n v_sqrt_f32 %7, %7"
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));)
        } else if (K == 5) {   // v_pk_mul_f32 with scalar broadcast via op_sel_hi from an SGPR pair
            REP8(asm volatile("v_pk_mul_f32 %0, %8, %0 op_sel_hi:[0,1]\n v_pk_mul_f32 %1, %8, %1 op_sel_hi:[0,1]\n v_pk_mul_f32 %2, %8, %2 op_sel_hi:[0,1]\n v_pk_mul_f32 %3, %8, %3 op_sel_hi:[0,1]\n v_pk_mul_f32 %4, %8, %4 op_sel_hi:[0,1]\n v_pk_mul_f32 %5, %8, %5 op_sel_hi:[0,1]\n v_pk_mul_f32 %6, %8, %6 op_sel_hi:[0,1]\n v_pk_mul_f32 %7, %8, %7 op_sel_hi:[0,1]"
                         : "+v"(p0), "+v"(p1), "+v"(p2), "+v"(p3), "+v"(p4), "+v"(p5), "+v"(p6), "+v"(p7) : "s"(bb));)
        } else if (K == 6) {   // v_mad_u64_u32 (full 64-bit product)
            uint64_t r0, r1, r2, r3;
            REP8(asm volatile("v_mad_u64_u32 %0, s[0:1], %4, %8, 0\n v_mad_u64_u32 %1, s[0:1], %5, %8, 0\n v_mad_u64_u32 %2, s[0:1], %6, %8, 0\n v_mad_u64_u32 %3, s[0:1], %7, %8, 0"
                         : "=&v"(r0), "=&v"(r1), "=&v"(r2), "=&v"(r3) : "v"(u0), "v"(u1), "v"(u2), "v"(u3), "s"(0xD2511F53u) : "s0", "s1");
                 u0 = (uint32_t)r0 ^ (uint32_t)(r1 >> 32); u1 = (uint32_t)r1; u2 = (uint32_t)r2; u3 = (uint32_t)(r3 >> 32);)
        }
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    float s = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + p0.x + p1.y + p2.x + p3.y + p4.x + p5.y + p6.x + p7.y + (float)(u0 ^ u1 ^ u2 ^ u3 ^ u4 ^ u5 ^ u6 ^ u7);
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if ((threadIdx.x & 63) == 0) cyc[(blockIdx.x * blockDim.x + threadIdx.x) / 64] = t1 - t0;
}

template <int K>
void run(const char* name, int per_op, int block, int grid) {
    float* out; unsigned long long* cyc;
    hipMalloc(&out, sizeof(float) * block * grid);
    hipMalloc(&cyc, sizeof(unsigned long long) * block * grid / 64);
    const int iters = 200;
    hipLaunchKernelGGL(k<K>, dim3(grid), dim3(block), 0, 0, out, cyc, iters);
    hipLaunchKernelGGL(k<K>, dim3(grid), dim3(block), 0, 0, out, cyc, iters);
    hipDeviceSynchronize();
    int nw = block * grid / 64;
    unsigned long long* h = new unsigned long long[nw];
    hipMemcpy(h, cyc, sizeof(unsigned long long) * nw, hipMemcpyDeviceToHost);
    double sum = 0; for (int i = 0; i < nw; ++i) sum += h[i];
    double ops = (double)iters * 64;   // instructions per wave (8 x 8 per iteration)
    // s_memtime counts at the shader clock?  report raw ticks per instruction
    printf("%-28s waves/CU %2d: %.2f memtime ticks per instruction per wave\n", name, block / 64, sum / nw / ops * (per_op));
    delete[] h; hipFree(out); hipFree(cyc);
}

int main() {
    const int grid = 256;
    for (int block : {256, 512, 768}) {
        run<0>("v_fma_f32", 1, block, grid);
        run<1>("v_pk_fma_f32", 1, block, grid);
        run<2>("v_mul_f32 (sgpr)", 1, block, grid);
        run<5>("v_pk_mul_f32 (sgpr bcast)", 1, block, grid);
        run<3>("v_mul_hi_u32", 1, block, grid);
        run<4>("v_sqrt_f32", 1, block, grid);
        run<6>("v_mad_u64_u32 (+xor/mov)", 2, block, grid);
    }
    return 0;
}
