#include <hip/hip_runtime.h>
#include <stdio.h>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)
__global__ void empty_kernel(float* p) { if (p == nullptr) p[threadIdx.x] = 0.f; }
__global__ void touch_kernel(float* p) { p[blockIdx.x * blockDim.x + threadIdx.x] += 1.f; }
int main() {
    hipStream_t st; CK(hipStreamCreate(&st));
    float* buf; CK(hipMalloc(&buf, 64 << 20)); CK(hipMemset(buf, 0, 64 << 20));
    struct Cfg { const char* name; int kind; unsigned grid, block; } cfgs[] = {
        {"empty 1x64", 0, 1, 64}, {"empty 256x256", 0, 256, 256}, {"empty 1024x64", 0, 1024, 64},
        {"empty 4096x64", 0, 4096, 64}, {"touch 1024x64 (256 KB rmw)", 1, 1024, 64}};
    for (auto& c : cfgs) {
        hipGraph_t g; hipGraphExec_t ge;
        CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
        for (int k = 0; k < 100; ++k) {
            if (c.kind == 0) hipLaunchKernelGGL(empty_kernel, dim3(c.grid), dim3(c.block), 0, st, buf);
            else hipLaunchKernelGGL(touch_kernel, dim3(c.grid), dim3(c.block), 0, st, buf);
        }
        CK(hipStreamEndCapture(st, &g)); CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        for (int w = 0; w < 3; ++w) CK(hipGraphLaunch(ge, st));
        hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
        CK(hipEventRecord(e0, st));
        for (int r = 0; r < 20; ++r) CK(hipGraphLaunch(ge, st));
        CK(hipEventRecord(e1, st)); CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1));
        printf("%-28s %6.2f us/launch\n", c.name, ms * 1e3 / 2000.0);
        CK(hipGraphExecDestroy(ge)); CK(hipGraphDestroy(g));
    }
    return 0;
}
