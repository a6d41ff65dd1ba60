// retrim.hip — the device batched Newton trim: exact second-episode resets (reset_mode RETRIM,
// SURVEY F8), hg_trim_batch and hg_trim_conds_batch.
//
// HelicopterDynamics.trim (helicopter_dynamics.py:491-555) for many winds at once, one wave per trim,
// fp64 throughout: the reference's Newton iteration (central-difference Jacobian, step halving,
// stop at ||y - y*||^2 <= 1e-4) with its 42 model evaluations per round spread over the lanes and
// the 16 x 16 solve one row per lane (retrim_body.h).  The device evaluates the model with fused
// multiply-adds (-ffp-contract=on: per source expression, so every kernel that includes the body
// rounds the same way), one-reduction sin/cos and reciprocal divisions by model constants (physics.h
// device overloads), a few-ulp rounding of the same fp64 arithmetic.  The host's serial trim
// (heligym_amd.hip::do_trim) is not reproduced bitwise (its libm transcendentals differ from any
// device library anyway); the tests hold the device trims to it and to the reference's recorded
// resets at fp32 resolution.
#include "../../include/heligym_amd.h"
// The iterate stays in registers here (retrim_body.h HG_RT_XLDS, bitwise either way): in LDS it
// helps the overlapped launch, whose step waves share the SIMDs, and costs this kernel 0.3 us per
// re-trim step.
#ifndef HG_RT_XLDS
#define HG_RT_XLDS 0
#endif
// The Jacobian column re-materialised each Newton round (retrim_body.h HG_RT_OPAQUE_COL): here it
// shortens the trim (same-step re-trim 28.96 -> 28.83 us), in the overlapped launch it costs 0.6 us
// (scripts/gpu_r06_ab.sh), so only this translation unit sets it.
#ifndef HG_RT_OPAQUE_COL
#define HG_RT_OPAQUE_COL 1
#endif
// The first job's setup written to LDS at entry (retrim_body.h HG_RT_SETUP_LDS): same-step re-trim
// 29.56 -> 28.85 us; the overlapped launch is 0.2 us slower with it and leaves it off.
#ifndef HG_RT_SETUP_LDS
#define HG_RT_SETUP_LDS 1
#endif
#include "retrim_body.h"

namespace hgk {
namespace {

// (one wave per SIMD, the whole register budget of a single wave, measured in round 6: 28.07 against
// 28.32 us per same-step re-trim step on one box, 28.28 against 28.27 on another; not adopted)
#ifndef HG_RETRIM_WAVES
#define HG_RETRIM_WAVES 2
#endif
// count_p / recs_p / T_p / P_p / Tstride_p = a.count / a.recs / a.T / a.P / a.setup_stride: leading
// arguments, preloaded into SGPRs (__graft_entry__.py builds this translation unit with
// -amdgpu-kernarg-preload-count=5)
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(HG_RETRIM_WAVES))) void retrim_kernel(
    const int32_t* count_p, const int4* recs_p, const hg::TrimSetup* T_p, const hg::Params<double>* P_p,
    int32_t Tstride_p, const RetrimArgs a) {
    retrim_jobs(a, blockIdx.x, gridDim.x, count_p, recs_p, T_p, P_p, Tstride_p);
}



}  // namespace

#if HG_TIMING
extern "C" int hg_debug_retrim_timing(void* dst, int64_t bytes) {
    return hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_rt_timing), (size_t)bytes) == hipSuccess ? 0 : -1;
}
#endif

#if HG_RT_DEBUG
extern "C" int hg_debug_rt_log_serial(void* dst, int64_t bytes, int32_t clear) {
    if (dst && hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_rt_dbg), (size_t)bytes) != hipSuccess) return -1;
    unsigned n = 0;
    if (hipMemcpyFromSymbol(&n, HIP_SYMBOL(g_rt_dbg_n), sizeof(n)) != hipSuccess) return -1;
    if (clear) {
        const unsigned z = 0;
        (void)hipMemcpyToSymbol(HIP_SYMBOL(g_rt_dbg_n), &z, sizeof(z));
    }
    return (int)n;
}
#endif

hipError_t launch_retrim(const RetrimArgs& a, unsigned grid, hipStream_t stream) {
    hipLaunchKernelGGL(retrim_kernel, dim3(grid), dim3(64), 0, stream, a.count, a.recs, a.T, a.P, a.setup_stride, a);
    return hipGetLastError();
}

}  // namespace hgk
