// step_rtc.hip — the step kernel specialised for one airframe, built at run time.
//
// The default AW109 airframe's model constants are compiled into the library's step kernel as
// instruction literals (baked.h); any other airframe runs the generic kernel, which reads ~120
// constants per RK stage with scalar loads and spills them through VGPR lanes (about 14 % slower
// per step at 65 536 envs).  This translation unit compiles the same step code (heligym_amd.hip's
// step_body, nothing else of the library) with another airframe's constant image
// (-DHG_BAKED_INC="<file>", the dword image hg_debug_params writes) into a gfx950 code object with
// the six per-step variants of one task under fixed names; heligym_amd._rtc builds and caches it
// with hipcc --genco, and hg_load_specialized loads it.  The results are bitwise those of the
// generic kernel (same operations; only the constants' source differs), which the GPU tests check.
#define HG_RTC 1
#include "heligym_amd.hip"

#ifndef HG_RTC_TASK
#define HG_RTC_TASK HG_TASK_HOVER
#endif

#define HG_RTC_KERNEL(name, NT, FEAT, NTS)                                                                \
    extern "C" __global__ __launch_bounds__(kStepBlock, NT ? HG_MIN_WAVES : HG_MIN_WAVES_BULK) void name( \
        float* __restrict__ state_p, int64_t n_p, uint64_t seed_p, int64_t envoff_p, ParamArg Pa,        \
        const Template<float>* __restrict__ Tp, const StepArgs a) {                                      \
        step_body<HG_RTC_TASK, false, NT, FEAT, false, true, NTS>(state_p, n_p, seed_p, envoff_p, Pa, Tp, a, blockIdx.x); \
    }

// the constant image and the task this code object was built with: hg_load_specialized reads them
// back (hipModuleGetGlobal) and refuses a code object whose image is not the one it is given
extern "C" __device__ __attribute__((used)) hg::ParamWords hg_rtc_image = __builtin_bit_cast(hg::ParamWords, hg::kBakedAW109);
extern "C" __device__ __attribute__((used)) int32_t hg_rtc_task = HG_RTC_TASK;

// names and order: hg_load_specialized (heligym_amd.hip) looks them up by these names
HG_RTC_KERNEL(hg_rtc_step_nt, true, false, false)
HG_RTC_KERNEL(hg_rtc_step_nt_feat, true, true, false)
HG_RTC_KERNEL(hg_rtc_step_nts, false, false, true)
HG_RTC_KERNEL(hg_rtc_step_nts_feat, false, true, true)
HG_RTC_KERNEL(hg_rtc_step_bulk, false, false, false)
HG_RTC_KERNEL(hg_rtc_step_bulk_feat, false, true, false)
