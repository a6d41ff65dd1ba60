// retrim.h — interface of the device batched trim (retrim.hip), shared with heligym_amd.hip.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "physics.h"
#include "trim.h"

namespace hgk {

struct RetrimArgs {
    const hg::Params<double>* P;
    const hg::TrimSetup* T;
    int32_t setup_stride;   // 0: one trim condition for all jobs; 1: T[job] (hg_trim_conds_batch)
    const int32_t* count;   // env mode: device job count; batch mode: NULL (count = njobs)
    int64_t njobs;
    const int32_t* list;    // env mode: env id of each job
    const float* wind;      // [N,3] by env id (env mode) or [count,3] by job (batch mode)
    float* state;           // env mode: SoA state (heli 18 and carry 4 rewritten)
    float* obs;             // env mode: [N,17] reset observation rows, or NULL
    int64_t n;
    float* out_state;       // batch mode outputs (rows by job), each may be NULL
    float* out_action;
    float* out_obs;
    int32_t* out_status;
    int32_t* fail_count;    // env mode: trims that failed (env keeps the template reset)
};

// Launch retrim_kernel (one 64-lane block per trim, up to `grid` blocks looping over the jobs).
hipError_t launch_retrim(const RetrimArgs& a, unsigned grid, hipStream_t stream);

}  // namespace hgk
