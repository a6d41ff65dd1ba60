// retrim.h — interface of the device batched trim (retrim.hip), shared with heligym_amd.hip.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/heligym_amd.h"
#include "physics.h"
#include "trim.h"

namespace hgk {

// Env state in HBM: wave tiles of 64 envs, [ceil(N/64)][kTileCols][64] 32-bit words -- columns
// 0..26 the fp32 state record (heli 18 | wind 5 | carry 4), 27..29 the int32 counters (episode
// step, success steps, episode index).  A wave's whole state is one contiguous 7.5 KB block, so
// every column of a step is an immediate offset from one base address.
#ifndef HG_TILE_ENVS
#define HG_TILE_ENVS 64
#endif
constexpr int kTileEnvs = HG_TILE_ENVS;
constexpr int kCtrCol0 = HG_STATE_COLS;
constexpr int kTileCols = HG_STATE_COLS + HG_COUNTER_COLS;
constexpr int kTileWords = kTileCols * kTileEnvs;
__host__ __device__ inline int64_t tix(int64_t env, int col) {
    return (env / kTileEnvs) * kTileWords + col * kTileEnvs + (env % kTileEnvs);
}
inline int64_t tile_words(int64_t n) { return ((n + kTileEnvs - 1) / kTileEnvs) * kTileWords; }

struct RetrimArgs {
    const hg::Params<double>* P;
    const hg::TrimSetup* T;
    int32_t setup_stride;   // 0: one trim condition for all jobs; 1: T[job] (hg_trim_conds_batch)
    const int32_t* count;   // env mode: device job count; batch mode: NULL (count = njobs)
    int64_t njobs;
    const int32_t* list;    // env mode: env id of each job
    const float* wind;      // [N,3] by env id (env mode) or [count,3] by job (batch mode)
    float* state;           // env mode: tiled state (tix; heli 18 and carry 4 rewritten)
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
