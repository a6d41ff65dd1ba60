// retrim.h — interface of the device batched trim (retrim.hip), shared with heligym_amd.hip.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/heligym_amd.h"
#include "physics.h"
#include "trim.h"

namespace hgk {

// Env state in HBM: wave tiles of 64 envs, [ceil(N/64)][7][64][4] 32-bit words.  An env has 28
// slots in seven groups of four; group g of a tile is 64 lanes x 16 bytes, so the step kernel moves a
// group with one 16-byte access per lane, 1 KB contiguous per wave (7 loads and 7 stores per env
// instead of 28 of 4 bytes).  The 30 logical columns -- the fp32 state record 0..26 (heli 18 | wind 5
// | carry 4) and the int32 counters 27..29 (episode step, success steps, episode index) -- sit in the
// groups in the order the step needs them: position and step counter, the noise key and carry, the
// wind state, then the heli state.  Columns 2 and 3, the rotor azimuths, have no slot: no force,
// observation, reward or flag reads them (helicopter_dynamics.py:203-300 take psi_mr / psi_tr and
// never use them) and each advances by the constant dt * Omega per step (:257-258, :288-289), so
// they live in an azimuth record per env (AzRec, below) and are reconstructed when the state is read.
// The step counter of an env waiting for its next-step auto-reset is -(n + 1), n = the steps its
// episode took (exported as -1).
constexpr int kTileEnvs = 64;
static_assert(HG_STATE_COLS + HG_COUNTER_COLS == 30, "the slot table covers 30 columns");
constexpr int kCtrCol0 = HG_STATE_COLS;
constexpr int kTileCols = HG_STATE_COLS + HG_COUNTER_COLS;   // logical columns
constexpr int kEnvSlots = 28;
constexpr int kTileWords = kEnvSlots * kTileEnvs;
constexpr int kAzCol0 = 2;   // psi_mr, psi_tr: the columns without a slot
// slot of logical column c (-1: an azimuth):  x y z step | epi succ carry3 carry0 |
// carry1 carry2 ws0 ws1 | ws2 ws3 ws4 psi | vi_mr vi_tr b0 b1 | u v w p | q r phi theta
__host__ __device__ constexpr int slot_of(int c) {
    constexpr int t[30] = {16, 17, -1, -1, 18, 19, 20, 21, 22, 23, 24, 25, 26, 27, 15, 0, 1, 2,
                           10, 11, 12, 13, 14, 7, 8, 9, 6, 3, 5, 4};
    return t[c];
}
__host__ __device__ inline int64_t tix(int64_t env, int col) {   // (col not an azimuth)
    const int s = slot_of(col);
    return (env / kTileEnvs) * kTileWords + (s >> 2) * (4 * kTileEnvs) + (env % kTileEnvs) * 4 + (s & 3);
}
__host__ __device__ inline bool has_slot(int col) { return slot_of(col) >= 0; }

// Azimuth record of an env: the rotor azimuths (mr, tr) at step `step0` of episode `epi0`.  Written
// only off the step path (create, reset, set_state, a re-trim, before a template change); an episode
// begun by an in-kernel auto-reset (episode index != epi0) starts from its reset template's azimuths.
struct AzRec {
    float mr, tr;
    int32_t step0, epi0;
};
// steps an env's episode has taken, from its step counter (negative: waiting for its next-step reset)
__host__ __device__ inline int32_t episode_steps(int32_t step) { return step >= 0 ? step : -(step + 1); }
inline int64_t tile_words(int64_t n) { return ((n + kTileEnvs - 1) / kTileEnvs) * kTileWords; }

// a fused same-step launch's counters (one slot of a ring of three): ints [0, 1] the 64-bit {queued jobs,
// waves with jobs}, [2] the trim waves' claim counter, then kFusedWaveCtrs counters of the waves without
// jobs, each at the start of a 64-byte line of its own (kFusedLine ints)
constexpr int kFusedLine = 16;
constexpr int kFusedWaveCtrs = 16;
constexpr int kFusedSlot = kFusedLine * (kFusedWaveCtrs + 1);

struct RetrimArgs {
    const hg::Params<double>* P;
    const hg::TrimSetup* T;
    int32_t setup_stride;   // 0: one trim condition for all jobs; 1: T[job] (hg_trim_conds_batch)
    const int32_t* count;   // env mode: device job count; batch mode: NULL (count = njobs)
    int64_t njobs;
    const int32_t* list;    // env mode: env id of each job (winds by env) ...
    const int4* recs;       // ... or jobs {env, wind bits} (a step's auto-resets)
    const float* wind;      // [N,3] by env id (env mode) or [count,3] by job (batch mode) ...
    int32_t wind_soa;       // ... or [3][N] by env id (env mode: the step's per-env wind records)
    float* state;           // env mode: tiled state (tix; heli 18 and carry 4 rewritten)
    AzRec* az;              // env mode: azimuth records (the trim's azimuths at step 0)
    float* obs;             // env mode: [N,17] reset observation rows, or NULL
    int64_t n;
    float* out_state;       // batch mode outputs (rows by job), each may be NULL
    float* out_action;
    float* out_obs;
    int32_t* out_status;
    int32_t* fail_count;    // env mode: trims that failed (env keeps the template reset)
    // ov mode (env mode, jobs from recs): the next-step resets of envs whose step runs concurrently.
    // That step stores only their step counter, so the trim writes the whole reset -- the wind
    // states and success counter zeroed, the episode index advanced -- and on failure the template.
    int32_t ov;
    const float* tmpl;      // ov: the shared reset template (heli 18 | carry 4 | obs 17) ...
    const float* tmpl_env;  // ... or the per-env ones [N][39] (Params::env_templates), else NULL
    int32_t* bad_jobs;      // env mode: job records naming no env (or a count past N), skipped and counted
    int32_t* solve_stats;   // [0] Newton solves tried with the setup's pivot order, [1] of them rejected
                            // by the residual test (and searched instead); may be NULL
    // fused same-step mode (step_fused_kernel): the trims run in the step's own launch and take each
    // job as soon as the step wave that queued it has published its record (device-coherent stores,
    // env last); claim hands out job indices; ctr is the launch's slot (kFusedSlot ints): the queue is
    // complete once every step wave has counted itself
    int32_t* claim;         // NULL: not fused
    const unsigned long long* ctr;
    int32_t nwaves;         // step waves of the launch
};

// Launch retrim_kernel (one 64-lane block per trim, up to `grid` blocks looping over the jobs).
hipError_t launch_retrim(const RetrimArgs& a, unsigned grid, hipStream_t stream);

}  // namespace hgk
