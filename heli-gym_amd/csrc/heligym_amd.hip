// heligym_amd.hip — gfx950 (MI355X) kernels and the C-ABI of include/heligym_amd.h.
//
// One launch of `step_kernel` advances N independent helicopters by one env step
// (Heli.step, heligym/envs/helicopter.py:192-206): Dryden wind RK (k4-only), RK4 of the 18-state
// helicopter model, task reward, termination flags and same-step auto-reset.  One thread = one
// env.  Data layout in HBM (all written/read coalesced):
//   state    wave tiles [ceil(N/64)][7][64][4] 32-bit words (retrim.h tix): fp32 heli 16 | wind 5 |
//            carry 4, the i32 counters (episode step, success steps, episode index); the two rotor
//            azimuths in a per-env record written off the step path (retrim.h AzRec)
//   actions  [N,4] fp32 (one float4 per lane)      obs [N,17] fp32 (LDS-staged, float4 stores)
//   reward [N] fp32, terminated/truncated/info [N] u8
// Model constants are read with scalar loads from a device copy; the terrain map (8 MiB float2
// {hi, lo}) stays cache-resident.
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <string>
#include <type_traits>
#include <vector>

#include "../../include/heligym_amd.h"
#include "physics.h"
#include "trim.h"
#include "retrim.h"
#include "retrim_body.h"
#include "baked.h"

using hg::Params;
using hg::Template;
using hgk::kCtrCol0;
using hgk::kTileEnvs;
using hgk::kTileWords;
using hgk::tix;
using hgk::AzRec;

namespace {

thread_local std::string g_last_error;

void dfree(void* p) {
    if (p) (void)hipFree(p);
}

int32_t fail(int32_t code, const std::string& msg) {
    g_last_error = msg;
    return code;
}

#define HIP_TRY(expr)                                                                         \
    do {                                                                                      \
        hipError_t e_ = (expr);                                                               \
        if (e_ != hipSuccess)                                                                 \
            return fail(HG_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e_));         \
    } while (0)

constexpr int kBlock = 256;
#ifndef HG_STEP_BLOCK
#define HG_STEP_BLOCK 64
#endif
using hgk::kFusedLine;
using hgk::kFusedSlot;
using hgk::kFusedWaveCtrs;
constexpr int kStepBlock = HG_STEP_BLOCK;   // step kernel block: one or more waves, one state tile each
static_assert(kTileEnvs == 64, "a state tile is one wave");
constexpr int kStateCols = HG_STATE_COLS;
constexpr int kCtrCols = HG_COUNTER_COLS;


// ------------------------------------------------------------------------------ Philox4x32-10
struct U4 {
    uint32_t x, y, z, w;
};

#ifndef HG_PHILOX_ROUNDS   // (A/B builds only: the library's noise stream is Philox4x32-10)
#define HG_PHILOX_ROUNDS 10
#endif
__device__ __forceinline__ U4 philox(U4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int i = 0; i < HG_PHILOX_ROUNDS; ++i) {
        const uint32_t lo0 = 0xD2511F53u * c.x, hi0 = __umulhi(0xD2511F53u, c.x);
        const uint32_t lo1 = 0xCD9E8D57u * c.z, hi1 = __umulhi(0xCD9E8D57u, c.z);
#ifndef HG_NO_BITOP3
        // hi ^ y ^ k as one three-input bitwise instruction (truth table 0x96 = XOR3)
        c = U4{(uint32_t)__builtin_amdgcn_bitop3_b32(hi1, c.y, k0, 0x96), lo1,
               (uint32_t)__builtin_amdgcn_bitop3_b32(hi0, c.w, k1, 0x96), lo0};
#else
        c = U4{hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
#endif
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    return c;
}

// ((x >> 8) + 0.5) 2^-24 in fp32: from 2^23 on the + 0.5 rounds to even, so u is in (0, 1] (1 at the top:
// a zero Box-Muller radius, never a log of 0); tests/philox_ref.py restates it bitwise
__device__ __forceinline__ float u01(uint32_t x) {
    return ((float)(x >> 8) + 0.5f) * (1.0f / 16777216.0f);
}

// ------------------------------------------------------------------------------ kernels

// Kernel arguments.  What the state loads wait for -- the state base, n (a lane is active), the noise
// key -- are the step kernel's first scalar parameters, preloaded into SGPRs at wave launch
// (-amdgpu-kernarg-preload-count), so no scalar-load round trip sits in front of the state loads;
// StepArgs follows, its feature-only fields last.  192 bytes in all, three scalar-cache lines (200
// bytes, a fourth line on the critical path, cost 0.23 us per step).
constexpr int kStepPreloadArgs = 6;   // state, n, seed, env_offset, Pa, Tp
struct StepArgs {
    const float2* hmap;
    const float* actions;
    float* obs;
    float* reward;
    uint8_t* terminated;
    uint8_t* truncated;
    uint8_t* info;
    const float* eta;
    float* final_obs_rows;       // [N,17] terminal observations of this step's auto-resets at their rows (hg_step_rows), or NULL
    int32_t nsteps;          // MULTI: steps per launch (inputs / outputs stacked [nsteps][N])
    int32_t retrim_slot;     // -1, or the slot of retrim_count's ring of three this step counts into (it
                             // zeroes the next one)
    // FEAT only
    int32_t* reset_count;
    int32_t* reset_count_next;   // zeroed by this launch for a later step (hg_step_chained), or NULL
    int32_t* reset_index;
    float* final_obs;
    float* retrim_wind;      // reset_mode RETRIM: [3][N] wind of the step (the trim wind of a reset)
    int4* retrim_recs;       // ... compacted jobs {env, trim wind} of the envs to re-trim
    int32_t* retrim_count;   // ... their number: retrim_count[max(retrim_slot, 0)]
    const float* tmpl_env;   // per-env reset templates [N][39] (Params::env_templates), else unused
    // next-step auto-resets re-trimmed concurrently with the following step (reset_mode RETRIM):
    int4* ov_recs;           // jobs {env, trim wind} of the envs whose episode ends this step, or NULL
    int32_t* ov_count;       // ... their number (zeroed by the previous step of the sequence)
    int32_t* ov_count_next;  // ... the next step's count, zeroed by this launch
    int32_t ov_active;       // the resets due this step are being trimmed by a concurrent retrim_kernel
                             // (ov mode): their state, but for the step counter, and their observation
                             // rows are that kernel's to write
    // fused same-step re-trim (step_fused_kernel): records published by device-coherent stores (env
    // last), the resets deferred as in ov mode (the trim writes all but the step counter)
    unsigned long long* fused_ctr;   // this launch's fused slot (kFusedSlot ints), or NULL (not fused)
    int32_t* fused_next;     // the next launch's slot, zeroed by this launch
};

// Model constants travel as a pointer to a device copy (scalar loads); by value they would take
// ~0.6 KB of kernel arguments and spill more SGPRs.
using ParamArg = const Params<float>* __restrict__;

#ifndef HG_NTS_WAVES   // bulk per-step launches store non-temporally up to this many waves per SIMD
#define HG_NTS_WAVES 4
#endif
#ifndef HG_NT_WAVES   // the lone-wave (NT) variant up to this many waves per SIMD
#define HG_NT_WAVES 2
#endif
#ifndef HG_MIN_WAVES
#define HG_MIN_WAVES 1
#endif
#ifndef HG_EARLY_POST   // post-step terrain texels requested right after the RK update (0: after the reward)
#define HG_EARLY_POST 1
#endif
#ifndef HG_MIN_WAVES_BULK   // launches with more waves than SIMDs (not NT): waves per SIMD the
#define HG_MIN_WAVES_BULK 3   // registers must fit (3: <= 168 VGPRs; uncapped the bulk variant took
#endif                        // 173 and ran two: 262 144 envs 21.1 -> 19.3 us, 1 M and 4 M unchanged)

constexpr int kTplFloats = (int)(sizeof(Template<float>) / sizeof(float));
static_assert(kTplFloats <= 64, "reset template must fit one float per lane");
// the template's device copy holds one float per lane of a wave (HG_TPL_FULL: every lane loads one)
constexpr size_t kTplAlloc = 64 * sizeof(float);
#ifndef HG_RT_QUEUE_LATE   // the re-trim queue's records written after the state stores (lone-wave kernels)
#define HG_RT_QUEUE_LATE 1
#endif
#ifndef HG_TPL_FULL_HELP
#define HG_TPL_FULL_HELP 1
#endif
__device__ __forceinline__ float lane_value(float v, int lane) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), lane));
}

// Output stores.  NT = non-temporal for the dword-and-wider columns (the byte flags stay plain):
// used when the whole batch is resident at once (<= one wave per SIMD), where the step is latency
// bound and streaming the outputs shortens the end-of-kernel write-back; with more waves than
// SIMDs the plain write-back path is faster.
typedef float f32x4 __attribute__((ext_vector_type(4)));
template <bool NT, typename T>
__device__ __forceinline__ void st_out(T* p, T v) {
    if constexpr (NT && sizeof(T) >= 4) __builtin_nontemporal_store(v, p);
    else *p = v;
}
template <bool NT>
__device__ __forceinline__ void st_out4(float* p, const float* s) {
    const f32x4 v = *reinterpret_cast<const f32x4*>(s);
    if constexpr (NT) __builtin_nontemporal_store(v, reinterpret_cast<f32x4*>(p));
    else *reinterpret_cast<f32x4*>(p) = v;
}

typedef __attribute__((address_space(4))) const Params<float> ConstParams;
__device__ __forceinline__ const Params<float>* reload_params(const Params<float>* p) {
    ConstParams* c = (ConstParams*)p;
    asm volatile("" : "+s"(c));   // opaque: the loads cannot be hoisted out of the step loop
    return (const Params<float>*)c;
}

// Per-lane access at a small byte offset from a uniform base (SGPR-base global load / store).  The
// explicit global address space keeps the saddr form (`global_store_dword voff, v, s[base]`) even
// for bases that went through an opaque copy, which would otherwise be flat stores with a 64-bit
// VALU address add each.
#define HG_GLOBAL __attribute__((address_space(1)))
template <typename T>
__device__ __forceinline__ T ld_lane(const T* __restrict__ base, uint32_t idx) {
    const HG_GLOBAL char* g = (const HG_GLOBAL char*)base + idx * (uint32_t)sizeof(T);
    if constexpr (sizeof(T) == 16) {   // float4: load as a plain vector (no address-space copy ctor)
        typedef float v4 __attribute__((ext_vector_type(4)));
        return __builtin_bit_cast(T, *(const HG_GLOBAL v4*)g);
    } else {
        return *(const HG_GLOBAL T*)g;
    }
}
template <bool NT, typename T>
__device__ __forceinline__ void st_lane(T* base, uint32_t idx, T v) {
    HG_GLOBAL T* p = (HG_GLOBAL T*)((HG_GLOBAL char*)base + idx * (uint32_t)sizeof(T));
    if constexpr (NT && sizeof(T) >= 4) __builtin_nontemporal_store(v, p);
    else *p = v;
}

// Observations of a step: each wave stages its 64 rows in its own LDS slice (stride 17 is
// bank-conflict free) and writes them back as contiguous float4, with no block-wide barrier.
// MULTI (hg_rollout): step s's rows start at obs + s*N*17 floats, 16-byte aligned only when
// N % 4 == 0 (or s % 4 == 0); unaligned rows go out as dwords.
// `skip` (uniform): rows another kernel writes (the concurrently re-trimmed resets), stored around.
template <bool NT, bool MULTI>
__device__ __forceinline__ void store_obs_wave(float* w_obs, const float obs[17], float* dst, int64_t so, int64_t w0,
                                               int64_t n, int lane, uint64_t skip = 0) {
#pragma unroll
    for (int c = 0; c < 17; ++c) w_obs[lane * 17 + c] = obs[c];
    __builtin_amdgcn_wave_barrier();
    const int nw = (n - w0) < 64 ? (int)(n - w0) : 64;
    const int cnt = nw > 0 ? nw * 17 : 0;
    float* out = dst + (so + w0) * 17;
    if (skip) {
        for (int j = lane; j < cnt; j += 64)
            if (!((skip >> (j / 17)) & 1)) st_out<NT>(out + j, w_obs[j]);
        return;
    }
    const bool aligned = !MULTI || (((uintptr_t)out & 15) == 0);
    if (nw == 64 && aligned) {   // full wave: 272 float4, all LDS reads issued before the first store
        f32x4 v[5];
#pragma unroll
        for (int t = 0; t < 4; ++t) v[t] = *reinterpret_cast<const f32x4*>(w_obs + 4 * (lane + 64 * t));
        if (lane < 16) v[4] = *reinterpret_cast<const f32x4*>(w_obs + 4 * (lane + 256));
#pragma unroll
        for (int t = 0; t < 4; ++t) st_out4<NT>(out + 4 * (lane + 64 * t), reinterpret_cast<const float*>(&v[t]));
        if (lane < 16) st_out4<NT>(out + 4 * (lane + 256), reinterpret_cast<const float*>(&v[4]));
        return;
    }
    const int n4 = aligned ? cnt >> 2 : 0;
    for (int j = lane; j < n4; j += 64) st_out4<NT>(out + 4 * j, w_obs + 4 * j);
    for (int j = (n4 << 2) + lane; j < cnt; j += 64) st_out<NT>(out + j, w_obs[j]);
}


// x in [-pi, pi) (fp32 pi rounds up, so the strict bounds are the fp32 values in [-pi, pi)); NaN: false
__device__ __forceinline__ bool in_pi_range(float x) {
    return x > -3.14159274101257324f && x < 3.14159274101257324f;
}

// RK4 combinations (dynamics.py:158-171) on pairs of state components, so that they issue as packed
// fp32 (v_pk_fma_f32: two lanes' worth of fma per instruction at the issue cost of one): each
// component is rounded exactly as the scalar `acc += 2k; st = hs + k h` / `hs += (acc + k) dt/6`.
typedef float f32x2 __attribute__((ext_vector_type(2)));
template <bool FIRST>
__device__ __forceinline__ void rk_stage(const float* hs, const float* k, float* acc, float* st, float h) {
#pragma unroll
    for (int c = 0; c < 18; c += 2) {
        const f32x2 kk = {k[c], k[c + 1]}, hh = {hs[c], hs[c + 1]};
        f32x2 aa;
        if (FIRST) {
            aa = kk;
        } else {
            const f32x2 a0 = {acc[c], acc[c + 1]};
            aa = a0 + 2.f * kk;
        }
        const f32x2 ss = hh + kk * h;
        acc[c] = aa.x; acc[c + 1] = aa.y;
        st[c] = ss.x; st[c + 1] = ss.y;
    }
}

__device__ __forceinline__ void rk_update(float* hs, const float* k, const float* acc, float dt6) {
#pragma unroll
    for (int c = 0; c < 18; c += 2) {
        const f32x2 kk = {k[c], k[c + 1]}, hh = {hs[c], hs[c + 1]}, aa = {acc[c], acc[c + 1]};
        const f32x2 r = hh + (aa + kk) * dt6;
        hs[c] = r.x; hs[c + 1] = r.y;
    }
}

// Turbulence noise of a step (wind_dynamics.py:49-52: eta = randn(3) / sqrt(dt)): injected by the
// caller (ETA), or Box-Muller normals from Philox4x32-10 keyed by (global env id, step, episode).
template <bool ETA>
__device__ __forceinline__ void draw_eta(const StepArgs& a, uint64_t seed, int64_t env_offset, const Params<float>& P,
                                         int64_t so, int64_t blk0,
                                         uint32_t lo, int32_t step, int32_t epi, float eta[3]) {
    if (ETA) {
        const float* eb = a.eta + 3 * (so + blk0);
        eta[0] = ld_lane(eb + 0, 3 * lo);
        eta[1] = ld_lane(eb + 1, 3 * lo);
        eta[2] = ld_lane(eb + 2, 3 * lo);
    } else {
        const uint64_t gid = (uint64_t)(env_offset + blk0 + lo);
        const U4 r = philox(U4{(uint32_t)gid, (uint32_t)(gid >> 32), (uint32_t)step, (uint32_t)epi},
                            (uint32_t)seed, (uint32_t)(seed >> 32));
        // Box-Muller.  Radii sqrt(-2 ln u) / sqrt(dt) = sqrt(log2(u) * (-2 ln 2 / dt)) with u in (0, 1]
        // from the top 24 bits; angles in revolutions for the hardware sin / cos (v_sin_f32 takes
        // revolutions: sin(2 pi u) = v_sin(u)), u in [1, 2) from the top 23 bits (a whole turn apart)
        const float rk = P.eta_norm * P.eta_norm * -1.38629436111989061f;   // -2 ln 2 / dt
        const float r0 = sqrtf(__log2f(u01(r.x)) * rk);
        const float r1 = sqrtf(__log2f(u01(r.z)) * rk);
        const float a1 = __uint_as_float((r.y >> 9) | 0x3f800000u), a3 = __uint_as_float((r.w >> 9) | 0x3f800000u);
        eta[0] = r0 * __builtin_amdgcn_cosf(a1);
        eta[1] = r0 * __builtin_amdgcn_sinf(a1);
        eta[2] = r1 * __builtin_amdgcn_cosf(a3);
    }
}

// Diagnostic build only: per-wave phase timestamps (s_memtime) of one launch, for latency
// attribution; lane 0 of each of the first HG_TIMING_WAVES waves records them.
#ifndef HG_TIMING
#define HG_TIMING 0
#endif

#if HG_TIMING
#define HG_TIMING_WAVES 2048
#define HG_TIMING_SLOTS 17   // 0..13 phase stamps, 14/15 realtime end/start, 16 the wave's branch flags
__device__ unsigned long long g_timing[HG_TIMING_WAVES][HG_TIMING_SLOTS];
#define TSTAMP(j, ...)                                                                          \
    do {                                                                                        \
        asm volatile("" ::__VA_ARGS__);                                                         \
        const unsigned long long t_ = __builtin_amdgcn_s_memtime();                             \
        const int w_ = (int)(i >> 6);                                                           \
        if ((tid & 63) == 0 && w_ < HG_TIMING_WAVES) g_timing[w_][j] = t_;                      \
    } while (0)
// the stamping wave's tile from the hardware ids (the small-batch kernel's blocks are a stepping wave and
// its helper: the stepping wave is wave 0, its tile the block).  A 128-thread block is taken for the
// small-batch kernel's, so the timing build keeps the one-wave step blocks of the default build.
static_assert(HG_STEP_BLOCK != 128, "HG_TIMING builds tell the helper kernel's blocks by their 128 threads");
#define HG_STAMP_WAVE() (blockDim.x == 128 ? (int)blockIdx.x : (int)((blockIdx.x * blockDim.x + threadIdx.x) >> 6))
// the same stamp from inside the RK driver (stage_f32.h), where only the hardware ids are in scope
#define HG_STAGE_STAMP(j, ...)                                                                  \
    do {                                                                                        \
        asm volatile("" ::__VA_ARGS__);                                                         \
        const unsigned long long t_ = __builtin_amdgcn_s_memtime();                             \
        const int w_ = HG_STAMP_WAVE();                                                         \
        if ((threadIdx.x & 63) == 0 && w_ < HG_TIMING_WAVES) g_timing[w_][j] = t_;              \
    } while (0)
// which wave-uniform branches the wave took (HG_TIMING builds): 1 reset, 2 gear contact code,
// 4 the full sincos of a large attitude increment
#define HG_STAGE_FLAG(bit)                                                                      \
    do {                                                                                        \
        const int w_ = HG_STAMP_WAVE();                                                         \
        if ((threadIdx.x & 63) == 0 && w_ < HG_TIMING_WAVES) g_timing[w_][16] |= (bit);         \
    } while (0)
// the small-batch kernel's helper waves (one per tile): 0 start (s_memrealtime), 1 start (s_memtime),
// 2 the tile's counters arrived (noise key), 3 noise and wind step done, 4 past the hand-off barrier
__device__ unsigned long long g_timing_help[HG_TIMING_WAVES][5];
#define HSTAMP(j, ...)                                                                          \
    do {                                                                                        \
        asm volatile("" ::__VA_ARGS__);                                                         \
        const unsigned long long t_ = __builtin_amdgcn_s_memtime();                             \
        if (lane == 0 && tile < HG_TIMING_WAVES) g_timing_help[tile][j] = t_;                   \
    } while (0)
#else
#define TSTAMP(j, ...) do { } while (0)
#define HSTAMP(j, ...) do { } while (0)
#endif

}  // namespace
#include "stage_f32.h"   // (after the timing macros: HG_STAGE_STAMP)
namespace {

// TASK: reward / success of the task; ETA: noise injected by the caller (else in-kernel Philox);
// NT: streaming output stores (see st_out); FEAT: the optional features (reset-info compaction,
// per-reset re-trim, next-step auto-reset, TimeLimit) -- without them the kernel carries none of
// their registers; MULTI: a.nsteps consecutive steps per launch (hg_rollout) with the env state
// kept in registers between them; BAKED: the default airframe's model constants compiled in as
// instruction literals (baked.h), the runtime fields still read from the device copy.  All
// compile-time, so the hot kernel has no data-independent branches to merge around.
// The body is a device function so that the run-time specialised code objects (step_rtc.hip) wrap
// the same code in kernels of their own names.
template <int TASK, bool ETA, bool NT, bool FEAT, bool MULTI, bool BAKED, bool NTS, int HELP = 0>
__device__ __forceinline__ void step_body(float* __restrict__ state_p, int64_t n_p, uint64_t seed_p, int64_t envoff_p,
                                          ParamArg Pa, const Template<float>* __restrict__ Tp, const StepArgs& a,
                                          int64_t bid) {
    static_assert(HELP == 0 || (!ETA && !MULTI), "wind helper waves: in-kernel noise, one step per launch");
    __shared__ float s_obs[(HELP ? HELP * 64 : kStepBlock) * HG_N_OBS];   // one 64-row slice per wave
    __shared__ float s_wind[HELP ? HELP * 8 * 64 : 1];   // HELP: each tile's wind output and wind state
    constexpr bool kNTS = NT || NTS;   // non-temporal output stores
    const Params<float>& P0 = *Pa;   // model constants: scalar loads from a device copy
    // BAKED: the default airframe's constants as instruction literals (baked.h); only the runtime
    // fields (dt, target, limits, flags) are loaded
    Params<float> PB;
    if constexpr (BAKED) PB = hg::bake(*Pa);
    const int lane = threadIdx.x & 63;
    // HELP: blocks of HELP tiles, waves 0 .. HELP-1 step them, waves HELP .. 2 HELP-1 run their noise and
    // wind step (helper wave j + HELP for tile j) and hand it over in LDS
    const int wave_id = (kStepBlock == 64 && HELP == 0) ? 0 : __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wv = HELP ? wave_id % (HELP ? HELP : 1) : wave_id;   // uniform
    const int64_t tile = bid * (HELP ? HELP : kStepBlock / 64) + wv;
    const int64_t blk0 = tile * 64;   // this wave's first env
    const int tid = lane;
    const int64_t i = blk0 + tid;
    const int64_t n = n_p;
    const bool active = i < n;
    // Addressing: this wave's state tile (7 groups x 64 lanes x 16 bytes, contiguous, retrim.h) from
    // one uniform (SGPR) base at group 4, so every group is an immediate offset (-4 .. +2 KB, inside
    // the 13-bit field) of the same SGPR-base access with the lane's byte offset: no address
    // arithmetic per group.  Lanes past the end of a ragged last tile step its padding and store
    // nothing; for the caller's [N]-row buffers they read row blk0.
    const uint32_t lo = (uint32_t)(active ? tid : 0);
    const uint32_t lt = (uint32_t)tid;
    f32x4* st_b = reinterpret_cast<f32x4*>(state_p + tile * kTileWords) + 4 * kTileEnvs;
#define GRP(ptr, g) ((ptr) + ((g) - 4) * kTileEnvs)

#if HG_TIMING
    if ((tid & 63) == 0 && (i >> 6) < HG_TIMING_WAVES) {
        g_timing[i >> 6][15] = __builtin_amdgcn_s_memrealtime();
        g_timing[i >> 6][16] = 0;
    }
#endif
    if constexpr (HELP > 0) {
        const bool helper = wave_id >= HELP;
        if (tile * 64 >= n_p) {   // (a last block's missing tiles: both waves meet at the barrier)
            asm volatile("s_barrier" ::: "memory");
            return;
        }
        if (helper) {   // the tile's noise and wind step (Heli.step :195-199), the same code as below
#if HG_TIMING
            if (lane == 0 && tile < HG_TIMING_WAVES) g_timing_help[tile][0] = __builtin_amdgcn_s_memrealtime();
#endif
            HSTAMP(1, "v"(lane));
            const Params<float>& PH = BAKED ? PB : P0;
            const f32x4 g0 = ld_lane(GRP(st_b, 0), lt), g1 = ld_lane(GRP(st_b, 1), lt), g2 = ld_lane(GRP(st_b, 2), lt),
                        g3 = ld_lane(GRP(st_b, 3), lt);
            float ws[5], carry[4], eta[3], W[3];
            carry[3] = g1.z; carry[0] = g1.w; carry[1] = g2.x; carry[2] = g2.y;
            ws[0] = g2.z; ws[1] = g2.w; ws[2] = g3.x; ws[3] = g3.y; ws[4] = g3.z;
            HSTAMP(2, "v"(g0.w), "v"(g1.x));
            draw_eta<false>(a, seed_p, envoff_p, PH, 0, blk0, lo, __float_as_int(g0.w), __float_as_int(g1.x), eta);
            hg::wind_step_f32<true>(PH, ws, carry, eta, W);
            HSTAMP(3, "v"(W[0]), "v"(ws[4]));
            float* sw = s_wind + wv * 8 * 64 + lane;
            sw[0] = W[0]; sw[64] = W[1]; sw[128] = W[2];
#pragma unroll
            for (int c = 0; c < 5; ++c) sw[(3 + c) * 64] = ws[c];
            asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
            HSTAMP(4, "v"(lane));
            return;
        }
    }
    TSTAMP(0, "v"(tid));
    // reset template (heli[18] | carry[4] | obs[17]) one float per lane, requested with the state so
    // that a reset costs no round trip at the end (and no late load is outstanding when the step
    // ends: a load issued near the stage-4 code makes the compiler wait for it there)
    // the helper kernel: every lane loads (the device copy is padded to one float per lane, kTplAlloc),
    // no divergent load (4 096 envs 5.20 -> 5.15 us; the other kernels measured slower so)
    const float tpl = (HELP > 0 && HG_TPL_FULL_HELP) || lane < kTplFloats ? reinterpret_cast<const float*>(Tp)[lane] : 0.f;
    // The state groups in the order they are needed (retrim.h slot table): position and step
    // counter (-> terrain texel address, noise key), the rest of the key and the carry, the wind
    // state (-> wind step), then the heli state.  hs[2], hs[3] (the rotor azimuths) are not stepped.
    float hs[18], ws[5], carry[4];
    int32_t step, succ, epi;
    {
        // (HELP: group 2 -- carry[1..2], wind state -- is the helper wave's; the carry is rewritten
        // at the end of every step and the wind state comes back from the helper)
        const f32x4 g0 = ld_lane(GRP(st_b, 0), lt), g1 = ld_lane(GRP(st_b, 1), lt),
                    g2 = HELP ? f32x4{0.f, 0.f, 0.f, 0.f} : ld_lane(GRP(st_b, 2), lt),
                    g3 = ld_lane(GRP(st_b, 3), lt), g4 = ld_lane(GRP(st_b, 4), lt), g5 = ld_lane(GRP(st_b, 5), lt),
                    g6 = ld_lane(GRP(st_b, 6), lt);
        hs[15] = g0.x; hs[16] = g0.y; hs[17] = g0.z; step = __float_as_int(g0.w);
        epi = __float_as_int(g1.x); succ = __float_as_int(g1.y); carry[3] = g1.z; carry[0] = g1.w;
        carry[1] = g2.x; carry[2] = g2.y; ws[0] = g2.z; ws[1] = g2.w;
        ws[2] = g3.x; ws[3] = g3.y; ws[4] = g3.z; hs[14] = g3.w;
        hs[0] = g4.x; hs[1] = g4.y; hs[4] = g4.z; hs[5] = g4.w;
        hs[6] = g5.x; hs[7] = g5.y; hs[8] = g5.z; hs[9] = g5.w;
        hs[10] = g6.x; hs[11] = g6.y; hs[12] = g6.z; hs[13] = g6.w;
        hs[2] = 0.f; hs[3] = 0.f;
    }
#ifndef HG_EARLY_PAIRS   // 1: the stages' constant pairs formed while the state loads are in flight (round 5
#define HG_EARLY_PAIRS 0  // A/B: 7.062 -> 7.088 us, profiles/r05_valu_ab.txt; not adopted)
#endif
#if HG_EARLY_PAIRS
    // (data-independent: issued ahead of the first wait for the state, off the step's critical path)
    const hg::StepK Kpairs = hg::step_k<NT && HG_PIN_CONSTANTS>(BAKED ? PB : P0);
#endif
    if (FEAT && bid == 0 && tid == 0) {   // counters of a later step (rings of three)
        if (a.reset_count_next) *a.reset_count_next = 0;
        if (a.retrim_slot >= 0 && a.retrim_count) a.retrim_count[a.retrim_slot == 2 ? 0 : a.retrim_slot + 1] = 0;
        if (a.ov_count_next) *a.ov_count_next = 0;
    }
    if (FEAT && bid == 0 && a.fused_next && tid < kFusedWaveCtrs + 1) a.fused_next[kFusedLine * tid] = 0;
    if (FEAT && bid == 0 && a.fused_next && tid < 2) a.fused_next[1 + tid] = 0;
    const int nsteps = MULTI ? a.nsteps : 1;
    bool defer_st = false;   // (one step per launch) a deferred reset: the step counter alone is stored
    // the re-trim queue (below): the wave's job mask, the slot counter's old value (leader lane), this
    // lane's job and its trim wind
    unsigned long long rt_mask = 0;
    int rt_base = 0;
    bool rt_job = false, rt_next = false;
    // (the bulk variant writes them at once: the values kept live past the stores cost it registers,
    // 262 144 envs 46.6 -> 47.3 us with the late write)
    constexpr bool kRtLate = HG_RT_QUEUE_LATE && NT && !MULTI;
    unsigned long long rc_mask = 0;   // the same for the compacted reset info
    int rc_base = 0;
    bool rc_job = false;
    float fo[kRtLate ? 17 : 1];
    float rw0 = 0.f, rw1 = 0.f, rw2 = 0.f;
    auto rt_queue = [&]() {
        if (FEAT && rt_mask) {
            const int leader = __ffsll((long long)rt_mask) - 1;
            const int slot = __builtin_amdgcn_readlane(rt_base, leader) + __popcll(rt_mask & ((1ull << lane) - 1ull));
            if (rt_job && slot < n) {
                if (rt_next) {   // a next-step reset: the wind recorded at the episode's last step
                    rw0 = a.retrim_wind[i];
                    rw1 = a.retrim_wind[n + i];
                    rw2 = a.retrim_wind[2 * n + i];
                }
                if (a.fused_ctr) {
                    // fused: the wind, then env, as device-coherent (agent-scope) stores with a wait for
                    // the wind's between them -- the trim polls env and then reads the wind the same
                    // way.  No release: the trim reads nothing else this wave stored (deferred reset),
                    // so no L2 write-back is needed, and its waits for the record flush no cache.
                    int* rp = reinterpret_cast<int*>(a.retrim_recs + slot);
                    __hip_atomic_store(rp + 1, __float_as_int(rw0), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    __hip_atomic_store(rp + 2, __float_as_int(rw1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    __hip_atomic_store(rp + 3, __float_as_int(rw2), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    __hip_atomic_store(rp, (int)i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                } else {
                    a.retrim_recs[slot] = make_int4((int32_t)i, __float_as_int(rw0), __float_as_int(rw1), __float_as_int(rw2));
                }
            }
        }
    };
    for (int sstep = 0; sstep < nsteps; ++sstep) {
    // MULTI: the constants are re-read (scalar cache) each step rather than kept live across the
    // loop, where ~130 of them would spill out of the SGPR file
    const Params<float>& P = BAKED ? PB : (MULTI ? *reload_params(Pa) : P0);
    const int64_t so = MULTI ? (int64_t)sstep * n : 0;   // first row of this step's inputs / outputs
    const float4 act = ld_lane(reinterpret_cast<const float4*>(a.actions) + so + blk0, lo);
    // terrain texels under the committed position (F6): issued now, combined after the wind step
    const hg::GroundCell<float> cell_c = hg::ground_cell(P, hs[15], hs[16]);
    const hg::GroundTexels tex_c = hg::ground_fetch(a.hmap, cell_c);

    TSTAMP(1, "v"(hs[17]), "v"(act.w), "v"(epi), "v"(carry[3]), "v"(ws[4]));
    float W[3];
    hg::StepCtx ctx;
    hg::RK4Step<NT, (HELP > 0)> rk;   // NT: the launch is one wave per SIMD; HELP: stage 1 split
    if constexpr (HELP > 0) {
        // the wind-independent part of the step's shared context and of stage 1 (kinematics, gear)
        // while the helper wave runs the wind
        const hg::Ground<float> h_c = hg::ground_combine<float>(tex_c, cell_c);
        ctx = hg::step_ctx(P, act.x, act.y, act.z, act.w, 0.f, 0.f, 0.f, h_c, hs[17]);
#if HG_EARLY_PAIRS
        rk.begin(P, ctx, hs, hg::att0(hs), Kpairs);
#else
        rk.begin(P, ctx, hs, hg::att0(hs));
#endif
        TSTAMP(2, "v"(ctx.z0), "v"(hs[0]));   // (HELP: the wind-independent context and stage-1 share done)
        asm volatile("s_barrier" ::: "memory");
        TSTAMP(3, "v"(tid));                  // (HELP: past the hand-off barrier)
        const float* sw = s_wind + wv * 8 * 64 + lane;
        W[0] = sw[0]; W[1] = sw[64]; W[2] = sw[128];
#pragma unroll
        for (int c = 0; c < 5; ++c) ws[c] = sw[(3 + c) * 64];
        ctx.W0 = W[0]; ctx.W1 = W[1]; ctx.W2 = W[2];
        TSTAMP(4, "v"(W[0]), "v"(ws[4]));     // (HELP: the wind read from LDS)
    } else {
    // turbulence noise (wind_dynamics.py:49-52): injected, or Philox normals
    float eta[3];
    draw_eta<ETA>(a, seed_p, envoff_p, P, so, blk0, lo, step, epi, eta);

    // ground height under the committed position (F6), wind step (Heli.step :195-199)
    TSTAMP(2, "v"(eta[2]), "v"(eta[0]));
    hg::wind_step_f32<NT>(P, ws, carry, eta, W);   // (the lone-wave kernels: the uniform-branch form)
    TSTAMP(3, "v"(W[2]), "v"(W[0]));
    const hg::Ground<float> h_c = hg::ground_combine<float>(tex_c, cell_c);

    TSTAMP(4, "v"(h_c.delta), "v"(h_c.hi));
    ctx = hg::step_ctx(P, act.x, act.y, act.z, act.w, W[0], W[1], W[2], h_c, hs[17]);
#if HG_EARLY_PAIRS
    rk.begin(P, ctx, hs, hg::att0(hs), Kpairs);
#else
    rk.begin(P, ctx, hs, hg::att0(hs));
#endif
    }
    // RK4 (dynamics.py:158-171); observation from the stage-4 input (F5)
    float k[18], obs[17];
    rk.finish(P, ctx, hs, k, obs);
#if HG_EARLY_POST
    // the terrain texels under the post-step position (the flags' ground height), requested now so
    // that their latency hides behind the wraps and the reward
    const hg::GroundCell<float> cell_p = hg::ground_cell(P, hs[15], hs[16]);
    const hg::GroundTexels tex_p = hg::ground_fetch(a.hmap, cell_p);
#endif
    TSTAMP(8, "v"(hs[8]), "v"(hs[11]), "v"(obs[16]));
    if (FEAT && P.reset_retrim && active && !(P.autoreset_next && step < 0)) {   // F8: a reset trims against this wind
        float* wb = a.retrim_wind + blk0;   // [3][N]: three coalesced rows
        st_lane<false>(wb, (uint32_t)tid, W[0]);
        st_lane<false>(wb + n, (uint32_t)tid, W[1]);
        st_lane<false>(wb + 2 * n, (uint32_t)tid, W[2]);
    }
    // step_after (helicopter_dynamics.py:73-77)
    // utils.py pi_bound, (x + pi) % 2pi - pi.  An angle already in [-pi, pi) is kept as is -- what
    // the reference's fp64 arithmetic returns to 1e-16, where the fp32 round trip through x + pi
    // costs up to half an ulp of pi.  The rotor azimuths wrap in nearly every wave every step; the
    // flapping and euler angles only in a wave-uniform branch taken when one of them left the range.
    // (The rotor azimuths' wrap is az_advance's.)
    {
        const int ang[5] = {4, 5, 12, 13, 14};
        // every angle in (-pi, pi) <=> the largest |angle| below fp32 pi (two v_max3 with |.| operand
        // modifiers and one compare instead of five range tests; a NaN angle drops out of the max
        // and stays NaN either way)
        const float amax = fmaxf(fmaxf(fmaxf(fabsf(hs[4]), fabsf(hs[5])), fabsf(hs[12])),
                                 fmaxf(fabsf(hs[13]), fabsf(hs[14])));
        const bool all_in = amax < 3.14159274101257324f;
        if (__any(!all_in)) {
#pragma unroll
            for (int j = 0; j < 5; ++j) {
                const float x = hs[ang[j]];
                hs[ang[j]] = in_pi_range(x) ? x : hg::pi_bound(x);
            }
        }
    }

    TSTAMP(9, "v"(hs[0]));
    // reward (helicopter_with_tasks.py) and flags (helicopter.py:201-205, 219-240)
    bool success_step = false;
    float rew = 0.f;
    if (TASK == HG_TASK_HOVER) rew = hg::reward_hover(P, hs, k, &success_step);
    if (TASK == HG_TASK_FORWARD_FLIGHT) rew = hg::reward_forward(P, hs, k, &success_step);
#if HG_EARLY_POST
    const hg::Ground<float> h_post = hg::ground_combine<float>(tex_p, cell_p);
#else
    const hg::Ground<float> h_post = hg::ground_height(P, a.hmap, hs[15], hs[16]);
#endif
    const bool waiting = step < 0;   // ended last step, reset due now (next-step auto-reset)
    step += 1;
    const bool failed = hg::is_failed(P, hs, k, h_post);
    TSTAMP(10, "v"(rew), "v"((int)failed));
    const bool successed = succ >= P.success_steps;   // successed_time before this step's add
    const bool time_up = step >= P.time_up_steps;
    // next-step auto-reset: an env that ended last step (counter -(n + 1)) only resets this step
    const bool pending = FEAT && P.autoreset_next && waiting;
    const bool term = (failed || successed) && !pending;
    const bool trunc = (time_up || (FEAT && step >= P.max_episode_steps)) && !pending;   // + TimeLimit
    const bool done = term || trunc;
    succ += success_step ? 1 : 0;

    // auto-reset (same step, or the step after the end)
    const bool do_reset = P.autoreset && active && ((FEAT && P.autoreset_next) ? pending : done);
    // a reset whose trim runs concurrently with this step -- a next-step reset in ov mode, any reset in
    // a fused launch: only the step counter is stored here, the trim writes the rest
#ifndef HG_FUSED_NOTRIM   // diagnostic: 1, a fused launch's trim blocks leave at once and its resets
#define HG_FUSED_NOTRIM 0   // take the template (the step's own cost in that launch)
#endif
    const bool defer = FEAT && (a.ov_active || (a.fused_ctr && !HG_FUSED_NOTRIM)) && do_reset;
    defer_st = defer;
    if (active) {
        st_lane<kNTS>(a.reward + so + blk0, (uint32_t)tid, pending ? 0.f : rew);
        st_lane<kNTS>(a.terminated + so + blk0, (uint32_t)tid, (uint8_t)term);
        st_lane<kNTS>(a.truncated + so + blk0, (uint32_t)tid, (uint8_t)trunc);
        if (a.info)
            st_lane<kNTS>(a.info + so + blk0, (uint32_t)tid, pending ? (uint8_t)0 : (uint8_t)((failed ? HG_INFO_FAILED : 0) | (successed ? HG_INFO_SUCCESSED : 0) |
                                  (time_up ? HG_INFO_TIME_UP : 0) | (success_step ? HG_INFO_SUCCESS_STEP : 0) |
                                  (do_reset ? HG_INFO_RESET : 0)));
    }
    // uncompacted reset info (hg_step_rows): the terminal observation at the env's own row, in a
    // wave-uniform branch taken only by waves with a reset
    if (!MULTI && a.final_obs_rows && __ballot(do_reset)) {
        if (do_reset) {   // the 68-byte row as four 16-byte stores and one dword (dword-aligned rows)
            typedef float f4u __attribute__((ext_vector_type(4), aligned(4)));
            f4u* row = reinterpret_cast<f4u*>(a.final_obs_rows + i * 17);
#pragma unroll
            for (int q = 0; q < 4; ++q) row[q] = f4u{obs[4 * q], obs[4 * q + 1], obs[4 * q + 2], obs[4 * q + 3]};
            a.final_obs_rows[i * 17 + 16] = obs[16];
        }
    }

    // compacted reset info with a wave-ballot compaction (HG_RT_QUEUE_LATE: as the re-trim queue
    // below, the slots used after the state stores, the terminal observations kept until then)
    if (FEAT && P.autoreset && a.reset_count) {
        if constexpr (kRtLate) asm volatile("" ::"v"(tpl));
        const unsigned long long mask = __ballot(do_reset);
        if constexpr (kRtLate) {
            rc_mask = mask;
            if (mask) {
                const int leader = __ffsll((long long)mask) - 1;
                if (lane == leader) rc_base = atomicAdd(a.reset_count, __popcll(mask));
            }
#pragma unroll
            for (int c = 0; c < 17; ++c) fo[c] = obs[c];
            rc_job = do_reset;
        } else if (mask) {
            const int leader = __ffsll((long long)mask) - 1;
            int base = 0;
            if (lane == leader) base = atomicAdd(a.reset_count, __popcll(mask));
            base = __shfl(base, leader);
            if (do_reset) {
                const int slot = base + __popcll(mask & ((1ull << lane) - 1ull));
                if (a.reset_index && slot < n) a.reset_index[slot] = (int32_t)i;
                if (a.final_obs && slot < n) {
#pragma unroll
                    for (int c = 0; c < 17; ++c) a.final_obs[(int64_t)slot * 17 + c] = obs[c];
                }
            }
        }
    }
    if (FEAT && a.ov_recs) {   // ov mode: the episodes ending now, trimmed while the next step runs
        const bool ends = active && done && P.autoreset;
        const unsigned long long mask = __ballot(ends);
        if (mask) {
            const int leader = __ffsll((long long)mask) - 1;
            int base = 0;
            if (lane == leader) base = atomicAdd(a.ov_count, __popcll(mask));
            base = __shfl(base, leader);
            const int slot = base + __popcll(mask & ((1ull << lane) - 1ull));
            if (ends && slot < n)
                a.ov_recs[slot] = make_int4((int32_t)i, __float_as_int(W[0]), __float_as_int(W[1]), __float_as_int(W[2]));
        }
    }
    // queue the resets for retrim_kernel (which overwrites the template).  HG_RT_QUEUE_LATE: the slot
    // counter's atomic is issued here and its value used after the state stores (lone-wave
    // kernels, one step per launch: 65 536 envs same-step re-trim 30.43 -> 30.11 us), so that the round trip of the device-scope atomic overlaps them instead of lengthening
    // the wave (the library is built without the atomic optimizer, which would read the value here)
    if (FEAT && P.reset_retrim) {
        // the reset template's load (issued at the start) waited for here, not after the atomic
        if constexpr (kRtLate) asm volatile("" ::"v"(tpl));
        rt_job = do_reset && !a.ov_active;
        rt_mask = __ballot(rt_job);
        if (a.fused_ctr) {
            // fused: every wave counts itself, so that the trim waves know the queue is complete once
            // the count reaches the wave count.  A wave with jobs reserves them and counts itself in
            // one atomic (its jobs in the low word, itself in the high word); a wave without, in one of
            // kFusedWaveCtrs counters on lines of their own, without waiting for the old value: every
            // wave on one address serialised the atomics (65 536 envs: the step waves ended 10 to 45 us
            // into the launch, scripts/fused_probe.py)
            if (rt_mask) {
                const int leader = __ffsll((long long)rt_mask) - 1;
                if (lane == leader)
                    rt_base = (int)(uint32_t)atomicAdd(a.fused_ctr, (1ull << 32) | (unsigned long long)__popcll(rt_mask));
            } else if (lane == 0) {
                int32_t* wc = reinterpret_cast<int32_t*>(a.fused_ctr) + kFusedLine * (1 + (int)(bid % kFusedWaveCtrs));
                __hip_atomic_fetch_add(wc, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        } else if (rt_mask) {
            const int leader = __ffsll((long long)rt_mask) - 1;
            if (lane == leader) rt_base = atomicAdd(a.retrim_count + (a.retrim_slot > 0 ? a.retrim_slot : 0), __popcll(rt_mask));
        }
        rt_next = P.autoreset_next;
        rw0 = W[0];   // the job's trim wind (same-step reset; a next-step reset reads its own, below)
        rw1 = W[1];
        rw2 = W[2];
    }
    if (!kRtLate) rt_queue();
    if (FEAT && P.env_templates) {   // this env's own reset target (its own trim condition)
        if (do_reset) {
            const float* tr = a.tmpl_env + (int64_t)i * kTplFloats;
#pragma unroll
            for (int c = 0; c < 18; ++c) hs[c] = tr[c];
#pragma unroll
            for (int c = 0; c < 4; ++c) carry[c] = tr[18 + c];
#pragma unroll
            for (int c = 0; c < 17; ++c) obs[c] = tr[22 + c];
            // the loads complete inside this branch (vmcnt(0)): the memory-counter waits after the join
            // then need not count the re-trim queue's atomic on the other path
            if constexpr (kRtLate) __builtin_amdgcn_s_waitcnt(0xF70);
        }
    } else if (__ballot(do_reset)) {
#if HG_TIMING
        HG_STAGE_FLAG(1);
#endif
        // Template<float> = heli[18] | carry[4] | obs[17], float c held by lane c.  The readlanes run
        // in this wave-uniform branch (every lane has loaded its template float), the selects per lane.
#pragma unroll
        for (int c = 0; c < 18; ++c) {
            const float v = lane_value(tpl, c);
            hs[c] = do_reset ? v : hs[c];
        }
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const float v = lane_value(tpl, 18 + c);
            carry[c] = do_reset ? v : carry[c];
        }
#pragma unroll
        for (int c = 0; c < 17; ++c) {
            const float v = lane_value(tpl, 22 + c);
            obs[c] = do_reset ? v : obs[c];
        }
    }
    if constexpr (NT) {
        // the lone-wave kernels: the same assignments as selects, no divergent branch (65 536 envs
        // -0.08 us; the bulk variant keeps the branch)
#pragma unroll
        for (int c = 0; c < 5; ++c) ws[c] = do_reset ? 0.f : ws[c];
        carry[0] = do_reset ? carry[0] : obs[4];
        carry[1] = do_reset ? carry[1] : obs[5];
        carry[2] = do_reset ? carry[2] : obs[6];
        carry[3] = do_reset ? carry[3] : obs[16];
        step = do_reset ? 0 : ((FEAT && P.autoreset_next && done) ? -step - 1 : step);
        succ = do_reset ? 0 : succ;
        epi = do_reset ? epi + 1 : epi;
    } else if (do_reset) {
#pragma unroll
        for (int c = 0; c < 5; ++c) ws[c] = 0.f;
        step = 0;
        succ = 0;
        epi += 1;
    } else {
        carry[0] = obs[4];
        carry[1] = obs[5];
        carry[2] = obs[6];
        carry[3] = obs[16];
        if (FEAT && P.autoreset_next && done) step = -step - 1;   // reset on the next step (n = step kept)
    }
    uint64_t skip_rows = 0;
    if (FEAT && !MULTI) skip_rows = __ballot(defer);
    store_obs_wave<kNTS, MULTI>(s_obs + wv * 64 * HG_N_OBS, obs, a.obs, so, blk0, n, lane, skip_rows);
    }   // steps
    TSTAMP(13, "v"(hs[0]), "v"(carry[3]));
    st_b = reinterpret_cast<f32x4*>(state_p + tile * kTileWords) + 4 * kTileEnvs;
    asm volatile("" : "+s"(st_b));
    if (FEAT && !MULTI && __ballot(defer_st)) {   // a deferred reset: its step counter only (the trim writes the rest)
        if (defer_st) reinterpret_cast<int32_t*>(GRP(st_b, 0) + tid)[3] = 0;
    }
    if (active && !(FEAT && !MULTI && defer_st)) {
        // the lane index re-materialised in this block, so that each store selects the SGPR-base
        // form (a 32-bit lane offset) instead of a 64-bit VALU address add per store
        uint32_t t = (uint32_t)tid;
        asm volatile("" : "+v"(t));
        st_lane<kNTS>(GRP(st_b, 0), t, f32x4{hs[15], hs[16], hs[17], __int_as_float(step)});
        st_lane<kNTS>(GRP(st_b, 1), t, f32x4{__int_as_float(epi), __int_as_float(succ), carry[3], carry[0]});
        st_lane<kNTS>(GRP(st_b, 2), t, f32x4{carry[1], carry[2], ws[0], ws[1]});
        st_lane<kNTS>(GRP(st_b, 3), t, f32x4{ws[2], ws[3], ws[4], hs[14]});
        st_lane<kNTS>(GRP(st_b, 4), t, f32x4{hs[0], hs[1], hs[4], hs[5]});
        st_lane<kNTS>(GRP(st_b, 5), t, f32x4{hs[6], hs[7], hs[8], hs[9]});
        st_lane<kNTS>(GRP(st_b, 6), t, f32x4{hs[10], hs[11], hs[12], hs[13]});
    }
#undef GRP
    if (kRtLate) rt_queue();
    if constexpr (kRtLate) {
        if (FEAT && rc_mask) {
            const int leader = __ffsll((long long)rc_mask) - 1;
            const int slot = __builtin_amdgcn_readlane(rc_base, leader) + __popcll(rc_mask & ((1ull << lane) - 1ull));
            if (rc_job && slot < n) {
                if (a.reset_index) a.reset_index[slot] = (int32_t)i;
                if (a.final_obs) {
#pragma unroll
                    for (int c = 0; c < 17; ++c) a.final_obs[(int64_t)slot * 17 + c] = fo[c];
                }
            }
        }
    }

    TSTAMP(11, "v"(tid));
#if HG_TIMING
    __builtin_amdgcn_s_waitcnt(0);
    TSTAMP(12, "v"(tid));
    if ((tid & 63) == 0 && (i >> 6) < HG_TIMING_WAVES) g_timing[i >> 6][14] = __builtin_amdgcn_s_memrealtime();
#endif
}

template <int TASK, bool ETA, bool NT, bool FEAT, bool MULTI, bool BAKED, bool NTS>
__global__ __launch_bounds__(kStepBlock, NT ? HG_MIN_WAVES : HG_MIN_WAVES_BULK) void step_kernel(float* __restrict__ state_p, int64_t n_p, uint64_t seed_p,
                                                      int64_t envoff_p, ParamArg Pa,
                                                      const Template<float>* __restrict__ Tp, const StepArgs a) {
    step_body<TASK, ETA, NT, FEAT, MULTI, BAKED, NTS>(state_p, n_p, seed_p, envoff_p, Pa, Tp, a, blockIdx.x);
}

// Small batches (up to half a wave per SIMD): each block is a tile's wave and a helper wave that runs
// the tile's noise and wind step (no input from the helicopter state) while the tile's wave loads
// its state and forms the rest of the step's context (density, controls, terrain, attitude
// sin/cos), the wind handed over in LDS at one barrier.  Bitwise the one-wave kernel (tested).
// Per step, against the one-wave kernel: 4 096 envs 5.80 -> 5.63 us, 16 384 6.29 -> 6.08,
// 32 768 6.73 -> 6.63 (profiles/r04_helper_ab.txt).  Not used at a wave per SIMD, where the helpers
// share SIMDs with the stepping waves: 65 536 envs 7.39 -> 7.44 us (blocks of 2 or 4 tiles with their
// helpers: 8.81, 7.59).
#ifndef HG_HELPER   // tiles per block in the small-batch helper kernel; 0: none
#define HG_HELPER 1
#endif
#ifndef HG_HELPER_DIV   // the helper kernel up to resident_envs / HG_HELPER_DIV envs (2: two tiles per CU)
#define HG_HELPER_DIV 2
#endif
#if HG_HELPER > 0
template <int TASK, bool FEAT, bool BAKED>
__global__ __launch_bounds__(128 * HG_HELPER, 1) void step_help_kernel(float* __restrict__ state_p, int64_t n_p, uint64_t seed_p,
                                                                    int64_t envoff_p, ParamArg Pa,
                                                                    const Template<float>* __restrict__ Tp, const StepArgs a) {
    step_body<TASK, false, true, FEAT, false, BAKED, false, HG_HELPER>(state_p, n_p, seed_p, envoff_p, Pa, Tp, a, blockIdx.x);
}
#endif

#ifndef HG_RTC
// reset_mode RETRIM with next-step auto-reset (hg_env::ov): one launch holds the trims of the previous
// step's ends -- its first `tb` blocks, one wave per trim (retrim_body.h) -- and this step, whose
// deferred resets store only their step counter while those trims write the rest.  Both parts fit
// two waves per SIMD (<= 256 VGPRs), so at one step wave per SIMD a trim wave shares a SIMD with a
// step wave; the trims, dispatched first, are the long pole.  One queue and no cross-stream events:
// dependent work on another queue waited about 10 us per hop on MI355X (scripts/r04_ov_trace.py).
// The leading (preloaded) arguments are the trims' job count, records, setup and model constants
// (r.count, r.recs, r.T, r.P): the trim waves are the long pole and request them at once; the step
// waves read the rest of their arguments from the argument segment instead.
template <int TASK, bool BAKED>
__global__ __launch_bounds__(kStepBlock) __attribute__((amdgpu_waves_per_eu(2))) void step_ov_kernel(
    const int32_t* __restrict__ rcount, const int4* __restrict__ rrecs, const hg::TrimSetup* __restrict__ rT,
    const hg::Params<double>* __restrict__ rP, float* __restrict__ state_p, int64_t n_p, uint64_t seed_p,
    int64_t envoff_p, ParamArg Pa, const Template<float>* __restrict__ Tp, const StepArgs a, const hgk::RetrimArgs r,
    int32_t tb) {
    if ((int32_t)blockIdx.x < tb) {
        // retrim_jobs treats threadIdx.x as the lane of one wave (Jacobian column, trial, LDS rows):
        // a trim block is its first wave (the others, with HG_STEP_BLOCK > 64, leave at once)
        if (kStepBlock == 64 || threadIdx.x < 64) hgk::retrim_jobs(r, blockIdx.x, tb, rcount, rrecs, rT, rP, 0);
        return;
    }
    step_body<TASK, false, true, true, false, BAKED, false>(state_p, n_p, seed_p, envoff_p, Pa, Tp, a,
                                                             (int64_t)blockIdx.x - tb);
}

// reset_mode RETRIM with same-step auto-reset, lone-wave sizes: one launch holds the step and the trims
// of the resets it queues.  Its first `tb` blocks are trim waves that claim jobs one at a time and wait
// (s_sleep polls) for each job's record, which the step wave that queued it publishes at its end; a
// trim starts as soon as its env's step wave is done instead of after the slowest wave, a launch gap
// and a retrim_kernel start-up.  The resets are deferred as in ov mode (the step wave stores only the
// step counter, the trim the rest), so the trim reads nothing the step wave stored but the record, and
// the hand-over is device-coherent stores and loads -- no release or acquire, whose L2 write-back and
// invalidate per poll slowed the whole launch (a first version: 65 536 envs 91 us per step against
// 29 serial).  Every step wave reserves its queue slots in one 64-bit counter that also counts the
// waves, so the trim waves leave once every wave has reserved and the claims are past the queue (and
// after a bounded wait in any case).  Bitwise the serial path (tested).
template <int TASK, bool BAKED>
__global__ __launch_bounds__(kStepBlock) __attribute__((amdgpu_waves_per_eu(2))) void step_fused_kernel(
    const int32_t* __restrict__ rcount, const int4* __restrict__ rrecs, const hg::TrimSetup* __restrict__ rT,
    const hg::Params<double>* __restrict__ rP, float* __restrict__ state_p, int64_t n_p, uint64_t seed_p,
    int64_t envoff_p, ParamArg Pa, const Template<float>* __restrict__ Tp, const StepArgs a, const hgk::RetrimArgs r,
    int32_t tb) {
    if ((int32_t)blockIdx.x < tb) {
        if (!HG_FUSED_NOTRIM && (kStepBlock == 64 || threadIdx.x < 64))
            hgk::retrim_jobs<true>(r, blockIdx.x, tb, rcount, rrecs, rT, rP, 0);
        return;
    }
    step_body<TASK, false, true, true, false, BAKED, false>(state_p, n_p, seed_p, envoff_p, Pa, Tp, a,
                                                             (int64_t)blockIdx.x - tb);
}
#endif

#ifdef HG_RTC   // step_rtc.hip: the step kernel's code and nothing else
}  // namespace
#else

// reset_mode RETRIM bookkeeping: the wind each env's next reset is trimmed against (the mean wind
// until the env has stepped, helicopter.py:55), and the compacted list of masked envs of hg_reset.
__global__ __launch_bounds__(kBlock) void fill_wind_kernel(float* wind, int64_t n, float w0, float w1, float w2) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    wind[i] = w0;   // [3][N]
    wind[n + i] = w1;
    wind[2 * n + i] = w2;
}

__global__ __launch_bounds__(kBlock) void mask_list_kernel(const uint8_t* mask, int64_t n, int32_t* list,
                                                           int32_t* count) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    const bool take = i < n && (!mask || mask[i]);
    const unsigned long long m = __ballot(take);
    if (!m) return;
    const int lane = threadIdx.x & 63, leader = __ffsll((long long)m) - 1;
    int base = 0;
    if (lane == leader) base = atomicAdd(count, __popcll(m));
    base = __shfl(base, leader);
    if (take) list[base + __popcll(m & ((1ull << lane) - 1ull))] = (int32_t)i;
}

// hg_clock_stamp: the constant 100 MHz GPU clock at the point of the stream this kernel occupies (the
// value is moved to a vector register and stored with a vector store)
__global__ __launch_bounds__(64) void clock_stamp_kernel(uint64_t* dst) {
    uint64_t t = __builtin_amdgcn_s_memrealtime();
    asm volatile("" : "+v"(t));
    if (threadIdx.x == 0) *dst = t;
}

// Job counters zeroed ahead of the launch that counts into them.  A one-thread kernel, not
// hipMemsetAsync: captured into a hipGraph, a 4-byte memset node left the counter non-zero on later
// replays on MI355X (0x08080808 and stale counts in scripts/r04_retrim_fault.py), so the re-trim
// read a job count past the records its step wrote; a kernel node keeps its arguments by value.
__global__ __launch_bounds__(64) void zero_counts_kernel(int32_t* a, int32_t* b, int32_t* c, int32_t* d) {
    if (threadIdx.x == 0) {
        if (a) *a = 0;
        if (b) *b = 0;
        if (c) *c = 0;
    }
    if (d && threadIdx.x < kFusedWaveCtrs + 1) d[kFusedLine * threadIdx.x] = 0;   // a fused launch's slot
    if (d && threadIdx.x < 2) d[1 + threadIdx.x] = 0;
}

// The rotor azimuths (psi_mr, psi_tr): their rates are the constants Omega (helicopter_dynamics.py:
// 257-258, :288-289), so RK4 adds dt/6 (O + 2 O + 2 O + O) = dt Omega (f_dpsi) per step, and
// step_after wraps them to [-pi, pi) (:74-75).  The step kernel does not carry them; these are the
// same fp32 operations it performed on them when they were part of its state, so an azimuth
// reconstructed from its record is bitwise the one the step would have carried.
__device__ __forceinline__ float az_wrap(float x) { return in_pi_range(x) ? x : hg::pi_bound(x); }

// The azimuths of an env now, from its record, its counters and its reset template's azimuths
// (t_mr, t_tr): an episode the record belongs to advances from it, any later episode (begun by an
// in-kernel auto-reset) from the template at its step 0.
__device__ float2 az_now(const AzRec& r, int32_t step, int32_t epi, float t_mr, float t_tr, float d_mr, float d_tr) {
    const int32_t n = hgk::episode_steps(step);
    float a = t_mr, b = t_tr;
    int32_t k = n;
    if (epi == r.epi0 && n >= r.step0) {
        a = r.mr;
        b = r.tr;
        k = n - r.step0;
    }
    for (int32_t j = 0; j < k; ++j) {
        a = az_wrap(a + d_mr);
        b = az_wrap(b + d_tr);
    }
    return make_float2(a, b);
}

// the reset template's azimuths of env i: the shared template, or the env's own ([N][39])
__device__ __forceinline__ const float* az_template(const Template<float>* T, const float* tmpl_env, int64_t i) {
    return tmpl_env ? tmpl_env + i * kTplFloats + hgk::kAzCol0 : T->heli + hgk::kAzCol0;
}

// Heli.reset for masked envs (helicopter.py:208-217)
__global__ __launch_bounds__(kBlock) void reset_kernel(const Template<float> T, const float* tmpl_env, float* state,
                                                       AzRec* az, const uint8_t* mask, float* obs, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    if (mask && !mask[i]) return;
    // the shared template, or this env's own ([N][39] = heli 18 | carry 4 | obs 17)
    const float* tr = tmpl_env ? tmpl_env + i * kTplFloats : reinterpret_cast<const float*>(&T);
#pragma unroll
    for (int c = 0; c < 18; ++c)
        if (hgk::has_slot(c)) state[tix(i, c)] = tr[c];
#pragma unroll
    for (int c = 0; c < 5; ++c) state[tix(i, 18 + c)] = 0.f;
#pragma unroll
    for (int c = 0; c < 4; ++c) state[tix(i, 23 + c)] = tr[18 + c];
    int32_t* ctr = reinterpret_cast<int32_t*>(state);
    ctr[tix(i, kCtrCol0 + 0)] = 0;
    ctr[tix(i, kCtrCol0 + 1)] = 0;
    const int32_t epi = ctr[tix(i, kCtrCol0 + 2)] + 1;
    ctr[tix(i, kCtrCol0 + 2)] = epi;
    az[i] = AzRec{tr[hgk::kAzCol0], tr[hgk::kAzCol0 + 1], 0, epi};
    if (obs) {
#pragma unroll
        for (int c = 0; c < 17; ++c) obs[i * 17 + c] = tr[22 + c];
    }
}

// every slot of every tile, the padding of a ragged last tile included (its lanes step like the
// others and store nothing); the azimuth record of every env
__global__ __launch_bounds__(kBlock) void init_kernel(const Template<float> T, float* state, int64_t slots, AzRec* az,
                                                      int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= slots) return;
    for (int c = 0; c < 18; ++c)
        if (hgk::has_slot(c)) state[tix(i, c)] = T.heli[c];
    for (int c = 0; c < 5; ++c) state[tix(i, 18 + c)] = 0.f;
    for (int c = 0; c < 4; ++c) state[tix(i, 23 + c)] = T.carry[c];
    int32_t* ctr = reinterpret_cast<int32_t*>(state);
    for (int c = 0; c < 3; ++c) ctr[tix(i, kCtrCol0 + c)] = 0;
    if (i < n) az[i] = AzRec{T.heli[hgk::kAzCol0], T.heli[hgk::kAzCol0 + 1], 0, 0};
}

// tiles -> [N, 27] state / [N, 3] counter records (get_state); the azimuths reconstructed, the step
// counter of an env waiting for its next-step reset exported as -1.  The reconstruction replays one
// add-and-wrap per step since the record's anchor, so the record is re-anchored at the values it
// returns: a later read replays only the steps taken since this one (bitwise the same values)
__global__ __launch_bounds__(kBlock) void get_rows_kernel(const uint32_t* tiles, AzRec* az,
                                                          const Template<float>* T, const float* tmpl_env,
                                                          const Params<float>* P, uint32_t* state_rows,
                                                          int32_t* counter_rows, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const int32_t* ctr = reinterpret_cast<const int32_t*>(tiles);
    const int32_t step = ctr[tix(i, kCtrCol0 + 0)], epi = ctr[tix(i, kCtrCol0 + 2)];
    if (state_rows) {
        for (int c = 0; c < kStateCols; ++c)
            if (hgk::has_slot(c)) state_rows[i * kStateCols + c] = tiles[tix(i, c)];
        const float* ta = az_template(T, tmpl_env, i);
        const float2 a = az_now(az[i], step, epi, ta[0], ta[1], P->f_dpsi_mr, P->f_dpsi_tr);
        state_rows[i * kStateCols + hgk::kAzCol0] = __float_as_uint(a.x);
        state_rows[i * kStateCols + hgk::kAzCol0 + 1] = __float_as_uint(a.y);
        az[i] = AzRec{a.x, a.y, hgk::episode_steps(step), epi};
    }
    if (counter_rows) {
        counter_rows[i * kCtrCols + 0] = step < 0 ? -1 : step;
        counter_rows[i * kCtrCols + 1] = ctr[tix(i, kCtrCol0 + 1)];
        counter_rows[i * kCtrCols + 2] = epi;
    }
}

// [N, 27] / [N, 3] records -> tiles (set_state; either may be NULL): the azimuth record is rewritten
// at the env's (new) counters, with the given azimuths or the current ones (both NULL: the
// azimuths are re-anchored in place, before a reset template changes)
__global__ __launch_bounds__(kBlock) void set_rows_kernel(uint32_t* tiles, AzRec* az, const Template<float>* T,
                                                          const float* tmpl_env, const Params<float>* P,
                                                          const uint32_t* state_rows, const int32_t* counter_rows,
                                                          int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    int32_t* ctr = reinterpret_cast<int32_t*>(tiles);
    int32_t step = ctr[tix(i, kCtrCol0 + 0)], epi = ctr[tix(i, kCtrCol0 + 2)];
    float2 a;
    if (state_rows) {
        a = make_float2(__uint_as_float(state_rows[i * kStateCols + hgk::kAzCol0]),
                        __uint_as_float(state_rows[i * kStateCols + hgk::kAzCol0 + 1]));
        for (int c = 0; c < kStateCols; ++c)
            if (hgk::has_slot(c)) tiles[tix(i, c)] = state_rows[i * kStateCols + c];
    } else {
        const float* ta = az_template(T, tmpl_env, i);
        a = az_now(az[i], step, epi, ta[0], ta[1], P->f_dpsi_mr, P->f_dpsi_tr);
    }
    if (counter_rows) {
        step = counter_rows[i * kCtrCols + 0];
        epi = counter_rows[i * kCtrCols + 2];
        ctr[tix(i, kCtrCol0 + 0)] = step;
        ctr[tix(i, kCtrCol0 + 1)] = counter_rows[i * kCtrCols + 1];
        ctr[tix(i, kCtrCol0 + 2)] = epi;
    }
    az[i] = AzRec{a.x, a.y, hgk::episode_steps(step), epi};
}

__global__ __launch_bounds__(kBlock) void random_actions_kernel(float* act, int64_t n, int64_t env_offset,
                                                                uint64_t seed, uint64_t step, float lo, float hi) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const uint64_t gid = (uint64_t)(env_offset + i);
    const U4 r = philox(U4{(uint32_t)gid, (uint32_t)(gid >> 32), (uint32_t)step, (uint32_t)(step >> 32)},
                        (uint32_t)seed ^ 0xA511E9B3u, (uint32_t)(seed >> 32) ^ 0x63D83595u);
    const float w = hi - lo;
    reinterpret_cast<float4*>(act)[i] =
        make_float4(lo + w * u01(r.x), lo + w * u01(r.y), lo + w * u01(r.z), lo + w * u01(r.w));
}

// hg_debug_eta: the turbulence noise each env's next in-kernel step draws (wind_dynamics.py:49-52), from
// its counters (episode step, episode index) in the state tile -- the same function (draw_eta<false>)
// with the same key, so a step with these normals injected is bitwise the in-kernel step.
__global__ __launch_bounds__(kBlock) void eta_kernel(const float* state, int64_t n, uint64_t seed, int64_t env_offset,
                                                     const Params<float>* P, float* out) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const int32_t* ctr = reinterpret_cast<const int32_t*>(state);
    StepArgs a;   // (read only by the injected-noise form)
    a.eta = nullptr;
    float eta[3];
    draw_eta<false>(a, seed, env_offset, *P, 0, i, 0u, ctr[tix(i, kCtrCol0 + 0)], ctr[tix(i, kCtrCol0 + 2)], eta);
    out[3 * i + 0] = eta[0];
    out[3 * i + 1] = eta[1];
    out[3 * i + 2] = eta[2];
}

// hg_debug_philox: the device Philox4x32-10 on given counters and keys, rows {c0, c1, c2, c3, k0, k1}
__global__ __launch_bounds__(kBlock) void philox_kernel(const uint32_t* in, uint32_t* out, int64_t count) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= count) return;
    const uint32_t* r = in + 6 * i;
    const U4 o = philox(U4{r[0], r[1], r[2], r[3]}, r[4], r[5]);
    out[4 * i + 0] = o.x;
    out[4 * i + 1] = o.y;
    out[4 * i + 2] = o.z;
    out[4 * i + 3] = o.w;
}

// ------------------------------------------------------------------------------ host model

constexpr double kD2R = 3.14159265358979323846 / 180.0;

// First n at which the reference's float accumulator crosses its threshold
// (helicopter.py:193 `time_counter += DT` vs `> max_time`; :205 `successed_time += DT` vs `>=`).
int32_t first_step_above(double dt, double thr, bool strict) {
    double t = 0.0;
    int64_t k = 0;
    while (k < (int64_t)2000000000) {
        if (strict ? (t > thr) : (t >= thr)) return (int32_t)k;
        t += dt;
        ++k;
    }
    return INT32_MAX;
}

template <typename R>
Params<R> derive(const hg_config& c, int rows, int cols) {
    const hg_airframe& a = c.af;
    Params<R> P;
    memset(&P, 0, sizeof(P));
    const double dt = c.dt;
    P.dt = (R)dt;
    P.half_dt = (R)(0.5 * dt);
    P.dt6 = (R)(0.16666666666666666 * dt);
    // helicopter_dynamics.py:414-422
    P.coll0 = (R)(kD2R * (a.COL_OS + 0.5 * (a.COL_H + a.COL_L)));
    P.coll1 = (R)(kD2R * 0.5 * (a.COL_H - a.COL_L));
    P.lon0 = (R)(kD2R * 0.5 * (a.LON_H + a.LON_L));
    P.lon1 = (R)(kD2R * 0.5 * (a.LON_H - a.LON_L));
    P.lat0 = (R)(kD2R * 0.5 * (a.LAT_H + a.LAT_L));
    P.lat1 = (R)(kD2R * 0.5 * (a.LAT_H - a.LAT_L));
    P.ped0 = (R)(kD2R * (a.PED_OS + 0.5 * (a.PED_H + a.PED_L)));
    P.ped1 = (R)(kD2R * 0.5 * (a.PED_H - a.PED_L));
    // :160-165
    P.lapse_t0 = (R)(a.env_LAPSE / a.env_T0);
    P.ro_sea = (R)a.env_RO_SEA;
    P.rho_exp = (R)(a.env_GRAV / (a.env_LAPSE * a.env_R) - 1.0);
    // :107-154
    const double mass = a.WT / a.env_GRAV;
    P.wt = (R)a.WT;
    P.inv_mass = (R)(1.0 / mass);
    P.p_loss = (R)(550.0 * a.HP_LOSS);
    P.vtrans = (R)a.VTRANS;
    P.wl_cg_ft = (R)(a.WL_CG / 12.0);
    const double mr_H = (a.mr_WL - a.WL_CG) / 12, mr_D = (a.mr_FS - a.FS_CG) / 12;
    const double fus_H = (a.fus_WL - a.WL_CG) / 12, fus_D = (a.fus_FS - a.FS_CG) / 12;
    const double ht_H = (a.ht_WL - a.WL_CG) / 12, ht_D = (a.ht_FS - a.FS_CG) / 12;
    const double vt_H = (a.vt_WL - a.WL_CG) / 12, vt_D = (a.vt_FS - a.FS_CG) / 12;
    const double tr_H = (a.tr_WL - a.WL_CG) / 12, tr_D = (a.tr_FS - a.FS_CG) / 12;
    const double mr_OM = a.mr_RPM * 2 * M_PI / 60, mr_VT = a.mr_R * mr_OM;
    const double mr_FR = a.mr_CD0 * a.mr_R * a.mr_B * a.mr_C;
    const double mr_SOL = a.mr_B * a.mr_C / (a.mr_R * M_PI);
    const double mr_ASIG = a.mr_A * mr_SOL;
    P.mr_H = (R)mr_H; P.mr_D = (R)mr_D; P.mr_IS = (R)a.mr_IS; P.mr_K1 = (R)a.mr_K1; P.mr_R = (R)a.mr_R;
    P.mr_OMEGA = (R)mr_OM; P.mr_inv_OMEGA = (R)(1.0 / mr_OM);
    P.mr_VTIP = (R)mr_VT; P.mr_inv_VTIP = (R)(1.0 / mr_VT);
    P.mr_tw75 = (R)(0.75 * a.mr_TWST); P.mr_tw50 = (R)(0.5 * a.mr_TWST);
    P.mr_two3_vtip = (R)(0.66667 * mr_VT);
    const double gam_dro = a.mr_A * a.mr_C * pow(a.mr_R, 4) / a.mr_IB * mr_OM / 16 * (1 + 8.0 / 3 * a.mr_E / a.mr_R);
    P.mr_gam_dro = (R)gam_dro;
    P.mr_inv_gam_dro = (R)(1.0 / gam_dro);
    P.mr_kc_num = (R)(0.75 * mr_OM * a.mr_E / a.mr_R);
    P.mr_DL_DB1 = (R)(a.mr_B / 2 * (1.5 * a.mr_IB * a.mr_E / a.mr_R * mr_OM * mr_OM));
    P.mr_DL_DA1_dro = (R)(0.5 * a.mr_A * a.mr_B * a.mr_C * a.mr_R * mr_VT * mr_VT * a.mr_E / 6);
    P.mr_coef = (R)(0.25 * mr_VT * a.mr_R * a.mr_A * a.mr_B * a.mr_C);
    P.mr_inflow = (R)(0.75 * M_PI / a.mr_R);
    P.mr_inv_thr_den = (R)(1.0 / (2 * M_PI * a.mr_R * a.mr_R));
    P.mr_inv_ct_den = (R)(1.0 / (M_PI * a.mr_R * a.mr_R * mr_VT * mr_VT));
    P.mr_prof = (R)(0.5 * (mr_FR / 4) * mr_VT);
    P.mr_vtip2 = (R)(mr_VT * mr_VT);
    P.mr_2_vtip = (R)(2.0 / mr_VT);
    P.mr_8_asig = (R)(8.0 / mr_ASIG);
    P.mr_inv_R = (R)(1.0 / a.mr_R);
    const double tr_OM = a.tr_RPM * 2 * M_PI / 60, tr_VT = a.tr_R * tr_OM;
    P.tr_H = (R)tr_H; P.tr_D = (R)tr_D; P.tr_OMEGA = (R)tr_OM;
    P.tr_VTIP = (R)tr_VT; P.tr_inv_VTIP = (R)(1.0 / tr_VT);
    P.tr_tw75 = (R)(0.75 * a.tr_TWST); P.tr_tw50 = (R)(0.5 * a.tr_TWST);
    P.tr_two3_vtip = (R)(0.66667 * tr_VT);
    P.tr_coef = (R)(0.25 * tr_VT * a.tr_R * a.tr_A * a.tr_B * a.tr_C);
    P.tr_inflow = (R)(0.5 * 0.75 * M_PI / a.tr_R);   // :285 halves the TR inflow rate
    P.tr_inv_thr_den = (R)(1.0 / (2 * M_PI * a.tr_R * a.tr_R));
    P.fus_H = (R)fus_H; P.fus_XUU = (R)a.fus_XUU; P.fus_YVV = (R)a.fus_YVV; P.fus_ZWW = (R)a.fus_ZWW;
    P.fus_COR = (R)a.fus_COR; P.fus_dfw_k = (R)(mr_H - fus_H); P.fus_dfw_c = (R)(fus_D - mr_D);
    P.ht_D = (R)ht_D; P.ht_ZUU = (R)a.ht_ZUU; P.ht_ZUW = (R)a.ht_ZUW; P.ht_ZMAX = (R)a.ht_ZMAX;
    P.ht_dw_k = (R)(mr_H - ht_H); P.ht_dw_c = (R)(ht_D - mr_D - a.mr_R);
    P.vt_H = (R)vt_H; P.vt_D = (R)vt_D; P.vt_YUU = (R)a.vt_YUU; P.vt_YUV = (R)a.vt_YUV; P.vt_YMAX = (R)a.vt_YMAX;
    P.wn_ZUU = (R)a.wn_ZUU; P.wn_ZUW = (R)a.wn_ZUW; P.wn_ZMAX = (R)a.wn_ZMAX;
    P.wn_on = a.wn_ZUW != 0.0;   // :367
    P.lg_K = (R)a.lg_K; P.lg_C = (R)a.lg_C;
    const double loc[3][3] = {{-(a.lg_FS_N - a.FS_CG), 0.0, -(a.lg_WL - a.WL_CG)},
                              {-(a.lg_FS_MN - a.FS_CG), a.lg_BL_MN, -(a.lg_WL - a.WL_CG)},
                              {-(a.lg_FS_MN - a.FS_CG), -a.lg_BL_MN, -(a.lg_WL - a.WL_CG)}};
    // The lone-wave kernels' gear (stage_f32.h gear_add, HG_GEAR_FACTORED 3) reads only lg_loc[0][0],
    // [1][0], [1][1] and [0][2]: it relies on this layout -- the nose wheel on the centre line, the
    // mains mirrored about it, all three on one waterline -- which the reference's geometry always
    // has (helicopter_dynamics.py:123-126).  hg_create checks it (gear_layout_ok) before any step.
    for (int g = 0; g < 3; ++g)
        for (int j = 0; j < 3; ++j) P.lg_loc[g][j] = (R)(loc[g][j] / 12.0);   // :123-126
    double reach = 0;
    for (int g = 0; g < 3; ++g)
        reach = fmax(reach, sqrt(loc[g][0] * loc[g][0] + loc[g][1] * loc[g][1] + loc[g][2] * loc[g][2]) / 12.0);
    P.lg_reach = (R)(reach * 1.001 + 1e-3);
    // inertia and inverse (:151-154)
    const double Ix = a.IX, Iy = a.IY, Iz = a.IZ, Ixz = -a.IXZ;
    const double det = Ix * Iz - Ixz * Ixz;
    P.Ixx = (R)Ix; P.Iyy = (R)Iy; P.Izz = (R)Iz; P.Ixz = (R)Ixz;
    P.Ji00 = (R)(Iz / det); P.Ji02 = (R)(-Ixz / det); P.Ji11 = (R)(1.0 / Iy);
    P.Ji20 = (R)(-Ixz / det); P.Ji22 = (R)(Ix / det);
    // terrain (:167-172)
    P.hm_sx = (R)(rows / a.env_NS_MAX);
    P.hm_sy = (R)(cols / a.env_EW_MAX);
    P.hm_cx = (R)(rows / 2);
    P.hm_cy = (R)(cols / 2);
    P.hm_rows = rows;
    P.hm_cols = cols;
    P.ns_half = (R)(a.env_NS_MAX / 2);
    P.ew_half = (R)(a.env_EW_MAX / 2);
    // wind (wind_dynamics.py:21-28, 56)
    const double wdir = a.env_WIND_DIR_deg * kD2R;
    P.wm[0] = (R)(a.env_WIND_SPD * (double)(float)cos(wdir));
    P.wm[1] = (R)(a.env_WIND_SPD * (double)(float)sin(wdir));
    P.wm[2] = (R)0;
    P.wind_dir_cos = (R)cos(wdir);
    P.wind_dir_sin = (R)sin(wdir);
    const double w20 = a.env_TURB_LVL / 7.0 * 88.61;
    P.w20 = (R)w20;
    P.sigma_low = (R)(0.1 * w20);
    P.turb_level = (R)a.env_TURB_LVL;
    hg::tep_row_values(P.turb_level, P.tep_row);
    P.eta_norm = (R)(1.0 / sqrt(dt));
    // folded constants of the packed fp32 step (stage_f32.h), formed in double
    P.f_kc_irho = (R)(0.75 * mr_OM * a.mr_E / a.mr_R / gam_dro);
    P.f_og_irho = (R)(mr_OM / gam_dro);
    P.f_mr_inflow_thr = (R)(0.75 * M_PI / a.mr_R * (0.25 * mr_VT * a.mr_R * a.mr_A * a.mr_B * a.mr_C) /
                            (2 * M_PI * a.mr_R * a.mr_R));
    P.f_tr_inflow_thr = (R)(0.5 * 0.75 * M_PI / a.tr_R * (0.25 * tr_VT * a.tr_R * a.tr_A * a.tr_B * a.tr_C) /
                            (2 * M_PI * a.tr_R * a.tr_R));
    P.f_mr_ct_k = (R)((0.25 * mr_VT * a.mr_R * a.mr_A * a.mr_B * a.mr_C) / (M_PI * a.mr_R * a.mr_R * mr_VT * mr_VT));
    P.f_mr_db_a = (R)(2.0 / mr_VT * 8.0 / mr_ASIG);
    P.f_mr_db_b = (R)(0.5 * (2.0 / mr_VT) * (2.0 / mr_VT));
    P.f_hXUU = (R)(0.5 * a.fus_XUU);
    P.f_hYVV = (R)(0.5 * a.fus_YVV);
    P.f_hZWW = (R)(0.5 * a.fus_ZWW);
    P.f_zd = (R)(-0.5 * a.fus_ZWW * a.fus_COR);
    P.f_m2_R = (R)(-2.0 / a.mr_R);
    P.f_rho_lz = (R)((a.env_GRAV / (a.env_LAPSE * a.env_R) - 1.0) * a.env_LAPSE / a.env_T0);
    {   // gyroscopic coefficients (stage_f32.h): g = M - pqr x I pqr, (p', q', r') = I^-1 g
        const double J00 = Iz / det, J02 = -Ixz / det, J20 = -Ixz / det, J22 = Ix / det, J11 = 1.0 / Iy;
        P.f_gyro[0] = (R)(-(J00 * Ixz + J02 * (Iy - Ix)));   // p' per pq
        P.f_gyro[1] = (R)(-(J20 * Ixz + J22 * (Iy - Ix)));   // r' per pq
        P.f_gyro[2] = (R)(-(J00 * (Iz - Iy) - J02 * Ixz));  // p' per qr
        P.f_gyro[3] = (R)(-(J20 * (Iz - Iy) - J22 * Ixz));  // r' per qr
        P.f_gyro[4] = (R)(-J11 * (Ix - Iz));                 // q' per pr
        P.f_gyro[5] = (R)(-J11 * Ixz);                       // q' per r^2 - p^2
    }
    P.f_dpsi_mr = (R)(dt * mr_OM);
    P.f_dpsi_tr = (R)(dt * tr_OM);
    // task (helicopter.py:63-68, helicopter_with_tasks.py:33, 87-88)
    const double n_t = sqrt(2 * a.mr_R / a.env_GRAV), n_x = 2 * a.mr_R, n_v = sqrt(2 * a.mr_R * a.env_GRAV);
    P.n_t = (R)n_t; P.n_t2 = (R)(n_t * n_t);
    P.inv_n_x = (R)(1.0 / n_x); P.inv_n_v = (R)(1.0 / n_v); P.inv_n_a = (R)(1.0 / a.env_GRAV);
    P.tgt_n[0] = (R)(c.target.north_loc / n_x);
    P.tgt_n[1] = (R)(c.target.east_loc / n_x);
    P.tgt_n[2] = (R)(-c.target.sea_alt / n_x);
    P.vel_tgt_n = (R)(c.target.vel / n_v);
    P.dwn_tgt_n = (R)(-c.target.sea_alt / n_x);
    P.fail_zdot = (R)(mr_VT * 0.05);
    P.fail_ang = (R)(60 * kD2R);
    P.task = c.task;
    P.time_up_steps = first_step_above(dt, c.max_time, true);
    P.success_steps = first_step_above(dt, c.max_time / 4, false);
    P.autoreset = c.autoreset ? 1 : 0;
    // RETRIM: every step records its wind (the trim wind of a later reset: an auto-reset in the
    // kernel, or hg_reset -- the single-env drop-in, whose reset() the caller issues)
    P.reset_retrim = (c.reset_mode == HG_RESET_RETRIM) ? 1 : 0;
    P.autoreset_next = (c.autoreset && c.autoreset_mode == HG_AUTORESET_NEXT_STEP) ? 1 : 0;
    P.max_episode_steps = (c.max_episode_steps > 0 && c.max_episode_steps < INT32_MAX) ? (int32_t)c.max_episode_steps
                                                                                        : INT32_MAX;
    return P;
}

// Trim setup for a condition (helicopter_dynamics.py:498-516): the fixed state entries, targets
// and initial guess; the ground under the trim position comes from the host copy of the terrain.
hg::TrimSetup trim_setup(const Params<double>& P, const float2* hmap, const hg_trim_cond& tc) {
    hg::TrimSetup t;
    memset(&t, 0, sizeof(t));
    t.piv[0][0] = -1;   // no pivot order (build_template records the env condition's)
    t.base[14] = (float)tc.yaw;
    t.base[2] = (float)tc.psi_mr;
    t.base[3] = (float)tc.psi_tr;
    t.base[15] = (float)tc.xy[0];
    t.base[16] = (float)tc.xy[1];
    t.hc = hg::ground_height(P, hmap, t.base[15], t.base[16]);
    t.base[17] = (float)(-(t.hc.h() + P.wl_cg_ft) - tc.gr_alt);
    t.yt[12] = (float)tc.yaw_rate;
    for (int i = 0; i < 3; ++i) t.yt[13 + i] = (float)tc.ned_vel[i] / (float)P.mr_R;
    const double x0[16] = {0.05f, 0.05f, 0, 0, 0, 0, 0, 0, 0, (float)tc.yaw_rate, -0.01f, 0.01f, 0, 0, 0, 0};
    for (int i = 0; i < 16; ++i) t.x0[i] = x0[i];
    for (int i = 0; i < 3; ++i) t.x0[4 + i] = (float)tc.ned_vel[i] / (float)P.mr_VTIP;
    hg::trim_precompute(P, t);
    return t;
}

// HelicopterDynamics.trim (helicopter_dynamics.py:491-555), serial: fp64 Newton with a central-
// difference Jacobian and step halving, the reference's iteration logic.
// piv_rec (4 x 16, optional): the pivot order of each of the first four Newton solves (hg::TrimSetup::piv;
// the later entries repeat the last solve's, and stay untouched when the trim took no Newton step).
int32_t do_trim(const Params<double>& P, const float2* hmap, const hg_trim_cond& tc, const double W[3],
                hg_trim_result* out, double* jac_rec = nullptr, int32_t jac_max = 0, int32_t* jac_n = nullptr,
                int8_t* piv_rec = nullptr) {
    const hg::TrimSetup T = trim_setup(P, hmap, tc);
    const double eps = hg::kTrimEps;
    double x[16], y[16];
    memcpy(x, T.x0, sizeof(x));
    hg::trim_fcn(P, T, x, W, y, nullptr, nullptr, nullptr);
    double tol = hg::trim_residual(y, T.yt);
    int it = 0, nsolve = 0;
    while (tol > eps) {
        double J[16][16], yp[16], ym[16], xp[16], xm[16], r[16], dir[16];
        for (int i = 0; i < 16; ++i) {
            memcpy(xp, x, sizeof(x));
            memcpy(xm, x, sizeof(x));
            xp[i] += eps;
            xm[i] -= eps;
            hg::trim_fcn(P, T, xp, W, yp, nullptr, nullptr, nullptr);
            hg::trim_fcn(P, T, xm, W, ym, nullptr, nullptr, nullptr);
            for (int k = 0; k < 16; ++k) J[k][i] = (yp[k] - ym[k]) / (2 * eps);
        }
        if (jac_rec && jac_n && *jac_n < jac_max) {   // (hg_debug_trim_jacobians)
            memcpy(jac_rec + (size_t)(*jac_n) * 256, J, sizeof(J));
            ++*jac_n;
        }
        for (int k = 0; k < 16; ++k) r[k] = y[k] - T.yt[k];
        int8_t piv[16];
        if (!hg::solve16(J, r, dir, piv)) return fail(HG_E_TRIM, "trim: singular Jacobian");
        if (piv_rec)
            for (int k = nsolve; k < 4; ++k) memcpy(piv_rec + 16 * k, piv, 16);   // later steps: this order
        ++nsolve;
        double step = 1.0, xn[16], yn[16], tn = 0;
        int j;
        for (j = 0; j < hg::kTrimLineSearch; ++j) {
            for (int k = 0; k < 16; ++k) xn[k] = x[k] - step * dir[k];
            hg::trim_fcn(P, T, xn, W, yn, nullptr, nullptr, nullptr);
            tn = hg::trim_residual(yn, T.yt);
            step *= 0.5;
            if (tn < tol) break;
        }
        if (j >= hg::kTrimLineSearch - 1) break;   // :540
        memcpy(x, xn, sizeof(x));
        memcpy(y, yn, sizeof(y));
        tol = tn;
        if (++it > hg::kTrimMaxIter) return fail(HG_E_TRIM, "Trim failed, please try a better trim condition!");
    }
    hg::trim_fcn(P, T, x, W, y, out->state, out->state_dots, out->obs);
    for (int i = 0; i < 4; ++i) out->action[i] = x[12 + i];
    out->residual = tol;
    out->iterations = it;
    const hg::Ground<double> h_post = hg::ground_height(P, hmap, out->state[15], out->state[16]);
    out->failed = hg::is_failed(P, out->state, out->state_dots, h_post) ? 1 : 0;
    return HG_OK;
}

int32_t check_config(const hg_config* c, int32_t rows, int32_t cols) {
    if (!c) return fail(HG_E_INVALID, "config is NULL");
    if (!(c->dt > 0) || !std::isfinite(c->dt)) return fail(HG_E_INVALID, "dt must be > 0");
    if (!(c->max_time > 0)) return fail(HG_E_INVALID, "max_time must be > 0");
    if (c->task < HG_TASK_HELI || c->task > HG_TASK_FORWARD_FLIGHT) return fail(HG_E_INVALID, "bad task");
    if (c->af.env_TURB_LVL < 0 || c->af.env_TURB_LVL > 7) return fail(HG_E_INVALID, "TURB_LVL must be 0..7");
    if (c->reset_mode != HG_RESET_TEMPLATE && c->reset_mode != HG_RESET_RETRIM)
        return fail(HG_E_INVALID, "reset_mode must be HG_RESET_TEMPLATE or HG_RESET_RETRIM");
    if (c->autoreset_mode != HG_AUTORESET_SAME_STEP && c->autoreset_mode != HG_AUTORESET_NEXT_STEP)
        return fail(HG_E_INVALID, "autoreset_mode must be HG_AUTORESET_SAME_STEP or HG_AUTORESET_NEXT_STEP");
    if (c->max_episode_steps < 0) return fail(HG_E_INVALID, "max_episode_steps must be >= 0");
    if (rows < 2 || cols < 2 || rows != cols)
        return fail(HG_E_INVALID, "terrain must be a square map of at least 2x2 samples");
    return HG_OK;
}

}  // namespace

// ------------------------------------------------------------------------------ handle

// Counter rings (hg_step_chained's reset count, the re-trim job count): a step counts into its slot
// and its kernel zeroes the next step's.  A launch may skip zeroing its own slot only when the
// previous step launch was a chained one of the same sequence: both eager, or both captured into the
// same graph (a graph's first step keeps its memset, so every replay starts from a zeroed slot).
constexpr uint64_t kChainBroken = ~0ull;
static hipError_t chain_key(hipStream_t s, uint64_t* key) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    unsigned long long id = 0;
    const hipError_t err = hipStreamGetCaptureInfo(s, &cs, &id);
    *key = cs == hipStreamCaptureStatusNone ? 0ull : (id | (1ull << 63));
    return err;
}

struct hg_env {
    hg_config cfg;
    int device = 0;                          // the HIP device the handle's memory lives on
    int64_t n = 0;
    int rows = 0, cols = 0;
    std::vector<float2> hmap_host;   // {hi, lo} split of the fp64 heights
    float2* hmap = nullptr;
    float* state = nullptr;                 // wave tiles (retrim.h tix): state columns + counters
    AzRec* az = nullptr;                    // rotor azimuth records [N] (retrim.h AzRec)
    Params<float> Pf;
    Params<double> Pd;
    Template<float> tmpl;
    Template<float>* tmpl_dev = nullptr;
    Params<float>* params_dev = nullptr;
    hg_trim_result trim;
    int64_t resident_envs = 0;   // one wave per SIMD on this device: 64 lanes x 4 SIMDs x CUs
    hg::TrimSetup setup;                    // trim condition -> Newton setup (host copy)
    hg::TrimSetup* setup_dev = nullptr;     // ... and device copy (re-trim kernel)
    Params<double>* pd_dev = nullptr;       // fp64 model constants for the re-trim kernel
    // one allocation (trim_block, one page) holds the re-trim job-count ring and counters, the trim
    // setup and the fp64 constants (placed there to keep the trims' first loads on a page the step
    // kernel's count atomics touch; no measurable change in the start-up, scripts/retrim_startup.py)
    void* trim_block = nullptr;
    float* retrim_wind = nullptr;           // reset_mode RETRIM work buffers
    int32_t* retrim_list = nullptr;         // hg_reset's masked envs (their winds by env)
    int4* retrim_recs = nullptr;            // a step's auto-reset jobs {env, wind}
    int32_t* retrim_count = nullptr;        // [0] jobs of hg_reset's re-trim, [1] failures so far, [2] invalid jobs,
                                            // [3] solves tried with the given pivot order, [4] of them rejected
    int32_t* fused_ring = nullptr;          // [3][kFusedSlot] a fused same-step launch's counters, by the same slot
    int32_t* retrim_ring = nullptr;         // [3] jobs of a step's re-trim: step k counts into [k % 3] and
    uint64_t retrim_gen = 0;                //     zeroes [(k + 1) % 3] from its kernel (no memset launch)
    uint64_t retrim_chain = kChainBroken;   // chain key of the previous re-trim step (see chain_key)
    // ov mode (reset_mode RETRIM with next-step auto-reset): the episodes a step ends are re-trimmed
    // while the next step runs.  Step k queues its ends into ov_recs[k % 3] / ov_ring[k % 3]; step k+1
    // is one launch of step_ov_kernel holding their trims and the step, whose due resets store only
    // their step counter (the trims write the rest, and their observation rows).
    bool ov = false;                        // configured (RETRIM + next-step auto-reset) and enabled
    bool ov_enabled = true;                 // hg_set_retrim_overlap
    bool fused_enabled = false;             // hg_set_retrim_overlap(2): the fused same-step launch
    uint64_t ov_chain = kChainBroken;       // chain key of the previous step when its ends can be trimmed
                                            // concurrently with this one (no other call in between)
    int4* ov_recs = nullptr;                // [3][N] jobs {env, trim wind}
    int32_t* ov_ring = nullptr;             // [3] their counts
    float* tmpl_env = nullptr;              // per-env reset templates [N][39] (hg_set_reset_templates)
    bool env_templates = false;
    bool baked = false;                     // step with the constant-specialised kernel (baked.h)
    bool baked_allowed = true;              // ... unless switched off (hg_set_specialized)
    // a run-time specialised code object for another airframe (step_rtc.hip, hg_load_specialized)
    hipModule_t rtc_mod = nullptr;
    hipFunction_t rtc_fn[6] = {};           // nt, nt_feat, nts, nts_feat, bulk, bulk_feat
    Params<float> rtc_image;                // the constant image it was built with
    int32_t rtc_task = -1;
    bool rtc = false;                       // in use: its image matches this env's constants
    hg::TrimSetup* setup_batch = nullptr;   // hg_trim_conds_batch scratch
    uint64_t chain_expect = kChainBroken;   // chain key of the previous step launch if it was a chained one
    bool ever_captured = false;             // a step was captured into a graph: replays the host cannot see may
                                            // leave any ring slot non-zero, so eager steps zero their own slot
    int64_t setup_batch_cap = 0;
    // launch counts (hg_debug_launches): step calls, steps holding overlapped re-trims, run-time
    // specialised / helper / lone-wave / bulk kernel launches
    mutable int64_t n_launch[6] = {0, 0, 0, 0, 0, 0};
};

// Every entry point that touches device memory runs on the handle's device (the caller's current
// device may be another one), and restores the caller's current device on return.
struct DevGuard {
    int prev = -1;
    bool ok = true;   // false: the handle's device could not be made current
    explicit DevGuard(const hg_env* e) {
        int cur = 0;
        if (!e || hipGetDevice(&cur) != hipSuccess || cur == e->device) return;
        if (hipSetDevice(e->device) == hipSuccess) prev = cur;
        else ok = false;
    }
    ~DevGuard() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

// The gear layout the lone-wave kernels' factored gear relies on (derive(), stage_f32.h gear_add):
// nose wheel on the centre line, mains mirrored about it, one waterline.
static bool gear_layout_ok(const Params<float>& P) {
    return P.lg_loc[0][1] == 0.f && P.lg_loc[2][0] == P.lg_loc[1][0] && P.lg_loc[2][1] == -P.lg_loc[1][1] &&
           P.lg_loc[1][2] == P.lg_loc[0][2] && P.lg_loc[2][2] == P.lg_loc[0][2];
}

// Model constants after a configuration change (create and the setters).
static void rederive(hg_env* e) {
    e->Pd = derive<double>(e->cfg, e->rows, e->cols);
    e->Pf = derive<float>(e->cfg, e->rows, e->cols);
    e->Pf.env_templates = e->env_templates ? 1 : 0;
    e->baked = e->baked_allowed && hg::bake_matches(e->Pf);
    e->rtc = !e->baked && e->baked_allowed && e->rtc_mod && e->rtc_task == e->cfg.task &&
             hg::bake_matches(e->Pf, e->rtc_image);
}

// Upload the fp32 model constants the step kernel reads (after create and every setter).
// Work already queued on any stream (including non-blocking ones) may still read the constants, so
// the device is drained first; the copy itself is synchronous.
static int32_t upload_params(hg_env* e) {
    if (!e->params_dev) return HG_OK;
    hipError_t err = hipDeviceSynchronize();
    if (err == hipSuccess) err = hipMemcpy(e->params_dev, &e->Pf, sizeof(e->Pf), hipMemcpyHostToDevice);
    if (err == hipSuccess && e->pd_dev) err = hipMemcpy(e->pd_dev, &e->Pd, sizeof(e->Pd), hipMemcpyHostToDevice);
    if (err != hipSuccess) return fail(HG_E_HIP, std::string("params upload: ") + hipGetErrorString(err));
    return HG_OK;
}

static inline unsigned grid_for(int64_t n);
// Re-anchor every env's azimuth record at its current counters (before a reset template changes:
// the records of episodes begun by an in-kernel reset point at the template).  Synchronous.
static hipError_t reanchor_azimuths(hg_env* e) {
    if (!e->az) return hipSuccess;
    hipLaunchKernelGGL(set_rows_kernel, dim3(grid_for(e->n)), dim3(kBlock), 0, 0, reinterpret_cast<uint32_t*>(e->state),
                       e->az, e->tmpl_dev, e->Pf.env_templates ? e->tmpl_env : nullptr,
                       (const Params<float>*)e->params_dev, nullptr, nullptr, e->n);
    hipError_t err = hipGetLastError();
    if (err == hipSuccess) err = hipDeviceSynchronize();
    return err;
}

static int32_t build_template(hg_env* e) {
    e->ov_chain = kChainBroken;   // the next step's pending resets take the serial re-trim
    const double W[3] = {e->Pd.wm[0], e->Pd.wm[1], e->Pd.wm[2]};   // helicopter.py:55 (mean wind)
    hg_trim_result r;
    memset(&r, 0, sizeof(r));
    int8_t piv[4][16];
    memset(piv, -1, sizeof(piv));
    const int32_t rc = do_trim(e->Pd, e->hmap_host.data(), e->cfg.trim, W, &r, nullptr, 0, nullptr, &piv[0][0]);
    if (rc != HG_OK) return rc;
    e->trim = r;
    for (int c = 0; c < 18; ++c) e->tmpl.heli[c] = (float)r.state[c];
    for (int c = 0; c < 17; ++c) e->tmpl.obs[c] = (float)r.obs[c];
    e->tmpl.carry[0] = (float)r.obs[4];
    e->tmpl.carry[1] = (float)r.obs[5];
    e->tmpl.carry[2] = (float)r.obs[6];
    e->tmpl.carry[3] = (float)r.obs[16];
    e->setup = trim_setup(e->Pd, e->hmap_host.data(), e->cfg.trim);
    memcpy(e->setup.piv, piv, sizeof(piv));   // the device trim's first-choice pivot order
    if (e->tmpl_dev) {   // device copies read by the step / re-trim kernels (after all queued work)
        hipError_t err = hipDeviceSynchronize();
        if (err == hipSuccess) err = reanchor_azimuths(e);   // (they may start from the old template's)
        if (err == hipSuccess) err = hipMemcpy(e->tmpl_dev, &e->tmpl, sizeof(e->tmpl), hipMemcpyHostToDevice);
        if (err == hipSuccess && e->setup_dev)
            err = hipMemcpy(e->setup_dev, &e->setup, sizeof(e->setup), hipMemcpyHostToDevice);
        if (err != hipSuccess) return fail(HG_E_HIP, std::string("template upload: ") + hipGetErrorString(err));
    }
    return HG_OK;
}

// pair (optional): a fused launch's {jobs, waves, claim}
static hipError_t zero_counts(int32_t* const p[3], hipStream_t s, int32_t* pair = nullptr) {
    if (!p[0] && !p[1] && !p[2] && !pair) return hipSuccess;
    hipLaunchKernelGGL(zero_counts_kernel, dim3(1), dim3(64), 0, s, p[0], p[1], p[2], pair);
    return hipGetLastError();
}

static inline unsigned grid_for(int64_t n) { return (unsigned)((n + kBlock - 1) / kBlock); }
// re-trim launches: one job per 64-lane block, at most HG_RETRIM_GRID blocks (jobs beyond loop)
#ifndef HG_RETRIM_GRID
#define HG_RETRIM_GRID 1024
#endif
static inline unsigned retrim_grid(int64_t jobs) {
    return (unsigned)(jobs < 1 ? 1 : (jobs > HG_RETRIM_GRID ? HG_RETRIM_GRID : jobs));
}

#define PARAM_ARG(e) ((const Params<float>*)(e)->params_dev)
// the step kernel's leading (preloaded) parameters
#define STEP_KARGS(e) (e)->state, (int64_t)(e)->n, (uint64_t)(e)->cfg.seed, (int64_t)(e)->cfg.env_offset, PARAM_ARG(e), \
                      (e)->tmpl_dev

// Occupancy of launches with more waves than SIMDs: three waves per SIMD (<= 168 VGPRs) at every
// size.  Until the azimuths left the stepped state, two waves per SIMD (a dynamic-LDS cap) were
// faster past 2 M envs, where the write-heavy HBM stream binds (4 M: 271 against 284 us); with the
// 28-word tile three are (4 M: 254.6 against 257.8 us, interleaved A/B), so the cap is gone.
template <int T, bool ETA, bool NT, bool FEAT, bool MULTI, bool BAKED, bool NTS = false>
static void launch_step(const hg_env* e, hipStream_t s, const StepArgs& a) {
#if HG_HELPER > 0
    if constexpr (NT && !ETA && !MULTI) if (e->n <= e->resident_envs / HG_HELPER_DIV) {
        const unsigned tiles = (unsigned)((e->n + 63) / 64);
        hipLaunchKernelGGL((step_help_kernel<T, FEAT, BAKED>), dim3((tiles + HG_HELPER - 1) / HG_HELPER),
                           dim3(128 * HG_HELPER), 0, s, STEP_KARGS(e), a);
        ++e->n_launch[3];
        return;
    }
#endif
    ++e->n_launch[NT ? 4 : 5];
    const unsigned grid = (unsigned)((e->n + kStepBlock - 1) / kStepBlock);
    hipLaunchKernelGGL((step_kernel<T, ETA, NT, FEAT, MULTI, BAKED, NTS>), dim3(grid), dim3(kStepBlock), 0, s,
                       STEP_KARGS(e), a);
}

// The step variant for a launch: NT (the lone-wave variant) while the batch fits two waves per SIMD;
// past it the bulk variant, whose per-step launches of the default airframe store their outputs
// non-temporally too up to four waves per SIMD (NTS: 196 608 envs 15.6 -> 14.7 us, 262 144 forward
// flight 20.1 -> 20.0 us; from 524 288 envs on, where the outputs of one step are read back by the
// next one through the Infinity Cache, plain stores are faster: 37.7 against 38.5 us, 1 M 67.1
// against 69.4 us); the default airframe's constant-specialised kernel (baked.h) when the env uses
// it; with or without the optional features.
// (returns the run-time specialised launch's status; the library's own launches report through
// hipGetLastError)
template <int T, bool MULTI>
static hipError_t dispatch_step(const hg_env* e, hipStream_t s, const StepArgs& a, bool eta, bool feat) {
    if (!MULTI && !eta && e->rtc) {   // the airframe's run-time specialised kernels, same size rules
        const int v = e->n <= HG_NT_WAVES * e->resident_envs ? 0 : (e->n <= HG_NTS_WAVES * e->resident_envs ? 2 : 4);
        float* state = e->state;
        int64_t n = e->n, off = (int64_t)e->cfg.env_offset;
        uint64_t seed = (uint64_t)e->cfg.seed;
        const Params<float>* pa = PARAM_ARG(e);
        const Template<float>* tp = e->tmpl_dev;
        StepArgs args = a;
        void* params[] = {&state, &n, &seed, &off, &pa, &tp, &args};
        const unsigned grid = (unsigned)((e->n + kStepBlock - 1) / kStepBlock);
        ++e->n_launch[2];
        return hipModuleLaunchKernel(e->rtc_fn[v + (feat ? 1 : 0)], grid, 1, 1, kStepBlock, 1, 1, 0, s, params, nullptr);
    }
    auto pick = [&](auto nt) {
        constexpr bool NT = decltype(nt)::value;
        if (e->baked) {
            if (!NT && !MULTI && e->n <= HG_NTS_WAVES * e->resident_envs) {
                if (feat) eta ? launch_step<T, true, false, true, false, true, true>(e, s, a) : launch_step<T, false, false, true, false, true, true>(e, s, a);
                else eta ? launch_step<T, true, false, false, false, true, true>(e, s, a) : launch_step<T, false, false, false, false, true, true>(e, s, a);
                return;
            }
            if (feat) eta ? launch_step<T, true, NT, true, MULTI, true>(e, s, a) : launch_step<T, false, NT, true, MULTI, true>(e, s, a);
            else eta ? launch_step<T, true, NT, false, MULTI, true>(e, s, a) : launch_step<T, false, NT, false, MULTI, true>(e, s, a);
        } else {
            if (feat) eta ? launch_step<T, true, NT, true, MULTI, false>(e, s, a) : launch_step<T, false, NT, true, MULTI, false>(e, s, a);
            else eta ? launch_step<T, true, NT, false, MULTI, false>(e, s, a) : launch_step<T, false, NT, false, MULTI, false>(e, s, a);
        }
    };
    if (e->n <= HG_NT_WAVES * e->resident_envs) pick(std::true_type{});
    else pick(std::false_type{});
    return hipSuccess;
}
template <bool MULTI>
static hipError_t dispatch_task(const hg_env* e, hipStream_t s, const StepArgs& a, bool eta, bool feat) {
    switch (e->cfg.task) {
        case HG_TASK_HOVER: return dispatch_step<HG_TASK_HOVER, MULTI>(e, s, a, eta, feat);
        case HG_TASK_FORWARD_FLIGHT: return dispatch_step<HG_TASK_FORWARD_FLIGHT, MULTI>(e, s, a, eta, feat);
        default: return dispatch_step<HG_TASK_HELI, MULTI>(e, s, a, eta, feat);
    }
}

// ov mode's launch: `ov_trim_blocks` trim blocks (the previous step's ends; blocks without a job exit at
// once) ahead of the step's blocks -- never more than one per env (a step ends at most n episodes)
#ifndef HG_OV_TB_DIV   // (A/B knob: the overlapped launch's trim blocks, n / 256 / this)
#define HG_OV_TB_DIV 1
#endif
static inline int32_t ov_trim_blocks(int64_t n) {
    int64_t b = n / 256 / HG_OV_TB_DIV;
    b = b < 64 ? 64 : (b > 1024 ? 1024 : b);
    return (int32_t)(b < n ? b : n);
}
static void launch_step_ov(const hg_env* e, hipStream_t s, const StepArgs& a, const hgk::RetrimArgs& r) {
    const int32_t tb = ov_trim_blocks(e->n);
    const unsigned grid = (unsigned)((e->n + kStepBlock - 1) / kStepBlock) + (unsigned)tb;
    auto go = [&](auto kern) {
        hipLaunchKernelGGL(kern, dim3(grid), dim3(kStepBlock), 0, s, r.count, r.recs, r.T, r.P, STEP_KARGS(e), a, r, tb);
    };
    switch (e->cfg.task) {
        case HG_TASK_HOVER: e->baked ? go(step_ov_kernel<HG_TASK_HOVER, true>) : go(step_ov_kernel<HG_TASK_HOVER, false>); break;
        case HG_TASK_FORWARD_FLIGHT:
            e->baked ? go(step_ov_kernel<HG_TASK_FORWARD_FLIGHT, true>) : go(step_ov_kernel<HG_TASK_FORWARD_FLIGHT, false>);
            break;
        default: e->baked ? go(step_ov_kernel<HG_TASK_HELI, true>) : go(step_ov_kernel<HG_TASK_HELI, false>); break;
    }
}

static void launch_step_fused(const hg_env* e, hipStream_t s, const StepArgs& a, const hgk::RetrimArgs& r, int32_t tb) {
    const unsigned grid = (unsigned)((e->n + kStepBlock - 1) / kStepBlock) + (unsigned)tb;
    auto go = [&](auto kern) {
        hipLaunchKernelGGL(kern, dim3(grid), dim3(kStepBlock), 0, s, r.count, r.recs, r.T, r.P, STEP_KARGS(e), a, r, tb);
    };
    switch (e->cfg.task) {
        case HG_TASK_HOVER: e->baked ? go(step_fused_kernel<HG_TASK_HOVER, true>) : go(step_fused_kernel<HG_TASK_HOVER, false>); break;
        case HG_TASK_FORWARD_FLIGHT:
            e->baked ? go(step_fused_kernel<HG_TASK_FORWARD_FLIGHT, true>) : go(step_fused_kernel<HG_TASK_FORWARD_FLIGHT, false>);
            break;
        default: e->baked ? go(step_fused_kernel<HG_TASK_HELI, true>) : go(step_fused_kernel<HG_TASK_HELI, false>); break;
    }
}

extern "C" {
#if HG_TIMING
int hg_debug_timing(void* dst, int64_t bytes) {
    return hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_timing), (size_t)bytes) == hipSuccess ? 0 : -1;
}
int hg_debug_timing_help(void* dst, int64_t bytes) {
    return hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_timing_help), (size_t)bytes) == hipSuccess ? 0 : -1;
}
int hg_debug_fused_probe(void* dst, int64_t bytes) {
    return hipMemcpyFromSymbol(dst, HIP_SYMBOL(hgk::g_fused_probe), (size_t)bytes) == hipSuccess ? 0 : -1;
}
#endif

int32_t hg_abi_version(void) { return HG_ABI_VERSION; }

int32_t hg_host_alloc(int64_t bytes, void** host, void** dev) {
    if (!host || !dev || bytes <= 0) return fail(HG_E_INVALID, "hg_host_alloc: bad arguments");
    *host = nullptr;
    *dev = nullptr;
    void* h = nullptr;
    HIP_TRY(hipHostMalloc(&h, (size_t)bytes, hipHostMallocMapped | hipHostMallocCoherent));
    void* d = nullptr;
    const hipError_t err = hipHostGetDevicePointer(&d, h, 0);
    if (err != hipSuccess || !d) {
        (void)hipHostFree(h);
        return fail(HG_E_HIP, std::string("hipHostGetDevicePointer: ") + hipGetErrorString(err));
    }
    memset(h, 0, (size_t)bytes);
    *host = h;
    *dev = d;
    return HG_OK;
}

void hg_host_free(void* host) {
    if (host) (void)hipHostFree(host);
}

int32_t hg_debug_params(const hg_config* cfg, int32_t rows, int32_t cols, int32_t baked_only, void* out,
                        int64_t bytes) {
    if (!cfg || !out || bytes != (int64_t)sizeof(Params<float>)) return fail(HG_E_INVALID, "hg_debug_params: bad arguments");
    const Params<float> P = derive<float>(*cfg, rows, cols);
    if (!baked_only) {
        memcpy(out, &P, sizeof(P));
        return HG_OK;
    }
    Params<float> B;
    memset(&B, 0, sizeof(B));
#define HG_COPY_ONE(f) B.f = P.f;
    HG_BAKED_FIELDS(HG_COPY_ONE)
#undef HG_COPY_ONE
    memcpy(out, &B, sizeof(B));
    return HG_OK;
}

int32_t hg_config_is_baked(const hg_config* cfg, int32_t rows, int32_t cols) {
    if (!cfg) return 0;
    return hg::bake_matches(derive<float>(*cfg, rows, cols)) ? 1 : 0;
}

const char* hg_last_error(void) { return g_last_error.c_str(); }

void hg_default_config(hg_config* c) {
    if (!c) return;
    memset(c, 0, sizeof(*c));
    hg_airframe& a = c->af;
    // aw109.yaml:2-101
    a.env_R = 1716.49; a.env_T0 = 518.4; a.env_LAPSE = 0.0035662; a.env_RO_SEA = 0.0023769;
    a.env_GRAV = 32.2; a.env_MAX_GR_ALT = 8809.0551; a.env_NS_MAX = 6561.6798; a.env_EW_MAX = 6561.6798;
    a.env_WIND_DIR_deg = 45.0; a.env_WIND_SPD = 20.0; a.env_TURB_LVL = 1;
    a.HP_LOSS = 90; a.VTRANS = 50; a.FS_CG = 132.7; a.WL_CG = 38.5; a.WT = 5401;
    a.IX = 1590; a.IY = 6761; a.IZ = 6407; a.IXZ = 598;
    a.COL_OS = 6; a.COL_L = -2; a.COL_H = 15; a.LON_L = -12; a.LON_H = 12; a.LAT_L = -10; a.LAT_H = 10;
    a.PED_OS = 15; a.PED_L = -15; a.PED_H = 15;
    a.mr_FS = 132.4; a.mr_WL = 98.2; a.mr_IS = 0.11; a.mr_E = 0.5; a.mr_IB = 212; a.mr_R = 18; a.mr_A = 5.8;
    a.mr_RPM = 385; a.mr_CD0 = 0.009; a.mr_B = 4; a.mr_C = 1.1; a.mr_TWST = -0.105; a.mr_K1 = 0.096;
    a.tr_FS = 391; a.tr_WL = 70; a.tr_R = 3.1; a.tr_A = 4.2; a.tr_C = 0.6525; a.tr_RPM = 2080; a.tr_CD0 = 0.009;
    a.tr_TWST = -0.137; a.tr_B = 2;
    a.fus_FS = 132; a.fus_WL = 38; a.fus_XUU = -10.8; a.fus_YVV = -167; a.fus_ZWW = -85; a.fus_COR = 3;
    a.ht_FS = 330; a.ht_WL = 54; a.ht_ZUU = 0.4; a.ht_ZUW = -34.0; a.ht_ZMAX = -22.0;
    a.vt_FS = 380; a.vt_WL = 80; a.vt_YUU = 3.3; a.vt_YUV = -47; a.vt_YMAX = -17;
    a.wn_FS = 0; a.wn_WL = 0; a.wn_ZUU = 0; a.wn_ZUW = 0; a.wn_ZMAX = 0; a.wn_B = 1;
    a.lg_K = 30000; a.lg_C = 2000; a.lg_BL_MN = 42; a.lg_FS_MN = 187; a.lg_FS_N = 40; a.lg_WL = -22;
    // helicopter.py:18-44, helicopter_with_tasks.py:9-22
    c->trim.gr_alt = 100.0;
    c->target.sea_alt = 4000.0;
    c->dt = 1.0 / 50.0;
    c->max_time = 40.0;
    c->task = HG_TASK_HOVER;
    c->autoreset = 1;
}

static std::vector<float2> split_terrain(const double* t, int32_t rows, int32_t cols) {
    std::vector<float2> v((size_t)rows * cols);
    for (size_t k = 0; k < v.size(); ++k) {
        const float hi = (float)t[k];
        v[k] = make_float2(hi, (float)(t[k] - (double)hi));
    }
    return v;
}

// every device resource of a handle (create's error paths and hg_destroy), then the handle
static void release(hg_env* e) {
    if (e->rtc_mod) {   // steps still queued on any stream may use its kernels
        (void)hipDeviceSynchronize();
        (void)hipModuleUnload(e->rtc_mod);
    }
    dfree(e->hmap); dfree(e->state); dfree(e->az); dfree(e->tmpl_dev); dfree(e->params_dev);
    dfree(e->trim_block); dfree(e->retrim_wind); dfree(e->retrim_list); dfree(e->retrim_recs);
    dfree(e->ov_recs); dfree(e->ov_ring); dfree(e->fused_ring);
    dfree(e->tmpl_env); dfree(e->setup_batch);
    delete e;
}

// Diagnostic (not in the header): the host trim's central-difference Jacobian of every Newton step
// (row-major [k][16][16] into jac, at most jac_max), for studying the solve offline.  Returns the
// number recorded, or an HG_E_* code.
int32_t hg_debug_trim_jacobians(const hg_config* cfg, const double* terrain_ft, int32_t rows, int32_t cols,
                                const double wind_ned[3], double* jac, int32_t jac_max) {
    int32_t rc = check_config(cfg, rows, cols);
    if (rc != HG_OK) return rc;
    if (!terrain_ft || !jac || jac_max < 1) return fail(HG_E_INVALID, "bad arguments");
    const Params<double> P = derive<double>(*cfg, rows, cols);
    double W[3] = {P.wm[0], P.wm[1], P.wm[2]};
    if (wind_ned) { W[0] = wind_ned[0]; W[1] = wind_ned[1]; W[2] = wind_ned[2]; }
    const std::vector<float2> hm = split_terrain(terrain_ft, rows, cols);
    hg_trim_result out;
    int32_t n = 0;
    rc = do_trim(P, hm.data(), cfg->trim, W, &out, jac, jac_max, &n);
    return rc == HG_OK ? n : rc;
}

int32_t hg_trim(const hg_config* cfg, const double* terrain_ft, int32_t rows, int32_t cols,
                const double wind_ned[3], hg_trim_result* out) {
    int32_t rc = check_config(cfg, rows, cols);
    if (rc != HG_OK) return rc;
    if (!terrain_ft || !out) return fail(HG_E_INVALID, "terrain/out is NULL");
    const Params<double> P = derive<double>(*cfg, rows, cols);
    double W[3] = {P.wm[0], P.wm[1], P.wm[2]};
    if (wind_ned) { W[0] = wind_ned[0]; W[1] = wind_ned[1]; W[2] = wind_ned[2]; }
    memset(out, 0, sizeof(*out));
    const std::vector<float2> hm = split_terrain(terrain_ft, rows, cols);
    return do_trim(P, hm.data(), cfg->trim, W, out);
}

int32_t hg_create(const hg_config* cfg, const double* terrain_ft, int32_t rows, int32_t cols, int64_t num_envs,
                  hg_env** out) {
    if (!out) return fail(HG_E_INVALID, "out is NULL");
    *out = nullptr;
    int32_t rc = check_config(cfg, rows, cols);
    if (rc != HG_OK) return rc;
    if (!terrain_ft) return fail(HG_E_INVALID, "terrain is NULL");
    if (num_envs < 1 || num_envs > ((int64_t)1 << 31) - kBlock)
        return fail(HG_E_INVALID, "num_envs must be in [1, 2^31 - 256)");
    hg_env* e = new hg_env();
    e->cfg = *cfg;
    e->n = num_envs;
    e->rows = rows;
    e->cols = cols;
    e->hmap_host = split_terrain(terrain_ft, rows, cols);
    rederive(e);   // model constants, and the constant-specialised kernel when they are the baked ones
    if (!gear_layout_ok(e->Pf)) {
        delete e;
        return fail(HG_E_INVALID, "landing gear: the step kernels need the nose wheel on the centre line and "
                                  "the mains mirrored about it on one waterline");
    }
    rc = build_template(e);
    if (rc != HG_OK) { delete e; return rc; }
    auto cleanup = [&](hipError_t err, const char* what) {
        release(e);
        return fail(HG_E_HIP, std::string(what) + ": " + hipGetErrorString(err));
    };
    hipError_t err;
    int dev = 0, cus = 0;
    if ((err = hipGetDevice(&dev)) != hipSuccess) return cleanup(err, "hipGetDevice");
    e->device = dev;
    if ((err = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev)) != hipSuccess)
        return cleanup(err, "hipDeviceGetAttribute");
    e->resident_envs = (int64_t)cus * 4 * 64;
    if ((err = hipMalloc(&e->hmap, sizeof(float2) * rows * cols)) != hipSuccess) return cleanup(err, "hipMalloc terrain");
    if ((err = hipMalloc(&e->state, sizeof(float) * hgk::tile_words(num_envs))) != hipSuccess)
        return cleanup(err, "hipMalloc state");
    if ((err = hipMalloc(&e->az, sizeof(AzRec) * num_envs)) != hipSuccess) return cleanup(err, "hipMalloc azimuths");
    if ((err = hipMemcpy(e->hmap, e->hmap_host.data(), sizeof(float2) * rows * cols, hipMemcpyHostToDevice)) != hipSuccess)
        return cleanup(err, "hipMemcpy terrain");
    if ((err = hipMalloc(&e->params_dev, sizeof(Params<float>))) != hipSuccess) return cleanup(err, "hipMalloc params");
    if ((err = hipMemcpy(e->params_dev, &e->Pf, sizeof(e->Pf), hipMemcpyHostToDevice)) != hipSuccess)
        return cleanup(err, "hipMemcpy params");
    if ((err = hipMalloc(&e->tmpl_dev, kTplAlloc)) != hipSuccess) return cleanup(err, "hipMalloc template");
    if ((err = hipMemset(e->tmpl_dev, 0, kTplAlloc)) != hipSuccess) return cleanup(err, "hipMemset template");
    if ((err = hipMemcpy(e->tmpl_dev, &e->tmpl, sizeof(e->tmpl), hipMemcpyHostToDevice)) != hipSuccess)
        return cleanup(err, "hipMemcpy template");
    {   // [0, 64) the job-count ring, [64, 128) the counters, then the setup and the constants
        constexpr size_t kSetupOff = 128;
        constexpr size_t kPdOff = (kSetupOff + sizeof(hg::TrimSetup) + 255) / 256 * 256;
        constexpr size_t kBlock = kPdOff + sizeof(Params<double>);
        static_assert(kBlock <= 4096, "the trim block fits one page");
        if ((err = hipMalloc(&e->trim_block, 4096)) != hipSuccess) return cleanup(err, "hipMalloc trim block");
        if ((err = hipMemset(e->trim_block, 0, 4096)) != hipSuccess) return cleanup(err, "hipMemset trim block");
        char* b = static_cast<char*>(e->trim_block);
        e->retrim_ring = reinterpret_cast<int32_t*>(b);
        e->retrim_count = reinterpret_cast<int32_t*>(b + 64);
        e->setup_dev = reinterpret_cast<hg::TrimSetup*>(b + kSetupOff);
        e->pd_dev = reinterpret_cast<Params<double>*>(b + kPdOff);
    }
    if ((err = hipMemcpy(e->setup_dev, &e->setup, sizeof(e->setup), hipMemcpyHostToDevice)) != hipSuccess)
        return cleanup(err, "hipMemcpy setup");
    if ((err = hipMemcpy(e->pd_dev, &e->Pd, sizeof(e->Pd), hipMemcpyHostToDevice)) != hipSuccess)
        return cleanup(err, "hipMemcpy params64");
    if ((err = hipMalloc(&e->fused_ring, 3 * kFusedSlot * sizeof(int32_t))) != hipSuccess) return cleanup(err, "hipMalloc fused ring");
    if ((err = hipMemset(e->fused_ring, 0, 3 * kFusedSlot * sizeof(int32_t))) != hipSuccess) return cleanup(err, "hipMemset fused ring");
    if (cfg->reset_mode == HG_RESET_RETRIM) {
        if ((err = hipMalloc(&e->retrim_wind, sizeof(float) * 3 * num_envs)) != hipSuccess)
            return cleanup(err, "hipMalloc retrim wind");
        if ((err = hipMalloc(&e->retrim_list, sizeof(int32_t) * num_envs)) != hipSuccess)
            return cleanup(err, "hipMalloc retrim list");
        if ((err = hipMalloc(&e->retrim_recs, sizeof(int4) * num_envs)) != hipSuccess)
            return cleanup(err, "hipMalloc retrim jobs");
        // job records never written name env -1: a trim reading one skips it (and counts it)
        if ((err = hipMemset(e->retrim_recs, 0xFF, sizeof(int4) * num_envs)) != hipSuccess)
            return cleanup(err, "hipMemset retrim jobs");
        hipLaunchKernelGGL(fill_wind_kernel, dim3(grid_for(num_envs)), dim3(kBlock), 0, 0, e->retrim_wind, num_envs,
                           (float)e->Pd.wm[0], (float)e->Pd.wm[1], (float)e->Pd.wm[2]);
        if ((err = hipGetLastError()) != hipSuccess) return cleanup(err, "fill_wind_kernel");

        if (cfg->autoreset && cfg->autoreset_mode == HG_AUTORESET_NEXT_STEP) {   // ov mode's job rings
            if ((err = hipMalloc(&e->ov_recs, sizeof(int4) * 3 * num_envs)) != hipSuccess)
                return cleanup(err, "hipMalloc ov jobs");
            if ((err = hipMemset(e->ov_recs, 0xFF, sizeof(int4) * 3 * num_envs)) != hipSuccess)
                return cleanup(err, "hipMemset ov jobs");
            if ((err = hipMalloc(&e->ov_ring, 3 * sizeof(int32_t))) != hipSuccess) return cleanup(err, "hipMalloc ov ring");
            if ((err = hipMemset(e->ov_ring, 0, 3 * sizeof(int32_t))) != hipSuccess) return cleanup(err, "hipMemset ov ring");
            e->ov = true;
        }
    }
    const int64_t slots = hgk::tile_words(num_envs) / hgk::kEnvSlots;
    hipLaunchKernelGGL(init_kernel, dim3(grid_for(slots)), dim3(kBlock), 0, 0, e->tmpl, e->state, slots, e->az,
                       num_envs);
    if ((err = hipGetLastError()) != hipSuccess) return cleanup(err, "init_kernel");
    if ((err = hipDeviceSynchronize()) != hipSuccess) return cleanup(err, "init sync");
    *out = e;
    return HG_OK;
}

void hg_destroy(hg_env* e) {
    if (!e) return;
    DevGuard dev_guard(e);
    release(e);
}

int64_t hg_num_envs(const hg_env* e) { return e ? e->n : -1; }

int32_t hg_set_max_time(hg_env* e, double max_time) {
    if (!e || !(max_time > 0)) return fail(HG_E_INVALID, "bad env or max_time");
    DevGuard dev_guard(e);
    if (!dev_guard.ok) return fail(HG_E_HIP, "hipSetDevice to the handle's device failed");
    e->cfg.max_time = max_time;
    rederive(e);
    return upload_params(e);
}

int32_t hg_set_specialized(hg_env* e, int32_t enable) {
    if (!e) return fail(HG_E_INVALID, "env is NULL");
    e->baked_allowed = enable != 0;
    rederive(e);
    return (e->baked || e->rtc) ? 1 : 0;
}

int32_t hg_load_specialized(hg_env* e, const char* code_object, int32_t task, const void* image, int64_t bytes) {
    if (!e || !code_object || !image) return fail(HG_E_INVALID, "hg_load_specialized: NULL argument");
    if (bytes != (int64_t)sizeof(Params<float>)) return fail(HG_E_INVALID, "hg_load_specialized: image size mismatch");
    DevGuard dev_guard(e);
    if (!dev_guard.ok) return fail(HG_E_HIP, "hipSetDevice to the handle's device failed");
    hipModule_t mod = nullptr;
    HIP_TRY(hipModuleLoad(&mod, code_object));
    static const char* const names[6] = {"hg_rtc_step_nt", "hg_rtc_step_nt_feat", "hg_rtc_step_nts",
                                         "hg_rtc_step_nts_feat", "hg_rtc_step_bulk", "hg_rtc_step_bulk_feat"};
    hipFunction_t fn[6];
    for (int k = 0; k < 6; ++k) {
        const hipError_t err = hipModuleGetFunction(&fn[k], mod, names[k]);
        if (err != hipSuccess) {
            (void)hipModuleUnload(mod);
            return fail(HG_E_HIP, std::string("hg_load_specialized: ") + names[k] + ": " + hipGetErrorString(err));
        }
    }
    {   // the image and task the code object was built with (step_rtc.hip): a code object built from a
        // truncated or foreign constant file is refused instead of stepping with its constants
        hipDeviceptr_t gi = nullptr, gt = nullptr;
        size_t bi = 0, bt = 0;
        Params<float> built;
        int32_t built_task = -1;
        hipError_t err = hipModuleGetGlobal(&gi, &bi, mod, "hg_rtc_image");
        if (err == hipSuccess) err = hipModuleGetGlobal(&gt, &bt, mod, "hg_rtc_task");
        if (err == hipSuccess && (bi != sizeof(built) || bt != sizeof(built_task))) err = hipErrorInvalidValue;
        if (err == hipSuccess) err = hipMemcpy(&built, gi, sizeof(built), hipMemcpyDeviceToHost);
        if (err == hipSuccess) err = hipMemcpy(&built_task, gt, sizeof(built_task), hipMemcpyDeviceToHost);
        if (err != hipSuccess) {
            (void)hipModuleUnload(mod);
            return fail(HG_E_HIP, std::string("hg_load_specialized: reading the built image: ") + hipGetErrorString(err));
        }
        if (memcmp(&built, image, sizeof(built)) != 0 || built_task != task) {
            (void)hipModuleUnload(mod);
            return fail(HG_E_INVALID, "hg_load_specialized: the code object was built with another constant image or task");
        }
    }
    HIP_TRY(hipDeviceSynchronize());   // queued steps may still use a previous module
    if (e->rtc_mod) (void)hipModuleUnload(e->rtc_mod);
    e->rtc_mod = mod;
    for (int k = 0; k < 6; ++k) e->rtc_fn[k] = fn[k];
    memcpy(&e->rtc_image, image, sizeof(e->rtc_image));
    e->rtc_task = task;
    rederive(e);
    return e->rtc ? 1 : 0;
}

int32_t hg_set_target(hg_env* e, const hg_target* t) {
    if (!e || !t) return fail(HG_E_INVALID, "bad env or target");
    DevGuard dev_guard(e);
    if (!dev_guard.ok) return fail(HG_E_HIP, "hipSetDevice to the handle's device failed");
    e->cfg.target = *t;
    rederive(e);
    return upload_params(e);
}

int32_t hg_set_trim_cond(hg_env* e, const hg_trim_cond* tc) {
    if (!e || !tc) return fail(HG_E_INVALID, "bad env or trim cond");
    DevGuard dev_guard(e);
    if (!dev_guard.ok) return fail(HG_E_HIP, "hipSetDevice to the handle's device failed");
    const hg_trim_cond old = e->cfg.trim;
    e->cfg.trim = *tc;
    const int32_t rc = build_template(e);
    if (rc != HG_OK) { e->cfg.trim = old; return rc; }
    return HG_OK;
}

int32_t hg_get_template(const hg_env* e, hg_trim_result* out) {
    if (!e || !out) return fail(HG_E_INVALID, "bad env or out");
    *out = e->trim;
    return HG_OK;
}

int32_t hg_reset(hg_env* e, const uint8_t* mask, float* obs, void* stream) {
    if (!e) return fail(HG_E_INVALID, "env is NULL");
    e->ov_chain = kChainBroken;   // the next step's pending resets take the serial re-trim
    DevGuard dev_guard(e);
    if (!dev_guard.ok) return fail(HG_E_HIP, "hipSetDevice to the handle's device failed");
    hipStream_t s = (hipStream_t)stream;
    hipLaunchKernelGGL(reset_kernel, dim3(grid_for(e->n)), dim3(kBlock), 0, s, e->tmpl,
                       e->Pf.env_templates ? e->tmpl_env : nullptr, e->state, e->az, mask, obs, e->n);
    HIP_TRY(hipGetLastError());
    if (e->cfg.reset_mode == HG_RESET_RETRIM) {   // trim each masked env against its last wind (F8)
        int32_t* zero[3] = {e->retrim_count, nullptr, nullptr};
        HIP_TRY(zero_counts(zero, s));
        hipLaunchKernelGGL(mask_list_kernel, dim3(grid_for(e->n)), dim3(kBlock), 0, s, mask, e->n, e->retrim_list,
                           e->retrim_count);
        hgk::RetrimArgs r;
        memset(&r, 0, sizeof(r));
        r.P = e->pd_dev;
        r.T = e->setup_dev;
        r.count = e->retrim_count;
        r.list = e->retrim_list;
        r.wind = e->retrim_wind;
        r.wind_soa = 1;
        r.state = e->state;
        r.az = e->az;
        r.obs = obs;
        r.n = e->n;
        r.fail_count = e->retrim_count + 1;
        r.bad_jobs = e->retrim_count + 2;
        r.solve_stats = e->retrim_count + 3;
        HIP_TRY(hgk::launch_retrim(r, retrim_grid(e->n), s));
        HIP_TRY(hipGetLastError());
    }
    return HG_OK;
}

static int32_t step_impl(hg_env* e, const float* actions, float* obs, float* reward, uint8_t* terminated,
                         uint8_t* truncated, uint8_t* info, const float* eta, int32_t* reset_count,
                         int32_t* reset_index, float* final_obs, int32_t* reset_count_next, float* final_obs_rows,
                         void* stream) {
    if (!e) return fail(HG_E_INVALID, "env is NULL");
    DevGuard dev_guard(e);
    if (!dev_guard.ok) return fail(HG_E_HIP, "hipSetDevice to the handle's device failed");
    if (!actions || !obs || !reward || !terminated || !truncated)
        return fail(HG_E_INVALID, "actions/obs/reward/terminated/truncated must be device pointers");
    if (((uintptr_t)actions & 15) || ((uintptr_t)obs & 15))
        return fail(HG_E_INVALID, "actions and obs must be 16-byte aligned");
    if ((reset_index || final_obs) && !reset_count)
        return fail(HG_E_INVALID, "reset_index/final_obs need reset_count");
    if (reset_count_next && (!reset_count || reset_count_next == reset_count))
        return fail(HG_E_INVALID, "reset_count_next needs reset_count and must be another buffer");
    hipStream_t s = (hipStream_t)stream;
    bool zero_count = reset_count != nullptr;
    uint64_t key = 0;
    const bool retrim = e->Pf.reset_retrim != 0 && e->Pf.autoreset != 0;   // auto-resets re-trimmed after the step
    if (reset_count_next || retrim) HIP_TRY(chain_key(s, &key));
    if (key != 0) e->ever_captured = true;
    // Once any step was captured, a replay of that graph (invisible here) may run between two eager
    // launches and leave the slot the next eager step counts into non-zero: eager steps then always
    // zero their own slot.  Inside one capture the graph's first step zeroes its slot (chain key of
    // a new capture) and each captured kernel zeroes the next one's, so every replay starts clean.
    const bool eager_after_capture = key == 0 && e->ever_captured;
    if (reset_count_next) {   // chained: the previous step zeroed reset_count if it was of the same sequence
        zero_count = e->chain_expect != key || eager_after_capture;
        e->chain_expect = key;
    } else {
        e->chain_expect = kChainBroken;
    }
    int32_t* zero[3] = {zero_count ? reset_count : nullptr, nullptr, nullptr};
    int32_t* rt_count = nullptr;
    int32_t rt_slot = -1;
    const bool ov = retrim && e->ov && e->ov_enabled;
    // ov mode: the previous step's ends are trimmed in this step's launch (step_ov_kernel) when it was
    // this sequence's previous launch (no other call in between; not across captures or from an eager
    // step after a capture, whose graphs may have run in between), for the lone-wave sizes, in-kernel
    // noise and the library's own kernels; otherwise this step's due resets take the serial re-trim
    const bool ov_active = ov && e->ov_chain == key && !eager_after_capture && !eta && !e->rtc &&
                           e->n <= HG_NT_WAVES * e->resident_envs;
    // fused same-step re-trim (step_fused_kernel, opt-in: hg_set_retrim_overlap(2)): the step's resets
    // trimmed in its own launch, for the lone-wave sizes, in-kernel noise and the library's own kernels
    const bool fused = retrim && !e->ov && e->fused_enabled && !eta && !e->rtc && e->n <= HG_NT_WAVES * e->resident_envs;
    int32_t* fused_pair = nullptr;
    if (retrim) {   // the step's re-trim job count: a slot of the ring, zeroed by the previous step's kernel
        rt_slot = (int32_t)(e->retrim_gen % 3);
        rt_count = e->retrim_ring + rt_slot;
        ++e->retrim_gen;
        if (e->retrim_chain != key || eager_after_capture) {
            zero[1] = rt_count;
            if (ov) zero[2] = e->ov_ring + rt_slot;
            if (fused) fused_pair = e->fused_ring + kFusedSlot * rt_slot;
        }
        e->retrim_chain = key;
    }
    HIP_TRY(zero_counts(zero, s, fused_pair));
    StepArgs a;
    a.hmap = e->hmap;
    a.actions = actions;
    a.obs = obs;
    a.reward = reward;
    a.terminated = terminated;
    a.truncated = truncated;
    a.info = info;
    a.eta = eta;
    a.reset_count = reset_count;
    a.reset_count_next = reset_count_next;
    a.final_obs_rows = final_obs_rows;
    a.reset_index = reset_index;
    a.final_obs = final_obs;
    a.retrim_wind = e->retrim_wind;
    a.retrim_recs = e->retrim_recs;
    a.retrim_count = retrim ? e->retrim_ring : e->retrim_count;   // (unused unless auto-resets re-trim)
    a.retrim_slot = rt_slot;
    a.tmpl_env = e->tmpl_env;
    a.nsteps = 1;
    a.ov_recs = ov ? e->ov_recs + (int64_t)rt_slot * e->n : nullptr;
    a.ov_count = ov ? e->ov_ring + rt_slot : nullptr;
    a.ov_count_next = ov ? e->ov_ring + (rt_slot == 2 ? 0 : rt_slot + 1) : nullptr;
    a.ov_active = ov_active ? 1 : 0;
    a.fused_ctr = fused ? reinterpret_cast<unsigned long long*>(e->fused_ring + kFusedSlot * rt_slot) : nullptr;
    a.fused_next = fused ? e->fused_ring + kFusedSlot * (rt_slot == 2 ? 0 : rt_slot + 1) : nullptr;
    const bool feat = reset_count || e->Pf.reset_retrim || e->Pf.autoreset_next ||
                      e->Pf.max_episode_steps != INT32_MAX || e->Pf.env_templates;
    ++e->n_launch[0];
    if (ov_active) {   // the previous step's ends trimmed in this launch's first blocks
        ++e->n_launch[1];
        const int prev = rt_slot == 0 ? 2 : rt_slot - 1;
        hgk::RetrimArgs r;
        memset(&r, 0, sizeof(r));
        r.P = e->pd_dev;
        r.T = e->setup_dev;
        r.count = e->ov_ring + prev;
        r.recs = e->ov_recs + (int64_t)prev * e->n;
        r.state = e->state;
        r.az = e->az;
        r.obs = obs;
        r.n = e->n;
        r.fail_count = e->retrim_count + 1;
        r.bad_jobs = e->retrim_count + 2;
        r.solve_stats = e->retrim_count + 3;
        r.ov = 1;
        r.tmpl = reinterpret_cast<const float*>(e->tmpl_dev);
        r.tmpl_env = e->Pf.env_templates ? e->tmpl_env : nullptr;
        launch_step_ov(e, s, a, r);
    } else if (fused) {   // this step's resets trimmed in its own launch's first blocks
        ++e->n_launch[1];
#ifndef HG_FUSED_TB_DIV
#define HG_FUSED_TB_DIV 1
#endif
        const int32_t tb = ov_trim_blocks(e->n) / HG_FUSED_TB_DIV;
        hgk::RetrimArgs r;
        memset(&r, 0, sizeof(r));
        r.P = e->pd_dev;
        r.T = e->setup_dev;
        r.recs = e->retrim_recs;   // (no count: the queue's end is r.ctr's low word once every wave reserved)
        r.state = e->state;
        r.az = e->az;
        r.obs = obs;
        r.n = e->n;
        r.fail_count = e->retrim_count + 1;
        r.bad_jobs = e->retrim_count + 2;
        r.solve_stats = e->retrim_count + 3;
        r.ov = 1;   // the deferred resets: the trim writes all but the step counter
        r.tmpl = reinterpret_cast<const float*>(e->tmpl_dev);
        r.tmpl_env = e->Pf.env_templates ? e->tmpl_env : nullptr;
        r.claim = e->fused_ring + kFusedSlot * rt_slot + 2;
        r.ctr = reinterpret_cast<const unsigned long long*>(e->fused_ring + kFusedSlot * rt_slot);
        r.nwaves = (int32_t)((e->n + kStepBlock - 1) / kStepBlock);
        launch_step_fused(e, s, a, r, tb);
    } else {
        HIP_TRY(dispatch_task<false>(e, s, a, eta != nullptr, feat));
    }
    HIP_TRY(hipGetLastError());
    if (ov) e->ov_chain = key;
    if (retrim && !ov_active && !fused) {   // re-trim this step's resets against their last wind (overwrites the template)
        hgk::RetrimArgs r;
        memset(&r, 0, sizeof(r));
        r.P = e->pd_dev;
        r.T = e->setup_dev;
        r.count = rt_count;
        r.recs = e->retrim_recs;
        r.state = e->state;
        r.az = e->az;
        r.obs = obs;
        r.n = e->n;
        r.fail_count = e->retrim_count + 1;
        r.bad_jobs = e->retrim_count + 2;
        r.solve_stats = e->retrim_count + 3;
        HIP_TRY(hgk::launch_retrim(r, retrim_grid(e->n), s));
    }
    HIP_TRY(hipGetLastError());
    return HG_OK;
}

int32_t hg_step(hg_env* e, const float* actions, float* obs, float* reward, uint8_t* terminated,
                uint8_t* truncated, uint8_t* info, const float* eta, int32_t* reset_count, int32_t* reset_index,
                float* final_obs, void* stream) {
    return step_impl(e, actions, obs, reward, terminated, truncated, info, eta, reset_count, reset_index, final_obs,
                     nullptr, nullptr, stream);
}

int32_t hg_step_chained(hg_env* e, const float* actions, float* obs, float* reward, uint8_t* terminated,
                        uint8_t* truncated, uint8_t* info, const float* eta, int32_t* reset_count,
                        int32_t* reset_index, float* final_obs, int32_t* reset_count_next, void* stream) {
    return step_impl(e, actions, obs, reward, terminated, truncated, info, eta, reset_count, reset_index, final_obs,
                     reset_count_next, nullptr, stream);
}

int32_t hg_step_rows(hg_env* e, const float* actions, float* obs, float* reward, uint8_t* terminated,
                     uint8_t* truncated, uint8_t* info, const float* eta, float* final_obs_rows, void* stream) {
    if (final_obs_rows && !info) return fail(HG_E_INVALID, "hg_step_rows: final_obs_rows needs info (HG_INFO_RESET)");
    return step_impl(e, actions, obs, reward, terminated, truncated, info, eta, nullptr, nullptr, nullptr, nullptr,
                     final_obs_rows, stream);
}

int32_t hg_rollout(hg_env* e, const float* actions, int32_t nsteps, float* obs, float* reward, uint8_t* terminated,
                   uint8_t* truncated, uint8_t* info, const float* eta, void* stream) {
    if (!e) return fail(HG_E_INVALID, "env is NULL");
    e->ov_chain = kChainBroken;   // the next step's pending resets take the serial re-trim
    DevGuard dev_guard(e);
    if (!dev_guard.ok) return fail(HG_E_HIP, "hipSetDevice to the handle's device failed");
    if (nsteps < 1) return fail(HG_E_INVALID, "nsteps must be >= 1");
    if (!actions || !obs || !reward || !terminated || !truncated)
        return fail(HG_E_INVALID, "actions/obs/reward/terminated/truncated must be device pointers");
    if (((uintptr_t)actions & 15) || ((uintptr_t)obs & 15))
        return fail(HG_E_INVALID, "actions and obs must be 16-byte aligned");
    if (e->Pf.reset_retrim && e->Pf.autoreset)
        return fail(HG_E_INVALID, "hg_rollout does not support auto-resets in reset_mode RETRIM (re-trims run between steps)");
    e->chain_expect = kChainBroken;
    StepArgs a;
    memset(&a, 0, sizeof(a));
    a.hmap = e->hmap;
    a.actions = actions;
    a.obs = obs;
    a.reward = reward;
    a.terminated = terminated;
    a.truncated = truncated;
    a.info = info;
    a.eta = eta;
    a.tmpl_env = e->tmpl_env;
    a.nsteps = nsteps;
    a.retrim_slot = -1;
    // reset_mode RETRIM without auto-reset: every step records its wind, the trim wind of a later
    // hg_reset (helicopter.py:208-212), as K hg_step calls would
    a.retrim_wind = e->retrim_wind;
    hipStream_t s = (hipStream_t)stream;
    const bool feat = e->Pf.autoreset_next || e->Pf.max_episode_steps != INT32_MAX || e->Pf.env_templates ||
                      e->Pf.reset_retrim;
    HIP_TRY(dispatch_task<true>(e, s, a, eta != nullptr, feat));
    HIP_TRY(hipGetLastError());
    return HG_OK;
}

int32_t hg_trim_batch(hg_env* e, const float* wind, int64_t count, float* state, float* action, float* obs,
                      int32_t* status, void* stream) {
    if (!e) return fail(HG_E_INVALID, "env is NULL");
    DevGuard dev_guard(e);
    if (!dev_guard.ok) return fail(HG_E_HIP, "hipSetDevice to the handle's device failed");
    if (count < 0 || (count > 0 && !wind)) return fail(HG_E_INVALID, "bad wind / count");
    if (count == 0) return HG_OK;
    hgk::RetrimArgs r;
    memset(&r, 0, sizeof(r));
    r.P = e->pd_dev;
    r.T = e->setup_dev;
    r.njobs = count;
    r.wind = wind;
    r.out_state = state;
    r.out_action = action;
    r.out_obs = obs;
    r.out_status = status;
    r.solve_stats = e->retrim_count + 3;
    HIP_TRY(hgk::launch_retrim(r, retrim_grid(count), (hipStream_t)stream));
    HIP_TRY(hipGetLastError());
    return HG_OK;
}

int32_t hg_trim_conds_batch(hg_env* e, const hg_trim_cond* conds, int64_t count, const float* wind, float* state,
                            float* action, float* obs, int32_t* status, void* stream) {
    if (!e) return fail(HG_E_INVALID, "env is NULL");
    DevGuard dev_guard(e);
    if (!dev_guard.ok) return fail(HG_E_HIP, "hipSetDevice to the handle's device failed");
    if (count < 0 || (count > 0 && !conds)) return fail(HG_E_INVALID, "bad conds / count");
    if (count == 0) return HG_OK;
    if (count > e->setup_batch_cap) {
        dfree(e->setup_batch);
        e->setup_batch = nullptr;
        e->setup_batch_cap = 0;
        HIP_TRY(hipMalloc(&e->setup_batch, sizeof(hg::TrimSetup) * count));
        e->setup_batch_cap = count;
    }
    std::vector<hg::TrimSetup> host((size_t)count);
    for (int64_t j = 0; j < count; ++j) {
        host[j] = trim_setup(e->Pd, e->hmap_host.data(), conds[j]);
        // the env condition's pivot order as the first choice (the residual test rejects it where
        // another condition's Jacobian needs other pivots, and the solve searches)
        memcpy(host[j].piv, e->setup.piv, sizeof(host[j].piv));
    }
    hipStream_t s = (hipStream_t)stream;
    HIP_TRY(hipMemcpyAsync(e->setup_batch, host.data(), sizeof(hg::TrimSetup) * count, hipMemcpyHostToDevice, s));
    hgk::RetrimArgs r;
    memset(&r, 0, sizeof(r));
    r.P = e->pd_dev;
    r.T = e->setup_batch;
    r.setup_stride = 1;
    r.njobs = count;
    r.wind = wind;
    r.out_state = state;
    r.out_action = action;
    r.out_obs = obs;
    r.out_status = status;
    r.solve_stats = e->retrim_count + 3;
    HIP_TRY(hgk::launch_retrim(r, retrim_grid(count), s));
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipStreamSynchronize(s));   // the host staging of the setups is released on return
    return HG_OK;
}

int32_t hg_set_reset_templates(hg_env* e, const float* templates, void* stream) {
    if (!e) return fail(HG_E_INVALID, "env is NULL");
    e->ov_chain = kChainBroken;   // the next step's pending resets take the serial re-trim
    DevGuard dev_guard(e);
    if (!dev_guard.ok) return fail(HG_E_HIP, "hipSetDevice to the handle's device failed");
    if (templates && e->cfg.reset_mode == HG_RESET_RETRIM)
        return fail(HG_E_INVALID, "per-env reset templates need reset_mode HG_RESET_TEMPLATE");
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(reanchor_azimuths(e));   // the records may point at the templates being replaced
    if (templates) {
        if (!e->tmpl_env) HIP_TRY(hipMalloc(&e->tmpl_env, sizeof(float) * kTplFloats * e->n));
        HIP_TRY(hipMemcpyAsync(e->tmpl_env, templates, sizeof(float) * kTplFloats * e->n, hipMemcpyDeviceToDevice,
                               (hipStream_t)stream));
        HIP_TRY(hipStreamSynchronize((hipStream_t)stream));
    }
    e->env_templates = templates != nullptr;
    e->Pf.env_templates = e->env_templates ? 1 : 0;
    return upload_params(e);
}

int32_t hg_retrim_failures(hg_env* e, int64_t* count) {
    if (!e || !count) return fail(HG_E_INVALID, "bad env or count");
    DevGuard dev_guard(e);
    if (!dev_guard.ok) return fail(HG_E_HIP, "hipSetDevice to the handle's device failed");
    int32_t v = 0;
    HIP_TRY(hipMemcpy(&v, e->retrim_count + 1, sizeof(int32_t), hipMemcpyDeviceToHost));
    *count = v;
    return HG_OK;
}

int32_t hg_debug_retrim_solves(hg_env* e, int64_t* counts) {
    if (!e || !counts) return fail(HG_E_INVALID, "bad env or counts");
    DevGuard dev_guard(e);
    if (!dev_guard.ok) return fail(HG_E_HIP, "hipSetDevice to the handle's device failed");
    int32_t v[2] = {0, 0};
    HIP_TRY(hipMemcpy(v, e->retrim_count + 3, sizeof(v), hipMemcpyDeviceToHost));
    counts[0] = v[0];
    counts[1] = v[1];
    return HG_OK;
}

int32_t hg_debug_retrim_invalid(hg_env* e, int64_t* count) {
    if (!e || !count) return fail(HG_E_INVALID, "bad env or count");
    DevGuard dev_guard(e);
    if (!dev_guard.ok) return fail(HG_E_HIP, "hipSetDevice to the handle's device failed");
    int32_t v = 0;
    HIP_TRY(hipMemcpy(&v, e->retrim_count + 2, sizeof(int32_t), hipMemcpyDeviceToHost));
    *count = v;
    return HG_OK;
}

#if HG_RT_DEBUG
int hg_debug_rt_log_ov(void* dst, int64_t bytes, int32_t clear) {
    if (dst && hipMemcpyFromSymbol(dst, HIP_SYMBOL(hgk::g_rt_dbg), (size_t)bytes) != hipSuccess) return -1;
    unsigned n = 0;
    if (hipMemcpyFromSymbol(&n, HIP_SYMBOL(hgk::g_rt_dbg_n), sizeof(n)) != hipSuccess) return -1;
    if (clear) {
        const unsigned z = 0;
        (void)hipMemcpyToSymbol(HIP_SYMBOL(hgk::g_rt_dbg_n), &z, sizeof(z));
    }
    return (int)n;
}
int hg_debug_ptrs(hg_env* e, int64_t* out) {
    out[0] = (int64_t)(uintptr_t)e->retrim_ring;
    out[1] = (int64_t)(uintptr_t)e->retrim_count;
    out[2] = (int64_t)(uintptr_t)e->ov_ring;
    return 0;
}
#endif

int32_t hg_debug_queues(hg_env* e, int32_t* out) {
    if (!e || !out) return fail(HG_E_INVALID, "bad env or out");
    DevGuard dev_guard(e);
    if (!dev_guard.ok) return fail(HG_E_HIP, "hipSetDevice to the handle's device failed");
    HIP_TRY(hipDeviceSynchronize());
    for (int k = 0; k < 9; ++k) out[k] = -7;
    HIP_TRY(hipMemcpy(out, e->retrim_ring, 3 * sizeof(int32_t), hipMemcpyDeviceToHost));
    if (e->ov_ring) HIP_TRY(hipMemcpy(out + 3, e->ov_ring, 3 * sizeof(int32_t), hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(out + 6, e->retrim_count, 3 * sizeof(int32_t), hipMemcpyDeviceToHost));
    return HG_OK;
}

int32_t hg_debug_launches(const hg_env* e, int64_t* out) {
    if (!e || !out) return fail(HG_E_INVALID, "bad env or out");
    for (int k = 0; k < 6; ++k) out[k] = e->n_launch[k];
    return HG_OK;
}

int32_t hg_set_retrim_overlap(hg_env* e, int32_t enable) {
    if (!e) return fail(HG_E_INVALID, "env is NULL");
    if (enable < 0 || enable > 2) return fail(HG_E_INVALID, "hg_set_retrim_overlap: enable is 0, 1 or 2");
    e->ov_enabled = enable != 0;
    e->fused_enabled = enable == 2;
    e->ov_chain = kChainBroken;
    return (e->ov && e->ov_enabled) ? 1 : 0;
}

int32_t hg_get_state(hg_env* e, float* state, int32_t* counters, void* stream) {
    if (!e) return fail(HG_E_INVALID, "env is NULL");
    DevGuard dev_guard(e);
    if (!dev_guard.ok) return fail(HG_E_HIP, "hipSetDevice to the handle's device failed");
    if (!state && !counters) return HG_OK;
    hipLaunchKernelGGL(get_rows_kernel, dim3(grid_for(e->n)), dim3(kBlock), 0, (hipStream_t)stream,
                       reinterpret_cast<const uint32_t*>(e->state), e->az, e->tmpl_dev,
                       e->Pf.env_templates ? e->tmpl_env : nullptr, PARAM_ARG(e), (uint32_t*)state, counters, e->n);
    HIP_TRY(hipGetLastError());
    return HG_OK;
}

int32_t hg_set_state(hg_env* e, const float* state, const int32_t* counters, void* stream) {
    if (!e) return fail(HG_E_INVALID, "env is NULL");
    e->ov_chain = kChainBroken;   // the next step's pending resets take the serial re-trim
    DevGuard dev_guard(e);
    if (!dev_guard.ok) return fail(HG_E_HIP, "hipSetDevice to the handle's device failed");
    if (!state && !counters) return HG_OK;
    hipLaunchKernelGGL(set_rows_kernel, dim3(grid_for(e->n)), dim3(kBlock), 0, (hipStream_t)stream,
                       reinterpret_cast<uint32_t*>(e->state), e->az, e->tmpl_dev,
                       e->Pf.env_templates ? e->tmpl_env : nullptr, PARAM_ARG(e), (const uint32_t*)state, counters,
                       e->n);
    HIP_TRY(hipGetLastError());
    return HG_OK;
}

int32_t hg_clock_stamp(uint64_t* dst, void* stream) {
    if (!dst || ((uintptr_t)dst & 7)) return fail(HG_E_INVALID, "hg_clock_stamp: dst must be an 8-byte aligned device pointer");
    hipLaunchKernelGGL(clock_stamp_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, dst);
    HIP_TRY(hipGetLastError());
    return HG_OK;
}

int32_t hg_random_actions(hg_env* e, float* actions, uint64_t seed, uint64_t step, float lo, float hi, void* stream) {
    if (!e || !actions) return fail(HG_E_INVALID, "env/actions is NULL");
    DevGuard dev_guard(e);
    if (!dev_guard.ok) return fail(HG_E_HIP, "hipSetDevice to the handle's device failed");
    if ((uintptr_t)actions & 15) return fail(HG_E_INVALID, "actions must be 16-byte aligned");
    hipLaunchKernelGGL(random_actions_kernel, dim3(grid_for(e->n)), dim3(kBlock), 0, (hipStream_t)stream, actions,
                       e->n, e->cfg.env_offset, seed, step, lo, hi);
    HIP_TRY(hipGetLastError());
    return HG_OK;
}

int32_t hg_debug_eta(hg_env* e, float* eta, void* stream) {
    if (!e || !eta) return fail(HG_E_INVALID, "env/eta is NULL");
    DevGuard dev_guard(e);
    if (!dev_guard.ok) return fail(HG_E_HIP, "hipSetDevice to the handle's device failed");
    hipLaunchKernelGGL(eta_kernel, dim3(grid_for(e->n)), dim3(kBlock), 0, (hipStream_t)stream, e->state, e->n,
                       (uint64_t)e->cfg.seed, (int64_t)e->cfg.env_offset, PARAM_ARG(e), eta);
    HIP_TRY(hipGetLastError());
    return HG_OK;
}

int32_t hg_debug_philox(const uint32_t* in, uint32_t* out, int64_t count, void* stream) {
    if (count < 0 || (count > 0 && (!in || !out))) return fail(HG_E_INVALID, "hg_debug_philox: bad arguments");
    if (count == 0) return HG_OK;
    hipLaunchKernelGGL(philox_kernel, dim3(grid_for(count)), dim3(kBlock), 0, (hipStream_t)stream, in, out, count);
    HIP_TRY(hipGetLastError());
    return HG_OK;
}

}  // extern "C"

#endif  // HG_RTC
