/*
 * heligym_amd.h — C-ABI of the MI355X-native vectorised heli-gym step().
 *
 * The reference (ugurcanozalp/heli-gym v2) has no FFI on this path: its boundary is the
 * gymnasium `Heli` env (heligym/envs/helicopter.py:28-243) calling two Python
 * `DynamicSystem.step` objects (heligym/envs/dynamics/dynamics.py:158-171).  Each entry point
 * below replaces one piece of that surface; the reference file:line it replaces is cited on it.
 * The only native precedent in the reference is its renderer C-ABI
 * (heligym/envs/renderer/src/py_api.h:17-90, opaque handles, ctypes-bound in pyapi.py:9-32);
 * this header follows the same opaque-handle style but every call returns an error code.
 *
 * Conventions
 *  - Units are the reference's US customary units (ft, slug, lb, s, rad).
 *  - All `*_dev` pointers are device (HBM) pointers owned by the caller, e.g. PyTorch-ROCm
 *    tensors; `stream` is a hipStream_t passed as void* (NULL = default stream).  Device calls
 *    are asynchronous on `stream`, never synchronise, never allocate, and are hipGraph-capturable.
 *  - Host pointers are plain host memory.  Sizes are element counts.
 *  - Return value: HG_OK (0) or a negative HG_E_* code; hg_last_error() gives the message of the
 *    last failure on the calling thread.  A handle is not re-entrant: one stream/thread at a time.
 *  - Layouts: actions [N,4] fp32 row-major; obs [N,17] fp32 row-major in the reference order
 *    (helicopter_dynamics.py:23-25); per-env state record [N,HG_STATE_COLS] fp32 (see below).
 */
#ifndef HELIGYM_AMD_H
#define HELIGYM_AMD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HG_ABI_VERSION 3

#define HG_N_OBS 17        /* helicopter_dynamics.py:23-27 */
#define HG_N_ACT 4         /* helicopter_dynamics.py:28 */
#define HG_N_HELI 18       /* vi_mr vi_tr psi_mr psi_tr betas[2] uvw[3] pqr[3] euler[3] xyz[3] (:55-64) */
#define HG_N_WIND 5        /* us vs[2] ws[2] (wind_dynamics.py:39-42) */
#define HG_N_CARRY 4       /* previous obs N_VEL, E_VEL, DES_RATE, GROUND_ALTITUDE (helicopter.py:195-196) */
/* state record columns: heli[18] | wind[5] | carry[4] */
#define HG_STATE_COLS (HG_N_HELI + HG_N_WIND + HG_N_CARRY)
/* counter record columns (int32): episode step, success steps, episode index */
#define HG_COUNTER_COLS 3

enum {
    HG_OK = 0,
    HG_E_INVALID = -1,   /* bad argument / shape */
    HG_E_HIP = -2,       /* HIP runtime error (no device, launch failure, ...) */
    HG_E_TRIM = -3,      /* trim did not converge (helicopter_dynamics.py:543-544) */
    HG_E_NOMEM = -4
};

/* Tasks: helicopter.py:242-243 (Heli, reward 0), helicopter_with_tasks.py:5-52 (HeliHover),
 * helicopter_with_tasks.py:54-115 (HeliForwardFlight). */
enum { HG_TASK_HELI = 0, HG_TASK_HOVER = 1, HG_TASK_FORWARD_FLIGHT = 2 };

/* Reset state of auto-reset envs (hg_config.reset_mode).
 *   HG_RESET_TEMPLATE: the trim against the mean wind, computed once (the reference's first reset,
 *                      helicopter.py:55 + helicopter_dynamics.py:66-71), broadcast in-kernel.
 *   HG_RESET_RETRIM:   every reset re-trimmed on the device against the wind of the env's last step,
 *                      as the reference does from its second episode on (the heli model keeps the
 *                      last set_wind, helicopter.py:198 -> helicopter_dynamics.py:66-71,491-555). */
enum { HG_RESET_TEMPLATE = 0, HG_RESET_RETRIM = 1 };

/* When auto-reset envs restart (hg_config.autoreset_mode, with autoreset = 1).
 *   HG_AUTORESET_SAME_STEP: the step that ends an episode returns the reset observation; the
 *                           terminal one goes to final_obs_dev (gymnasium SAME_STEP / SB3 style).
 *   HG_AUTORESET_NEXT_STEP: the ending step returns the terminal observation; the env's next step
 *                           ignores its action and returns the reset observation with reward 0 and
 *                           both flags false (gymnasium >= 1.0 vector default).  Between the two,
 *                           the env's episode-step counter reads -1. */
enum { HG_AUTORESET_SAME_STEP = 0, HG_AUTORESET_NEXT_STEP = 1 };

/* info bit-field written per env by hg_step (helicopter.py:219-224). */
enum { HG_INFO_FAILED = 1, HG_INFO_SUCCESSED = 2, HG_INFO_TIME_UP = 4, HG_INFO_SUCCESS_STEP = 8,
       HG_INFO_RESET = 16 /* auto-reset at the end of this step (same-step auto-reset) */ };

/* Raw airframe + environment parameters: the fields of heligym/envs/helis/aw109.yaml:2-101. */
typedef struct hg_airframe {
    /* ENV (aw109.yaml:2-16) */
    double env_R, env_T0, env_LAPSE, env_RO_SEA, env_GRAV, env_MAX_GR_ALT, env_NS_MAX, env_EW_MAX;
    double env_WIND_DIR_deg, env_WIND_SPD;
    int32_t env_TURB_LVL, _pad0;
    /* HELI (aw109.yaml:18-37) */
    double HP_LOSS, VTRANS, FS_CG, WL_CG, WT, IX, IY, IZ, IXZ;
    double COL_OS, COL_L, COL_H, LON_L, LON_H, LAT_L, LAT_H, PED_OS, PED_L, PED_H;
    /* MR (:39-52) */
    double mr_FS, mr_WL, mr_IS, mr_E, mr_IB, mr_R, mr_A, mr_RPM, mr_CD0, mr_B, mr_C, mr_TWST, mr_K1;
    /* TR (:54-63) */
    double tr_FS, tr_WL, tr_R, tr_A, tr_C, tr_RPM, tr_CD0, tr_TWST, tr_B;
    /* FUS (:65-71) */
    double fus_FS, fus_WL, fus_XUU, fus_YVV, fus_ZWW, fus_COR;
    /* HT (:73-78) */
    double ht_FS, ht_WL, ht_ZUU, ht_ZUW, ht_ZMAX;
    /* VT (:80-85) */
    double vt_FS, vt_WL, vt_YUU, vt_YUV, vt_YMAX;
    /* WN (:87-93) */
    double wn_FS, wn_WL, wn_ZUU, wn_ZUW, wn_ZMAX, wn_B;
    /* LG (:95-101) */
    double lg_K, lg_C, lg_BL_MN, lg_FS_MN, lg_FS_N, lg_WL;
} hg_airframe;

/* Trim condition (helicopter.py:36-44, helicopter_dynamics.py:45-53, consumed by trim :491-555). */
typedef struct hg_trim_cond {
    double yaw, yaw_rate, ned_vel[3], gr_alt, xy[2], psi_mr, psi_tr;
} hg_trim_cond;

/* Task target (helicopter_with_tasks.py:9-13, 59-63): north_loc, east_loc, sea_alt, heading, vel. */
typedef struct hg_target {
    double north_loc, east_loc, sea_alt, heading, vel;
} hg_target;

typedef struct hg_config {
    hg_airframe af;
    hg_trim_cond trim;
    hg_target target;
    double dt;            /* helicopter.py:18-19 (1/FPS = 0.02); north star uses 0.01 */
    double max_time;      /* helicopter.py:33-34,89-92 (40 s) */
    int32_t task;         /* HG_TASK_* */
    int32_t autoreset;    /* 1: reset finished envs inside hg_step (same-step autoreset) */
    uint64_t seed;        /* Philox key for the turbulence noise (wind_dynamics.py:49-52) */
    int64_t env_offset;   /* global id of local env 0 (sharding: results independent of rank count) */
    int32_t reset_mode;   /* HG_RESET_* */
    int32_t autoreset_mode; /* HG_AUTORESET_* */
    int64_t max_episode_steps; /* > 0: also truncate at this many steps (gymnasium TimeLimit, the
                                  registry's max_episode_steps=5000, heligym/__init__.py:4-18); 0: off */
} hg_config;

/* Reset template produced by the trim (host values). */
typedef struct hg_trim_result {
    double state[HG_N_HELI];       /* trimmed heli state (fp32-rounded, as the reference stores it) */
    double action[HG_N_ACT];       /* trim controls */
    double obs[HG_N_OBS];          /* observation at the trim state */
    double state_dots[HG_N_HELI];  /* dynamics at the trim state */
    double residual;               /* final ||y - y*||^2 of the Newton iteration */
    int32_t iterations;
    int32_t failed;                /* reset-time _is_failed() (helicopter.py:226-234) */
} hg_trim_result;

typedef struct hg_env hg_env;

/* Library / error ----------------------------------------------------------------------------- */
int32_t hg_abi_version(void);
const char* hg_last_error(void);

/* Model constants of a config as the step kernel sees them (Params<float> of csrc/physics.h,
 * `bytes` = its size), or only the fields that csrc/baked.h compiles in (`baked_only`, the rest
 * zero).  Host only; for scripts/gen_baked_constants.py and tests. */
int32_t hg_debug_params(const hg_config* cfg, int32_t rows, int32_t cols, int32_t baked_only, void* out,
                        int64_t bytes);
/* 1 when every compiled-in model constant (csrc/baked.h) equals this config's, i.e. hg_create will
 * select the constant-specialised step kernel for it; 0 otherwise.  Host only. */
int32_t hg_config_is_baked(const hg_config* cfg, int32_t rows, int32_t cols);

/* Host memory the kernels can read and write directly (pinned, mapped, coherent): `*host` is the
 * CPU address, `*dev` the address to pass to hg_step / hg_reset as a device pointer.  For
 * single-env or small-batch loops that want results on the host without separate copies (the
 * single-env drop-in: one launch and one stream synchronisation per step).  Free with
 * hg_host_free(host). */
int32_t hg_host_alloc(int64_t bytes, void** host, void** dev);
void hg_host_free(void* host);

/* Fill `cfg` with the AW109 / HeliHover defaults (aw109.yaml, helicopter.py:18-44,
 * helicopter_with_tasks.py:5-25).  Host only. */
void hg_default_config(hg_config* cfg);

/* Trim (host, fp64).  Replaces HelicopterDynamics.trim / __trim_fcn
 * (helicopter_dynamics.py:491-576) as called from reset (:66-71).  `terrain_ft` is the
 * [rows, cols] ground-height map in ft (helicopter_dynamics.py:39-43), `wind_ned` the wind the
 * trim is solved against (helicopter.py:55: the mean wind).  Heights are fp64 like the reference's
 * png/65535*MAX_GR_ALT; the library keeps each as an fp32 {hi, lo} pair. */
int32_t hg_trim(const hg_config* cfg, const double* terrain_ft, int32_t rows, int32_t cols,
                const double wind_ned[3], hg_trim_result* out);

/* Handle lifetime: replaces Heli.__init__ (helicopter.py:47-86: yaml params, HelicopterDynamics
 * and WindDynamics construction, terrain load) for `num_envs` independent helicopters, and
 * Heli.close (helicopter.py:185-187).  Uploads the terrain, derives the model constants, trims
 * the reset template against the mean wind. */
int32_t hg_create(const hg_config* cfg, const double* terrain_ft, int32_t rows, int32_t cols,
                  int64_t num_envs, hg_env** out);
void hg_destroy(hg_env* env);
int64_t hg_num_envs(const hg_env* env);

/* Setters: Heli.set_max_time (helicopter.py:89-92), set_target (:94-96), set_trim_cond
 * (:101-103; re-trims the reset template).  Host only; affect subsequent device calls. */
int32_t hg_set_max_time(hg_env* env, double max_time);
int32_t hg_set_target(hg_env* env, const hg_target* target);
/* Allow (1, the default) or forbid (0) the constant-specialised step kernel (csrc/baked.h), which
 * hg_create selects when the config's model constants are the compiled-in default airframe's.
 * Both kernels give bitwise-identical results; this switch exists for A/B timing and the tests.
 * Returns 1 if the specialised kernel is now in use, 0 if not, or an HG_E_* code. */
int32_t hg_set_specialized(hg_env* env, int32_t enable);
int32_t hg_set_trim_cond(hg_env* env, const hg_trim_cond* trim);
int32_t hg_get_template(const hg_env* env, hg_trim_result* out);

/* Reset: replaces Heli.reset (helicopter.py:208-217) -> WindDynamics.reset (wind_dynamics.py:44-47)
 * + HelicopterDynamics.reset (helicopter_dynamics.py:66-71).  Envs with mask_dev[i] != 0 (all
 * envs if mask_dev == NULL) get the trimmed state, zero turbulence state, zero counters; their
 * observation row is written to obs_dev [N,17] (other rows untouched).  In HG_RESET_RETRIM mode
 * each masked env is trimmed against the wind of its last step (the mean wind before its first
 * step), as the reference's reset trims against the model's last set_wind. */
int32_t hg_reset(hg_env* env, const uint8_t* mask_dev, float* obs_dev, void* stream);

/* Step: replaces Heli.step (helicopter.py:192-206) with everything it calls — WindDynamics.step
 * (dynamics.py:158-171 + wind_dynamics.py:49-125), HelicopterDynamics.step (dynamics.py:158-171
 * + helicopter_dynamics.py:73-77,400-489), the task reward (helicopter_with_tasks.py:27-52 /
 * 78-115) and _get_info (helicopter.py:219-240) — for all N envs in one kernel launch.
 *   actions_dev     [N,4]  fp32 in (no clipping, like the reference)
 *   obs_dev         [N,17] fp32 out (for auto-reset envs: the reset observation)
 *   reward_dev      [N]    fp32 out
 *   terminated_dev  [N]    u8 out   (failed or successed; helicopter.py:203)
 *   truncated_dev   [N]    u8 out   (time_up; helicopter.py:204)
 *   info_dev        [N]    u8 out or NULL (HG_INFO_* bits)
 *   eta_dev         [N,3]  fp32 in or NULL: turbulence noise already scaled by 1/sqrt(dt)
 *                          (parity / replay); NULL = in-kernel Philox4x32-10 normals keyed by
 *                          (seed, env_offset+i, episode, step)
 *   reset_count_dev [1]    i32 out or NULL: number of envs auto-reset this step (zeroed here)
 *   reset_index_dev [N]    i32 out or NULL: compacted ids of those envs (wave-ballot order)
 *   final_obs_dev   [N,17] fp32 out or NULL: their terminal observations, same compacted order */
int32_t hg_step(hg_env* env, const float* actions_dev, float* obs_dev, float* reward_dev,
                uint8_t* terminated_dev, uint8_t* truncated_dev, uint8_t* info_dev,
                const float* eta_dev, int32_t* reset_count_dev, int32_t* reset_index_dev,
                float* final_obs_dev, void* stream);

/* hg_step without the separate zeroing launch of the reset count: `reset_count_dev` must already be
 * 0 (the previous chained step zeroed it), and this launch zeroes `reset_count_next_dev` (another
 * buffer, for a later step) from inside the step kernel.  A caller rotating three count buffers
 * (step k: count[k % 3], next count[(k + 1) % 3]) keeps each step's count readable until the step
 * after next.  reset_count_dev is still zeroed by a memset launch when the handle's previous step
 * launch was not an hg_step_chained call of the same sequence -- the first call, after hg_step /
 * hg_step_rows / hg_rollout, the first call captured into a graph (so that every replay starts
 * from a zeroed count) and the first eager call after a capture.  Same results as hg_step. */
int32_t hg_step_chained(hg_env* env, const float* actions_dev, float* obs_dev, float* reward_dev,
                        uint8_t* terminated_dev, uint8_t* truncated_dev, uint8_t* info_dev,
                        const float* eta_dev, int32_t* reset_count_dev, int32_t* reset_index_dev,
                        float* final_obs_dev, int32_t* reset_count_next_dev, void* stream);

/* hg_step with the same-step reset info left uncompacted: the terminal observation of every env
 * auto-reset in this step goes to its own row of `final_obs_rows_dev` [N,17] (other rows are left
 * untouched) and its info byte carries HG_INFO_RESET, so the reset envs are the rows whose info has
 * that bit.  No count, no atomics, no zeroing launch: the step runs the same kernel as a plain
 * hg_step (the specialised one for the default airframe).  info_dev is required. */
int32_t hg_step_rows(hg_env* env, const float* actions_dev, float* obs_dev, float* reward_dev,
                     uint8_t* terminated_dev, uint8_t* truncated_dev, uint8_t* info_dev,
                     const float* eta_dev, float* final_obs_rows_dev, void* stream);

/* Open-loop rollout: `nsteps` consecutive hg_step calls in one launch, each env's state kept in
 * registers between steps (state is read and written once).  Results are identical to nsteps
 * hg_step calls with the same inputs (same auto-reset, noise keys, flags).  Inputs / outputs are
 * stacked per step: actions_dev [nsteps,N,4], obs_dev [nsteps,N,17], reward_dev [nsteps,N],
 * terminated_dev / truncated_dev / info_dev (or NULL) [nsteps,N], eta_dev [nsteps,N,3] or NULL.
 * For action sequences fixed in advance (sampling-based planning, data generation, replay); no
 * reset-info compaction; not available with HG_RESET_RETRIM. */
int32_t hg_rollout(hg_env* env, const float* actions_dev, int32_t nsteps, float* obs_dev, float* reward_dev,
                   uint8_t* terminated_dev, uint8_t* truncated_dev, uint8_t* info_dev, const float* eta_dev,
                   void* stream);

/* Batched device trim: HelicopterDynamics.trim (helicopter_dynamics.py:491-576) of the env's trim
 * condition against `count` winds at once — the reset path of reset_mode HG_RESET_RETRIM, exposed
 * for direct use.  Same Newton iteration as hg_trim (fp64, trial point rounded to fp32), with the
 * 32 Jacobian evaluations and the 10 line-search trials of each step evaluated in parallel lanes.
 *   wind_dev   [count,3] fp32 in (NED, ft/s)
 *   state_dev  [count,18] fp32 out or NULL, action_dev [count,4] fp32 out or NULL,
 *   obs_dev    [count,17] fp32 out or NULL, status_dev [count] i32 out or NULL
 *              (HG_OK, or HG_E_TRIM where the Newton iteration failed; outputs untouched there) */
int32_t hg_trim_batch(hg_env* env, const float* wind_dev, int64_t count, float* state_dev, float* action_dev,
                      float* obs_dev, int32_t* status_dev, void* stream);

/* Batched device trim for `count` trim conditions (host array `conds`, the reference's
 * set_trim_cond dicts, helicopter.py:101-106), against `wind_dev` [count,3] fp32 or, if NULL, the
 * mean wind: the first reset of `count` differently configured envs at once.  Outputs as
 * hg_trim_batch.  Synchronises with `stream` before returning. */
int32_t hg_trim_conds_batch(hg_env* env, const hg_trim_cond* conds, int64_t count, const float* wind_dev,
                            float* state_dev, float* action_dev, float* obs_dev, int32_t* status_dev,
                            void* stream);

/* Per-env reset targets (a batched set_trim_cond): templates_dev [N,39] fp32 = trimmed heli state
 * 18 | carry 4 (obs N/E/D velocity, ground altitude) | observation 17, one row per env, used by
 * hg_reset and by auto-reset instead of the shared template.  NULL reverts to the shared
 * template.  Copied; HG_RESET_TEMPLATE mode only. */
int32_t hg_set_reset_templates(hg_env* env, const float* templates_dev, void* stream);

/* Run-time specialisation for airframes other than the compiled-in default one (whose constants
 * are instruction literals of the library's step kernel): load a gfx950 code object built from
 * csrc/step_rtc.hip with this env's constant image (`image`, the sizeof(Params<float>) bytes
 * hg_debug_params returns with baked_only = 1) for `task`.  Per-step launches (no injected noise,
 * not hg_rollout) of an env whose constants match the image then run its kernels; results are
 * bitwise those of the generic kernel.  Returns 1 when in use, 0 when loaded but not matching,
 * < 0 on error.  Not part of the reference surface (replaces nothing: the reference has one
 * NumPy code path for every airframe). */
int32_t hg_load_specialized(hg_env* env, const char* code_object_path, int32_t task, const void* image,
                            int64_t bytes);

/* Number of RETRIM-mode auto-resets so far whose trim failed (those envs got the template state).
 * Synchronises with the device. */
int32_t hg_retrim_failures(hg_env* env, int64_t* count);

/* Diagnostic: re-trim job records that named no env (or a job count past N), skipped by the trim
 * instead of indexing the state with them; 0 in a correct run.  Synchronises with the device. */
int32_t hg_debug_retrim_invalid(hg_env* env, int64_t* count);

/* Diagnostic: the device trim's Newton solves since creation (every re-trim, hg_trim_batch and
 * hg_trim_conds_batch of this env): counts[0] solved with the pivot order of the host's trim of the
 * env's condition (gj_mfma.h gjs_solve), counts[1] of them rejected by the residual test and
 * re-solved with the pivot search.  Synchronous (reads device counters). */
int32_t hg_debug_retrim_solves(hg_env* env, int64_t* counts);

/* Diagnostic: the re-trim job-count rings (out[0..2] the step re-trim ring, out[3..5] the overlapped
 * re-trim ring or -7, out[6..8] hg_reset's job count, failures, invalid jobs).  Synchronises. */
int32_t hg_debug_queues(hg_env* env, int32_t* out);

/* Diagnostic: host-side launch counts of this handle since creation: out[0] step calls (hg_step,
 * hg_step_chained, hg_step_rows), out[1] steps whose launch held the previous step's re-trims
 * (hg_set_retrim_overlap), out[2] run-time specialised kernel launches, out[3] small-batch helper
 * kernel launches, out[4] lone-wave (one or two waves per SIMD) launches, out[5] bulk launches
 * (out[3..5] count hg_rollout's too).  Host only. */
int32_t hg_debug_launches(const hg_env* env, int64_t* out);

/* HG_RESET_RETRIM with next-step auto-reset (gymnasium's default, make_vec's): the episodes a step ends
 * are re-trimmed (helicopter.py:208-212 -> helicopter_dynamics.py:491-555) while the next step runs,
 * in the same kernel launch as that step (its first blocks), so the caller's stream sees every step
 * complete and the results are bitwise the serial path's.  A step holds the trims of the previous
 * step's ends only when that step was the previous launch of the same sequence (eager, or captured
 * into the same graph) with no other state-changing call on the handle in between, with in-kernel
 * noise and at most two step waves per SIMD (N <= 131 072 on MI355X); otherwise its due resets are
 * trimmed after it, serially.  enable = 1 (the default) or 0 (always serial: A/B and tests); 2 also
 * fuses, with same-step auto-reset, a step's re-trims into its own launch: trim blocks first, each
 * taking a reset as soon as its env's step wave has published it (in-kernel noise, at most two step
 * waves per SIMD).  Bitwise the serial path, but slower on MI355X (65 536 envs: 33.7 against 29.4 us
 * per step; the step waves run about 7 us longer beside the trims), so opt-in.  Returns 1 if the
 * next-step mode is configured and enabled, 0 otherwise, or HG_E_*. */
int32_t hg_set_retrim_overlap(hg_env* env, int32_t enable);

/* State access for parity tests / checkpointing (the reference's StateNumpy,
 * dynamics.py:75-128, exposed as one record per env): state [N,HG_STATE_COLS] fp32,
 * counters [N,HG_COUNTER_COLS] i32 (either may be NULL).  The rotor azimuths (state columns 2, 3)
 * are not part of the stepped state: hg_get_state reconstructs them (each step adds dt * Omega and
 * wraps, bitwise what the step would have carried), at a cost linear in the steps since the env's
 * last reset / set_state / hg_get_state (each read re-anchors the env's azimuth record at the values
 * it returns, so periodic reads keep every read short).  A negative episode-step counter marks an env whose next-step auto-reset
 * is due (read back as -1). */
int32_t hg_get_state(hg_env* env, float* state_dev, int32_t* counters_dev, void* stream);
int32_t hg_set_state(hg_env* env, const float* state_dev, const int32_t* counters_dev, void* stream);

/* Synthetic policy for benchmarks: actions [N,4] ~ U(lo, hi) from Philox4x32-10 keyed by
 * (seed, env_offset+i, step).  Not part of the reference surface. */
int32_t hg_random_actions(hg_env* env, float* actions_dev, uint64_t seed, uint64_t step,
                          float lo, float hi, void* stream);

/* Diagnostic (parity tests): the turbulence noise eta [N,3] fp32 (already scaled by 1/sqrt(dt)) that
 * each env's next hg_step with eta_dev == NULL draws in-kernel — WindDynamics.step_before
 * (wind_dynamics.py:49-52) restated as Philox4x32-10 keyed by (seed, env_offset+i, episode step,
 * episode index) and Box-Muller, computed by the same device function from the env's current
 * counters.  A step given these values as eta_dev is bitwise the in-kernel step. */
int32_t hg_debug_eta(hg_env* env, float* eta_dev, void* stream);

/* Diagnostic (known-answer tests): the device Philox4x32-10 on `count` rows of in_dev
 * {ctr0, ctr1, ctr2, ctr3, key0, key1} (u32) -> out_dev [count,4] u32.  It has no handle: it runs on
 * the calling thread's current HIP device, and both buffers must be device memory of that device
 * holding at least 6*count and 4*count words. */
int32_t hg_debug_philox(const uint32_t* in_dev, uint32_t* out_dev, int64_t count, void* stream);

/* Benchmark clock: one single-lane kernel on `stream` that writes the GPU's constant 100 MHz clock
 * (s_memrealtime) to dst_dev[0] when it runs.  Two stamps around K steps launched (or captured) on
 * the same stream time exactly those K kernels, each with its dependent-launch gap, plus the gap
 * after the first stamp.  Not part of the reference surface. */
int32_t hg_clock_stamp(uint64_t* dst_dev, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* HELIGYM_AMD_H */
