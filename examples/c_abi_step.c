/* Plain-C host of the heligym_amd C-ABI (include/heligym_amd.h): no Python, no torch.
 *
 * Creates N envs with the library's default AW109 / HeliHover configuration on a flat terrain,
 * resets them, steps them K times with constant trim controls, and prints a checksum of the final
 * observations plus the reset count.  Device buffers come from the HIP runtime directly.
 *
 *   gcc -O2 -std=c11 -I include -I /opt/rocm/include -D__HIP_PLATFORM_AMD__ examples/c_abi_step.c \
 *       -L heli-gym_amd/heligym_amd -lheligym_amd -L /opt/rocm/lib -lamdhip64 -o c_abi_step
 *   LD_LIBRARY_PATH=heli-gym_amd/heligym_amd:/opt/rocm/lib ./c_abi_step [N] [K]
 */
#include <hip/hip_runtime_api.h>
#include <stdio.h>
#include <stdlib.h>

#include "heligym_amd.h"

#define CHECK(x)                                                                   \
    do {                                                                           \
        int32_t rc_ = (x);                                                         \
        if (rc_ != HG_OK) {                                                        \
            fprintf(stderr, "%s failed (%d): %s\n", #x, rc_, hg_last_error());     \
            return 1;                                                              \
        }                                                                          \
    } while (0)
#define HIPCHECK(x)                                                                \
    do {                                                                           \
        if ((x) != hipSuccess) {                                                   \
            fprintf(stderr, "%s failed\n", #x);                                    \
            return 1;                                                              \
        }                                                                          \
    } while (0)

int main(int argc, char** argv) {
    const int64_t n = argc > 1 ? atoll(argv[1]) : 4096;
    const int k_steps = argc > 2 ? atoi(argv[2]) : 200;
    if (hg_abi_version() != HG_ABI_VERSION) {
        fprintf(stderr, "ABI mismatch\n");
        return 1;
    }
    hg_config cfg;
    hg_default_config(&cfg);
    cfg.dt = 0.01;
    const int rows = 64, cols = 64;
    double* terrain = (double*)malloc(sizeof(double) * rows * cols);
    for (int i = 0; i < rows * cols; ++i) terrain[i] = 1000.0;   /* flat 1000 ft */

    hg_trim_result tr;
    const double wind[3] = {14.142136, 14.142136, 0.0};
    CHECK(hg_trim(&cfg, terrain, rows, cols, wind, &tr));

    hg_env* env = NULL;
    CHECK(hg_create(&cfg, terrain, rows, cols, n, &env));
    float *act, *obs, *rew;
    uint8_t *term, *trunc;
    int32_t* nreset;
    HIPCHECK(hipMalloc((void**)&act, sizeof(float) * 4 * n));
    HIPCHECK(hipMalloc((void**)&obs, sizeof(float) * HG_N_OBS * n));
    HIPCHECK(hipMalloc((void**)&rew, sizeof(float) * n));
    HIPCHECK(hipMalloc((void**)&term, n));
    HIPCHECK(hipMalloc((void**)&trunc, n));
    HIPCHECK(hipMalloc((void**)&nreset, sizeof(int32_t)));
    float* h_act = (float*)malloc(sizeof(float) * 4 * n);
    for (int64_t i = 0; i < n; ++i)
        for (int c = 0; c < 4; ++c) h_act[4 * i + c] = (float)tr.action[c];
    HIPCHECK(hipMemcpy(act, h_act, sizeof(float) * 4 * n, hipMemcpyHostToDevice));

    CHECK(hg_reset(env, NULL, obs, NULL));
    int64_t resets = 0;
    for (int k = 0; k < k_steps; ++k) {
        CHECK(hg_step(env, act, obs, rew, term, trunc, NULL, NULL, nreset, NULL, NULL, NULL));
        int32_t r = 0;
        HIPCHECK(hipMemcpy(&r, nreset, sizeof(r), hipMemcpyDeviceToHost));
        resets += r;
    }
    float* h_obs = (float*)malloc(sizeof(float) * HG_N_OBS * n);
    HIPCHECK(hipMemcpy(h_obs, obs, sizeof(float) * HG_N_OBS * n, hipMemcpyDeviceToHost));
    double sum_alt = 0, sum_pow = 0;
    for (int64_t i = 0; i < n; ++i) {
        sum_pow += h_obs[HG_N_OBS * i + 0];
        sum_alt += h_obs[HG_N_OBS * i + 16];
    }
    printf("envs %lld steps %d resets %lld mean_power_hp %.4f mean_ground_alt_ft %.4f trim_iterations %d\n",
           (long long)n, k_steps, (long long)resets, sum_pow / n, sum_alt / n, tr.iterations);
    hg_destroy(env);
    hipFree(act); hipFree(obs); hipFree(rew); hipFree(term); hipFree(trunc); hipFree(nreset);
    free(terrain); free(h_act); free(h_obs);
    return 0;
}
