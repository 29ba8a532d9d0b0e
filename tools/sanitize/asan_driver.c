/*
 * asan_driver.c — host-side sanitizer run (SURVEY.md §5 "Race detection /
 * sanitizers": AddressSanitizer + UndefinedBehaviorSanitizer on the host
 * code; GPU-side sanitizers are not available on this pool).
 *
 * Built by tools/sanitize/Makefile with clang -fsanitize=address,undefined
 * against
 *   - the CPU oracle (oracle/salp_oracle.c, compiled into this binary), every
 *     entry point at several sizes, masks, 0 and 4 obstacles, randomisation
 *     switches, recording;
 *   - libsalp_asan.so: the C ABI of include/salp.h built with the host half
 *     instrumented (hipcc -Xarch_host -fsanitize=...).  Without a GPU only
 *     the argument checks and error paths run (salp_create then fails in
 *     hipSetDevice and must clean up); with --gpu a small end-to-end run goes
 *     through every entry point.
 * Exit status 0 = clean (the sanitizers abort on the first finding).
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "salp.h"

#ifdef SALP_SAN_GPU
#include <hip/hip_runtime_api.h>
#endif

int oracle_init(const SalpParams* p, int64_t n, double* state);
int oracle_reset_to(const SalpParams* p, int64_t n, double* state, const uint8_t* mask, const float* targets,
                    const float* obstacles, const int32_t* n_obst, float* obs_out, int obs_dim);
int oracle_reset(const SalpParams* p, int64_t n, double* state, const uint8_t* mask, uint64_t seed,
                 int64_t env_offset, float* obs_out, int obs_dim);
int oracle_step(const SalpParams* p, int64_t n, double* state, const float* actions, float* obs_out,
                double* reward_out, uint8_t* term_out, uint8_t* trunc_out, int auto_reset, float* term_obs_out,
                double* info_out, int64_t* ticks_out, uint64_t seed, int64_t env_offset, int obs_dim);
int64_t oracle_step_random(const SalpParams* p, int64_t n, double* state, int32_t n_steps, uint64_t seed,
                           int64_t env_offset, double* reward_sum, int nthreads);
int64_t oracle_robot_trace(const SalpParams* p, const float* actions, int n_actions, double* out,
                           int64_t max_rows);
int oracle_robot_reset(const SalpParams* p, int64_t n, double* state, const uint8_t* mask);
int oracle_nozzle_set_angles(const SalpParams* p, int64_t n, double* state, const double* ang);
int oracle_nozzle_solve(const SalpParams* p, int64_t n, double* state, const double* yaw, int yaw32);
int oracle_robot_set_control(const SalpParams* p, int64_t n, double* state, const double* ctl, int c32,
                             uint64_t seed, int64_t env_offset);
int oracle_robot_cycle(const SalpParams* p, int64_t n, double* state, double* rows, int64_t max_samples,
                       int64_t* n_samples, int64_t* ticks_out, uint64_t seed, int64_t env_offset);
void oracle_math_selftest(const double* x, const double* y, int64_t n, double* out);

#define CHECK(c)                                                         \
    do {                                                                 \
        if (!(c)) {                                                      \
            fprintf(stderr, "%s:%d: check failed: %s\n", __FILE__, __LINE__, #c); \
            exit(1);                                                     \
        }                                                                \
    } while (0)

static double frand(uint64_t* s) {
    *s = *s * 6364136223846793005ull + 1442695040888963407ull;
    return (double)(*s >> 11) * 0x1.0p-53;
}

static void oracle_suite(int n, int num_obstacles, int randomized) {
    SalpParams p;
    salp_default_params(&p);
    p.num_obstacles = num_obstacles;
    p.dynamics_randomization = p.disturbances = p.action_randomization = p.observation_randomization =
        p.latency = randomized;
    const int od = 6 + 2 * num_obstacles;
    double* st = calloc((size_t)SALP_NUM_FIELDS * n, sizeof(double));
    float* obs = calloc((size_t)n * od, sizeof(float));
    float* tobs = calloc((size_t)n * od, sizeof(float));
    float* act = calloc((size_t)n * 3, sizeof(float));
    double* rew = calloc((size_t)n, sizeof(double));
    double* info = calloc((size_t)n * SALP_INFO_DIM, sizeof(double));
    uint8_t *te = calloc((size_t)n, 1), *tr = calloc((size_t)n, 1), *mask = calloc((size_t)n, 1);
    int64_t* ticks = calloc((size_t)n, sizeof(int64_t));
    float* tg = calloc((size_t)n * 2, sizeof(float));
    float* ob = calloc((size_t)n * 2 * SALP_MAX_OBSTACLES, sizeof(float));
    int32_t* nob = calloc((size_t)n, sizeof(int32_t));
    uint64_t s = 12345u + (uint64_t)n;
    CHECK(oracle_init(&p, n, st) == 0);
    CHECK(oracle_reset(&p, n, st, NULL, 7, 100, obs, od) == 0);
    for (int i = 0; i < n; ++i) {
        tg[2 * i] = (float)(4 * frand(&s) - 2);
        tg[2 * i + 1] = (float)(3 * frand(&s) - 1.5);
        for (int k = 0; k < 2 * SALP_MAX_OBSTACLES; ++k) ob[2 * SALP_MAX_OBSTACLES * i + k] = (float)(4 * frand(&s) - 2);
        nob[i] = (int32_t)(i % (num_obstacles + 1));
        mask[i] = (uint8_t)(i % 3 != 0);
    }
    CHECK(oracle_reset_to(&p, n, st, mask, tg, ob, nob, obs, od) == 0);
    for (int t = 0; t < 4; ++t) {
        for (int i = 0; i < n; ++i) {
            act[3 * i] = (float)frand(&s);
            act[3 * i + 1] = (float)(t == 2 ? 0.0 : frand(&s));
            act[3 * i + 2] = (float)(2 * frand(&s) - 1);
        }
        CHECK(oracle_step(&p, n, st, act, obs, rew, te, tr, t & 1, tobs, info, ticks, 7, 100, od) == 0);
        CHECK(oracle_step(&p, n, st, act, NULL, NULL, NULL, NULL, 1, NULL, NULL, NULL, 7, 100, od) == 0);
    }
    double* rs = calloc((size_t)n, sizeof(double));
    CHECK(oracle_step_random(&p, n, st, 3, 7, 100, rs, 2) > 0);
    CHECK(oracle_step_random(&p, n, st, 1, 7, 100, NULL, 1) >= 0);
    /* Robot / Nozzle level + recording */
    CHECK(oracle_robot_reset(&p, n, st, mask) == 0);
    double* ang = calloc((size_t)n * 2, sizeof(double));
    double* yaw = calloc((size_t)n, sizeof(double));
    double* ctl = calloc((size_t)n * 4, sizeof(double));
    for (int i = 0; i < n; ++i) {
        ang[2 * i] = frand(&s) - 0.5;
        ang[2 * i + 1] = frand(&s) - 0.5;
        yaw[i] = 3 * frand(&s) - 1.5;
    }
    CHECK(oracle_nozzle_set_angles(&p, n, st, ang) == 0);
    CHECK(oracle_nozzle_solve(&p, n, st, yaw, 1) == 0);
    CHECK(oracle_nozzle_solve(&p, n, st, yaw, 0) == 0);
    for (int i = 0; i < n; ++i) {
        ctl[4 * i] = 0.06 * frand(&s);
        ctl[4 * i + 1] = 2 * frand(&s);
        ctl[4 * i + 2] = st[SALP_F_ANGLE1 * (size_t)n + i];
        ctl[4 * i + 3] = st[SALP_F_ANGLE2 * (size_t)n + i];
    }
    CHECK(oracle_robot_set_control(&p, n, st, ctl, n % 2, 7, 100) == 0);
    const int64_t ms = 64;
    double* rows = calloc((size_t)ms * SALP_TRACE_DIM * n, sizeof(double));
    int64_t* ns = calloc((size_t)n, sizeof(int64_t));
    CHECK(oracle_robot_cycle(&p, n, st, rows, ms, ns, ticks, 7, 100) == 0);
    for (int i = 0; i < n; ++i) CHECK(ns[i] >= 1);
    CHECK(oracle_robot_cycle(&p, n, st, NULL, 0, NULL, NULL, 7, 100) == 0);
    free(rows); free(ns); free(ang); free(yaw); free(ctl); free(rs);
    free(st); free(obs); free(tobs); free(act); free(rew); free(info); free(te); free(tr); free(mask);
    free(ticks); free(tg); free(ob); free(nob);
}

static void oracle_misc(void) {
    SalpParams p;
    salp_default_params(&p);
    float acts[30];
    for (int i = 0; i < 10; ++i) { acts[3 * i] = 0.1f * i; acts[3 * i + 1] = 0.05f * i; acts[3 * i + 2] = 0.2f * i - 1; }
    double* out = calloc(200000 * 29, sizeof(double));
    CHECK(oracle_robot_trace(&p, acts, 10, out, 200000) > 0);
    CHECK(oracle_robot_trace(&p, acts, 10, out, 3) < 0);   /* too small: reports, no overflow */
    free(out);
    double x[5] = {0.0, -0.0, 1e-300, 3.0, -1e5}, y[5] = {1.0, -2.0, 0.0, INFINITY, 7.0}, m[SALP_MATH_SELFTEST_ROWS * 5];
    oracle_math_selftest(x, y, 5, m);
}

static void abi_host_paths(void) {
    SalpParams p;
    salp_default_params(&p);
    SalpEnv* h = (SalpEnv*)0x1;
    CHECK(salp_abi_version() == SALP_ABI_VERSION);
    CHECK(salp_create(NULL, 8, 0, 0, 0, &h) == SALP_EINVAL && h == (SalpEnv*)0x1);
    CHECK(salp_create(&p, 0, 0, 0, 0, &h) == SALP_EINVAL && h == NULL);
    SalpParams q = p;
    q.num_obstacles = 5;
    CHECK(salp_create(&q, 8, 0, 0, 0, &h) == SALP_EINVAL);
    q = p;
    q.init_length = 0;
    CHECK(salp_create(&q, 8, 0, 0, 0, &h) == SALP_EINVAL);
    CHECK(strlen(salp_last_error(NULL)) > 0);
    CHECK(salp_destroy(NULL) == SALP_OK);
    CHECK(salp_reset(NULL, NULL, NULL, NULL) == SALP_EINVAL);
    CHECK(salp_step(NULL, NULL, NULL, NULL, NULL, NULL, 0, NULL, NULL, NULL) == SALP_EINVAL);
    CHECK(salp_rollout(NULL, 1, NULL, NULL) == SALP_EINVAL);
    CHECK(salp_step_random(NULL, 1, NULL, NULL) == SALP_EINVAL);
    CHECK(salp_num_envs(NULL) == -1 && salp_obs_dim(NULL) == -1);
    CHECK(salp_field_name(-1) == NULL && salp_field_name(SALP_NUM_FIELDS) == NULL);
    CHECK(strcmp(salp_field_name(0), "v0") == 0);
    CHECK(salp_gae(-1, 1, NULL, NULL, NULL, NULL, NULL, 0.99, 0.95, NULL, NULL, NULL) == SALP_EINVAL);
    CHECK(salp_ppo_loss(0, NULL, NULL, NULL, NULL, NULL, NULL, NULL, 0.2, 0, 0.5, 1, NULL, NULL, NULL, NULL, NULL) ==
          SALP_EINVAL);
    CHECK(salp_math_selftest(NULL, NULL, 1, NULL, NULL) == SALP_EINVAL);
    /* fused PPO step: layout queries and argument checks (no GPU) */
    CHECK(salp_ppo_mlp_num_params(10) == 2 * (64 * 10 + 64 + 64 * 64 + 64) + 3 * 64 + 3 + 3 + 64 + 1);
    CHECK(salp_ppo_mlp_offset(10, SALP_MLP_N_TENSORS) == salp_ppo_mlp_num_params(10));
    CHECK(salp_ppo_mlp_num_params(0) == -1 && salp_ppo_mlp_workspace_doubles(0, 10) == -1);
    CHECK(salp_ppo_mlp_grads(NULL, NULL) == SALP_EINVAL);
    CHECK(salp_lstm_cell_forward(4, 0, NULL, NULL, NULL, NULL, NULL, NULL, NULL) == SALP_EINVAL);
    CHECK(salp_lstm_cell_forward(4, 8, NULL, NULL, NULL, NULL, NULL, NULL, NULL) == SALP_EINVAL);
    CHECK(salp_lstm_cell_backward(-1, 8, NULL, NULL, NULL, NULL, NULL, NULL, NULL, NULL, NULL) == SALP_EINVAL);
    CHECK(salp_lstm_step_forward(4, 8, NULL, NULL, NULL, NULL, NULL, NULL, NULL, NULL, NULL, NULL) == SALP_EINVAL);
    CHECK(salp_lstm_step_backward(4, -1, NULL, NULL, NULL, NULL, NULL, NULL, NULL, NULL, NULL, NULL, NULL) ==
          SALP_EINVAL);
    {
        SalpPpoMinibatch mb;
        memset(&mb, 0, sizeof mb);
        mb.batch = 64;
        mb.obs_dim = 10;
        CHECK(salp_ppo_mlp_grads(&mb, NULL) == SALP_EINVAL);   /* null buffers */
        SalpPpoAdam ad;
        memset(&ad, 0, sizeof ad);
        ad.obs_dim = 10;
        CHECK(salp_ppo_mlp_apply(&ad, NULL) == SALP_EINVAL);
        ad.obs_dim = 99;
        CHECK(salp_ppo_mlp_apply(&ad, NULL) == SALP_EINVAL);
    }
}

#ifdef SALP_SAN_GPU
#define HC(x) CHECK((x) == hipSuccess)
static void abi_gpu_run(void) {
    SalpParams p;
    salp_default_params(&p);
    const int n = 300;   /* ragged: not a multiple of the 256-lane workgroup */
    SalpEnv* h = NULL;
    CHECK(salp_create(&p, n, 3, 10, 0, &h) == SALP_OK && h);
    float *act, *obs, *tobs;
    double *rew, *info, *state;
    uint8_t *te, *tr;
    HC(hipMalloc((void**)&act, sizeof(float) * 3 * n));
    HC(hipMalloc((void**)&obs, sizeof(float) * 10 * n));
    HC(hipMalloc((void**)&tobs, sizeof(float) * 10 * n));
    HC(hipMalloc((void**)&rew, sizeof(double) * n));
    HC(hipMalloc((void**)&info, sizeof(double) * SALP_INFO_DIM * n));
    HC(hipMalloc((void**)&state, sizeof(double) * SALP_NUM_FIELDS * n));
    HC(hipMalloc((void**)&te, n));
    HC(hipMalloc((void**)&tr, n));
    float ha[3 * 300];
    for (int i = 0; i < 3 * n; ++i) ha[i] = (i % 3 == 2) ? 0.5f : 0.3f;
    HC(hipMemcpy(act, ha, sizeof ha, hipMemcpyHostToDevice));
    CHECK(salp_reset(h, NULL, obs, NULL) == SALP_OK);
    CHECK(salp_step(h, act, obs, rew, te, tr, 1, tobs, info, NULL) == SALP_OK);
    CHECK(salp_step_random(h, 2, rew, NULL) == SALP_OK);
    SalpRolloutBuffers b;
    memset(&b, 0, sizeof b);
    int64_t* done;
    HC(hipMalloc((void**)&done, sizeof(int64_t) * n));
    HC(hipMemset(done, 0, sizeof(int64_t) * n));
    b.steps_done = done;
    b.chunk = 64;
    CHECK(salp_rollout(h, 500, &b, NULL) == SALP_OK);
    CHECK(salp_get_state(h, state, NULL) == SALP_OK);
    CHECK(salp_set_state(h, state, NULL) == SALP_OK);
    CHECK(salp_set_randomization(h, 1, 1, 1, 1, 1) == SALP_OK);
    CHECK(salp_step(h, act, obs, rew, te, tr, 1, NULL, NULL, NULL) == SALP_OK);
    CHECK(salp_set_randomization(h, 0, 0, 0, 0, 0) == SALP_OK);
    CHECK(salp_robot_reset(h, NULL, NULL) == SALP_OK);
    CHECK(salp_robot_step_through_cycle(h, NULL) == SALP_OK);
    CHECK(salp_rollout(h, -1, &b, NULL) == SALP_EINVAL);
    CHECK(strlen(salp_last_error(h)) > 0);
    HC(hipDeviceSynchronize());
    CHECK(salp_destroy(h) == SALP_OK);
    hipFree(act); hipFree(obs); hipFree(tobs); hipFree(rew); hipFree(info); hipFree(state);
    hipFree(te); hipFree(tr); hipFree(done);
    printf("gpu ABI run ok\n");
}
#endif

int main(int argc, char** argv) {
    const int gpu = argc > 1 && strcmp(argv[1], "--gpu") == 0;
    const int sizes[3] = {1, 7, 64};
    for (int k = 0; k < 3; ++k) {
        oracle_suite(sizes[k], 2, 0);
        oracle_suite(sizes[k], 0, 0);
        oracle_suite(sizes[k], 4, 1);
    }
    oracle_misc();
    abi_host_paths();
    printf("oracle + ABI host paths ok\n");
    if (gpu) {
#ifdef SALP_SAN_GPU
        abi_gpu_run();
#else
        fprintf(stderr, "built without SALP_SAN_GPU\n");
        return 2;
#endif
    }
    return 0;
}
