/*
 * salp_philox.h — Philox4x32-10 counter-based RNG (Salmon et al., SC'11,
 * "Parallel random numbers: as easy as 1, 2, 3") and the fixed mapping from
 * (seed, global env id, counters) to the synthetic action / reset draws.
 *
 * The reference draws actions from the policy (SB3) or gym's Box.sample and
 * targets/obstacles from the process-global MT19937 (src/salp_robot_env.py:
 * 484-487, 547-550) and ignores reset(seed) — neither is reproducible per env
 * in a batch.  Here every draw is a pure function of (seed, env id, counter),
 * so 1/2/4/8-GPU shardings produce bitwise-identical per-env trajectories.
 * Integer-only, so host (oracle) and device agree bit for bit.
 */
#ifndef SALP_PHILOX_H
#define SALP_PHILOX_H

#include <stdint.h>

#if defined(__HIP__)
#include <hip/hip_runtime.h>
#define SP_QUAL __host__ __device__ static inline
#else
#define SP_QUAL static inline
#endif

typedef struct { uint32_t v[4]; } sp_u32x4;

SP_QUAL sp_u32x4 sp_philox4x32_10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                  uint32_t k0, uint32_t k1) {
    const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u, W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
    for (int r = 0; r < 10; ++r) {
        uint64_t p0 = (uint64_t)M0 * c0, p1 = (uint64_t)M1 * c2;
        uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
        c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
        k0 += W0; k1 += W1;
    }
    sp_u32x4 o; o.v[0] = c0; o.v[1] = c1; o.v[2] = c2; o.v[3] = c3;
    return o;
}

/* Stream tags (counter word 3). */
#define SP_STREAM_ACTION 0u
#define SP_STREAM_RESET 1u

/* float32 uniform in [0,1) with 24 random bits. */
SP_QUAL float sp_u01f(uint32_t x) { return (float)(x >> 8) * 0x1.0p-24f; }
/* float64 uniform in [0,1) with 53 random bits. */
SP_QUAL double sp_u01d(uint32_t a, uint32_t b) {
    return ((double)(a >> 5) * 67108864.0 + (double)(b >> 6)) * 0x1.0p-53;
}

/* Synthetic action of env `env_id` at its `step`-th env-step: U(Box([0,0,-1],
 * [1,1,1])) in float32, the distribution of gym's Box.sample for the
 * reference action space (src/salp_robot_env.py:63-67). */
SP_QUAL void sp_action(uint64_t seed, uint64_t env_id, uint64_t step, float a[3]) {
    sp_u32x4 r = sp_philox4x32_10((uint32_t)step, (uint32_t)(step >> 32), (uint32_t)env_id,
                                  SP_STREAM_ACTION | ((uint32_t)(env_id >> 32) << 1),
                                  (uint32_t)seed, (uint32_t)(seed >> 32));
    a[0] = sp_u01f(r.v[0]);
    a[1] = sp_u01f(r.v[1]);
    a[2] = 2.0f * sp_u01f(r.v[2]) - 1.0f;
}

/* Two float64 uniforms for draw `draw` of episode `episode` of env `env_id`
 * (draw 0 = target, draws 1.. = obstacle placement attempts). */
SP_QUAL void sp_reset_pair(uint64_t seed, uint64_t env_id, uint64_t episode, uint32_t draw,
                           double* u0, double* u1) {
    sp_u32x4 r = sp_philox4x32_10((uint32_t)episode, draw, (uint32_t)env_id,
                                  SP_STREAM_RESET | ((uint32_t)(env_id >> 32) << 1),
                                  (uint32_t)seed ^ 0x5A17u, (uint32_t)(seed >> 32));
    *u0 = sp_u01d(r.v[0], r.v[1]);
    *u1 = sp_u01d(r.v[2], r.v[3]);
}

/* ------------------------------------------------ randomisation streams */
/* Domain randomisation, disturbances, action / observation noise and latency
 * (src/robot.py:210-242, 594-628, 796-800, 834-838; src/salp_robot_env.py:
 * 176-194, 293-297) draw from NumPy's global MT19937 in the reference; here
 * from Philox keyed by (seed, stream), counter (ctr, env id, group).  Device
 * and oracle share this mapping, so they agree bit for bit; agreement with the
 * reference is statistical (tests/test_randomization.py). */
#define SP_STREAM_COEF 2u      /* Robot._randomize_parameters, per set_control    */
#define SP_STREAM_NOISE 3u     /* OU disturbance increments, per physics tick     */
#define SP_STREAM_ACTNOISE 4u  /* SalpRobotEnv._randomize_actions, per env-step   */
#define SP_STREAM_OBSNOISE 5u  /* SalpRobotEnv._randomize_observations, per step  */
#define SP_STREAM_LATENCY 6u   /* the latency set_control's coast time, per step  */

SP_QUAL sp_u32x4 sp_draw(uint64_t seed, uint64_t env_id, uint64_t ctr, uint32_t stream, uint32_t group) {
    return sp_philox4x32_10((uint32_t)ctr, (uint32_t)(ctr >> 32), (uint32_t)env_id,
                            ((uint32_t)(env_id >> 32) & 0xFFFFu) | (group << 16),
                            (uint32_t)seed ^ (0x6C8E9CF5u * stream), (uint32_t)(seed >> 32) ^ stream);
}
/* float64 uniform in [0, 1) with 32 random bits (np.random.random_sample
 * stand-in; distributional, not bitwise, parity with the reference). */
SP_QUAL double sp_u01_32(uint32_t x) { return (double)x * 0x1.0p-32; }

#endif /* SALP_PHILOX_H */
