/*
 * salp_random.h — the reference's randomisation features on Philox draws,
 * shared by the device kernels and the CPU oracle (bitwise-identical there).
 *
 *  - Robot._randomize_parameters (src/robot.py:594-628) with
 *    geometry.randomize_scalar_jit (src/geometry.py:207-222): discharge
 *    coefficient, drag ratios and the diagonal added-mass coefficient matrices
 *    ±50 %, redrawn at every set_control;
 *  - OUDisturbance (src/robot.py:210-242, constructed at :279-280): force
 *    (theta 2, sigma 0.05) and torque (theta 2, sigma 0.01) Ornstein-Uhlenbeck
 *    processes stepped every tick in _newton_equations / _euler_equations
 *    (:796-800, :834-838);
 *  - SalpRobotEnv._randomize_actions / _randomize_observations
 *    (src/salp_robot_env.py:176-194) and the latency set_control (:293-297).
 *
 * The reference draws from NumPy's global MT19937, so agreement with it is
 * distributional (tests/test_randomization.py compares against samples of
 * the reference itself); the arithmetic around the draws follows the
 * reference's expressions and NumPy 2's float32 promotion.
 */
#ifndef SALP_RANDOM_H
#define SALP_RANDOM_H

#include "salp_math.h"
#include "salp_philox.h"

#if defined(__HIP__)
#define SR_QUAL __host__ __device__ static inline
#else
#define SR_QUAL static inline
#endif

/* randomize_scalar_jit: uniform(v*(1-u), v*(1+u)) clipped to [lo, hi] (the
 * sample bounds when lo / hi are NaN) with Python's min/max semantics.  u01
 * is the random_sample() of np.random.uniform(low, high) = low + (high-low)*u01. */
SR_QUAL double sr_randomize_scalar(double v, double unc, double lo, double hi, double u01) {
    const double ls = v * (1.0 - unc), us = v * (1.0 + unc);
    if (lo != lo) lo = ls;
    if (hi != hi) hi = us;
    const double s = ls + (us - ls) * u01;
    const double m = lo > s ? lo : s;      /* max(sample, lo) */
    return hi < m ? hi : m;                /* min(., hi)      */
}

/* The randomised coefficients of one set_control (means when off). */
typedef struct SrCoef {
    double cd, dfr, dtr;            /* discharge coefficient, drag force / torque ratios */
    double amf[3], amrf[3];         /* diag of added_mass(_rate)_coefficient_force       */
    double amt[3], amrt[3];         /* diag of added_mass(_rate)_coefficient_torque      */
} SrCoef;

/* src/robot.py:300-306 */
SR_QUAL void sr_coef_means(SrCoef* k) {
    k->cd = 0.3; k->dfr = 0.25; k->dtr = 0.1;
    k->amf[0] = 0.5; k->amf[1] = 0.6; k->amf[2] = 0.6;
    k->amrf[0] = 0.2; k->amrf[1] = 0.2; k->amrf[2] = 0.2;
    k->amt[0] = 0.3; k->amt[1] = 0.6; k->amt[2] = 0.6;
    k->amrt[0] = 0.2; k->amrt[1] = 0.2; k->amrt[2] = 0.2;
}
/* np.random.uniform(mean * (1 - 0.5), mean * (1 + 0.5)) on a diagonal matrix:
 * the off-diagonal draws are uniform(0, 0) = 0. */
SR_QUAL double sr_uniform_pm50(double mean, double u01) {
    const double lo = mean * (1 - 0.5), hi = mean * (1 + 0.5);
    return lo + (hi - lo) * u01;
}
/* Robot._randomize_parameters (src/robot.py:594-628); ctr = the env's
 * set_control counter. */
SR_QUAL void sr_draw_coefs(uint64_t seed, uint64_t env_id, uint64_t ctr, SrCoef* k) {
    SrCoef m;
    sr_coef_means(&m);
    const sp_u32x4 a = sp_draw(seed, env_id, ctr, SP_STREAM_COEF, 0);
    const sp_u32x4 b = sp_draw(seed, env_id, ctr, SP_STREAM_COEF, 1);
    const sp_u32x4 c = sp_draw(seed, env_id, ctr, SP_STREAM_COEF, 2);
    const sp_u32x4 d = sp_draw(seed, env_id, ctr, SP_STREAM_COEF, 3);
    k->cd = sr_randomize_scalar(m.cd, 0.5, 0.0, 1.0, sp_u01_32(a.v[0]));
    k->dfr = sr_randomize_scalar(m.dfr, 0.5, NAN, NAN, sp_u01_32(a.v[1]));
    k->dtr = sr_randomize_scalar(m.dtr, 0.5, NAN, NAN, sp_u01_32(a.v[2]));
    const uint32_t w[12] = {a.v[3], b.v[0], b.v[1], b.v[2], b.v[3], c.v[0],
                            c.v[1], c.v[2], c.v[3], d.v[0], d.v[1], d.v[2]};
    for (int j = 0; j < 3; ++j) {
        k->amf[j] = sr_uniform_pm50(m.amf[j], sp_u01_32(w[j]));
        k->amrf[j] = sr_uniform_pm50(m.amrf[j], sp_u01_32(w[3 + j]));
        k->amt[j] = sr_uniform_pm50(m.amt[j], sp_u01_32(w[6 + j]));
        k->amrt[j] = sr_uniform_pm50(m.amrt[j], sp_u01_32(w[9 + j]));
    }
}

/* Three standard normals for tick `ctr` (Box-Muller on two Philox pairs):
 * force-noise x, y and torque-noise z, the components the reference keeps. */
SR_QUAL void sr_normals3(uint64_t seed, uint64_t env_id, uint64_t ctr, double* n0, double* n1,
                         double* n2) {
    const double two_pi = 6.283185307179586;
    const sp_u32x4 r = sp_draw(seed, env_id, ctr, SP_STREAM_NOISE, 0);
    const double u1 = ((double)r.v[0] + 1.0) * 0x1.0p-32;      /* (0, 1] */
    const double u3 = ((double)r.v[2] + 1.0) * 0x1.0p-32;
    const double rad1 = sqrt(-2.0 * sm_log(u1)), rad2 = sqrt(-2.0 * sm_log(u3));
    double s1, c1, s2, c2;
    sm_sincos(two_pi * sp_u01_32(r.v[1]), &s1, &c1);
    sm_sincos(two_pi * sp_u01_32(r.v[3]), &s2, &c2);
    *n0 = rad1 * c1;
    *n1 = rad1 * s1;
    *n2 = rad2 * c2;
    (void)s2;
}

/* OUDisturbance.sample, one component (mu = 0, dt = 0.01):
 * x + (theta * (mu - x) * dt + sigma * sqrt(dt) * n). */
SR_QUAL double sr_ou_step(double x, double theta, double sigma, double n) {
    const double dx = theta * (0.0 - x) * 0.01 + sigma * sqrt(0.01) * n;
    return x + dx;
}
#define SR_OU_FORCE_THETA 2.0
#define SR_OU_FORCE_SIGMA 0.05
#define SR_OU_TORQUE_THETA 2.0
#define SR_OU_TORQUE_SIGMA 0.01

/* _randomize_actions (src/salp_robot_env.py:176-181) of the float32 rescaled
 * action r: float32 sample bounds (np.float32 * Python float), float64 result
 * (np.random.uniform returns a Python float). */
SR_QUAL void sr_randomize_action(uint64_t seed, uint64_t env_id, uint64_t ctr, const float r[3], double out[3]) {
    const sp_u32x4 a = sp_draw(seed, env_id, ctr, SP_STREAM_ACTNOISE, 0);
    const double lo[3] = {0.0, 0.0, -3.141592653589793 / 2};
    const double hi[3] = {1.0, 20.0, 3.141592653589793 / 2};
    for (int k = 0; k < 3; ++k) {
        const float ls = r[k] * (float)(1.0 - 0.1), us = r[k] * (float)(1.0 + 0.1);
        const double s = (double)ls + ((double)us - (double)ls) * sp_u01_32(a.v[k]);
        const double m = lo[k] > s ? lo[k] : s;
        out[k] = hi[k] < m ? hi[k] : m;
    }
}

/* _randomize_observations (src/salp_robot_env.py:183-194) of the first six
 * float32 observation entries, in place.  With no explicit bounds a negative
 * entry always comes out as v * (1 + u) (the clip bounds are the sample bounds
 * in reverse order), as in the reference. */
SR_QUAL void sr_randomize_obs(uint64_t seed, uint64_t env_id, uint64_t ctr, float* obs) {
    const double unc[6] = {0.05, 0.05, 0.2, 0.2, 0.02, 0.1};
    const sp_u32x4 a = sp_draw(seed, env_id, ctr, SP_STREAM_OBSNOISE, 0);
    const sp_u32x4 b = sp_draw(seed, env_id, ctr, SP_STREAM_OBSNOISE, 1);
    const uint32_t w[6] = {a.v[0], a.v[1], a.v[2], a.v[3], b.v[0], b.v[1]};
    for (int k = 0; k < 6; ++k) {
        const float ls = obs[k] * (float)(1.0 - unc[k]), us = obs[k] * (float)(1.0 + unc[k]);
        const double s = (double)ls + ((double)us - (double)ls) * sp_u01_32(w[k]);
        const double m = (double)ls > s ? (double)ls : s;
        obs[k] = (float)((double)us < m ? (double)us : m);
    }
}

/* The latency coast time randomize_scalar_jit(0.05, 1.0) (src/salp_robot_env.py:294-295). */
SR_QUAL double sr_latency(uint64_t seed, uint64_t env_id, uint64_t ctr) {
    const sp_u32x4 a = sp_draw(seed, env_id, ctr, SP_STREAM_LATENCY, 0);
    return sr_randomize_scalar(0.05, 1.0, NAN, NAN, sp_u01_32(a.v[0]));
}

#endif /* SALP_RANDOM_H */
