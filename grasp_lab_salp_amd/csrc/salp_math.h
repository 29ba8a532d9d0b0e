/*
 * salp_math.h — portable, bit-reproducible fp64/fp32 elementary functions and
 * the NumPy/OpenBLAS evaluation-order primitives the reference's arithmetic
 * goes through.
 *
 * Why this exists.  The reference (Avielstein/GRASP_LAB_SALP, src/ Python) runs
 * its physics through NumPy.  Two facts about that arithmetic shape the design:
 *
 *  1. Every 3x3 product, mat-vec and norm in the reference is a BLAS call on
 *     NumPy 2.2 + OpenBLAS, and those kernels accumulate with FMA in a fixed
 *     order.  Probed in the build container (tests/test_numpy_semantics.py pins
 *     it):
 *        np.linalg.norm(v)      = sqrt(fma(v2,v2, fma(v1,v1, v0*v0)))
 *        (A @ B)[i,j]           = fma(A[i,2],B[2,j], fma(A[i,1],B[1,j], A[i,0]*B[0,j]))
 *        (A.T @ v)[i]           = fma(A[2,i],v2, fma(A[1,i],v1, A[0,i]*v0))
 *        (A @ v)[i]  (C-contig) = fma(A[i,2],v2, fma(A[i,0],v0, A[i,1]*v1))
 *        np.linalg.solve(diag(d), b) = b / d
 *     The np_* helpers below restate exactly those orders, so the device
 *     kernel and the CPU oracle both reproduce the reference's rounding.
 *
 *  2. The nozzle inverse kinematics (src/robot.py:71-98) feed float32
 *     cos/sin of the yaw into arcsin() right next to |x|=1, where a one-ulp
 *     change of the float32 inputs moves angle1 by ~1e-4 rad.  NumPy's float32
 *     sin/cos is its own SIMD algorithm (Cody-Waite reduction + minimax
 *     polynomials evaluated with fmaf; NumPy >= 1.22 loops_trigonometric) and
 *     is not correctly rounded, so sm_np_sincosf() restates that published
 *     algorithm bit for bit (0 mismatches over the action range, see tests).
 *
 * The fp64 transcendentals (sin, cos, tan, atan, atan2, asin, acos) are
 * fdlibm-style (Cody-Waite pi/2 reduction, minimax kernels) and accurate to
 * about one ulp; glibc/SVML, which the reference uses, are not reproducible
 * bit for bit on a GPU, so oracle-vs-reference agreement is ulp-level there
 * (DESIGN.md §Parity).  The device kernel and the oracle include THIS header,
 * so device-vs-oracle comparisons are exact.
 *
 * Everything here uses only IEEE-754 correctly rounded operations (+ - * /
 * sqrt, fma, rint, conversions) so gcc (x86-64, -ffp-contract=off) and hipcc
 * (gfx950, -ffp-contract=off) produce identical bits.
 */
#ifndef SALP_MATH_H
#define SALP_MATH_H

#include <stdint.h>

#if defined(__HIP__)
#include <hip/hip_runtime.h>
#define SM_QUAL __host__ __device__ static inline
#else
#include <math.h>
#include <string.h>
#define SM_QUAL static inline
#endif

#if defined(__clang__)
#pragma clang fp contract(off)
#endif

/* ---------------------------------------------------------------- bits */
SM_QUAL uint64_t sm_d2u(double x) {
#if defined(__HIP_DEVICE_COMPILE__)
    return (uint64_t)__double_as_longlong(x);
#else
    uint64_t u; memcpy(&u, &x, 8); return u;
#endif
}
SM_QUAL double sm_u2d(uint64_t u) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __longlong_as_double((long long)u);
#else
    double x; memcpy(&x, &u, 8); return x;
#endif
}
SM_QUAL int32_t sm_hi(double x) { return (int32_t)(sm_d2u(x) >> 32); }

SM_QUAL double sm_fma(double a, double b, double c) { return fma(a, b, c); }
SM_QUAL float sm_fmaf(float a, float b, float c) { return fmaf(a, b, c); }

/* a * b + c at the points where the reference's NumPy expression is a
 * product feeding a sum.  SALP_FMA = 1 (the default, device and oracle
 * alike): fused, one rounding.  SALP_FMA = 0: NumPy's two roundings, the
 * exact elementwise semantics of the reference (every other operation is the
 * same in both modes).  The two modes differ by at most an ulp per such
 * operation; tests/test_fma_mode.py measures how far that carries over whole
 * episodes, tests/test_oracle_golden.py pins both against the reference.  The
 * device and the oracle are always built in the same mode, so they agree bit
 * for bit in either. */
#ifndef SALP_FMA
#define SALP_FMA 1
#endif
SM_QUAL double sm_mad(double a, double b, double c) {
#if SALP_FMA
    return fma(a, b, c);
#else
    return a * b + c;
#endif
}

/* ------------------------------------------------ NumPy/OpenBLAS orders */
/* np.linalg.norm of a 3-vector / 2-vector (ddot FMA chain, then sqrt). */
SM_QUAL double np_norm3(double a, double b, double c) {
    return sqrt(sm_fma(c, c, sm_fma(b, b, a * a)));
}
SM_QUAL double np_norm2(double a, double b) { return sqrt(sm_fma(b, b, a * a)); }
/* One entry of a 3x3 @ 3x3 product, or of a transposed mat-vec. */
SM_QUAL double np_dot_fwd(double a0, double a1, double a2, double b0, double b1, double b2) {
    return sm_fma(a2, b2, sm_fma(a1, b1, a0 * b0));
}
/* One row of a C-contiguous 3x3 @ 3-vector (dgemv) product. */
SM_QUAL double np_matvec_row(double a0, double a1, double a2, double v0, double v1, double v2) {
    return sm_fma(a2, v2, sm_fma(a0, v0, a1 * v1));
}
/* Correctly rounded x**3 (glibc pow agrees except in ~1e-3 of inputs). */
SM_QUAL double sm_cube(double x) {
    double p = x * x, pe = sm_fma(x, x, -p);
    double h = p * x, he = sm_fma(p, x, -h);
    return h + sm_fma(pe, x, he);
}

/* ------------------------------------------- NumPy float32 sin / cos */
/* NumPy SIMD float32 sin/cos: quadrant by x*(2/pi) rounded with the 1.5*2^23
 * magic constant, three-constant Cody-Waite reduction with fmaf, and the
 * degree-8 cos / degree-9 sin minimax polynomials in r^2. */
SM_QUAL void sm_np_sincosf(float x, float* s_out, float* c_out) {
    const float two_over_pi = 0x1.45f306p-01f;
    const float magic = 0x1.800000p+23f;
    const float pio2_hi = -0x1.921fb0p+00f;
    const float pio2_med = -0x1.5110b4p-22f;
    const float pio2_lo = -0x1.846988p-48f;
    float q = x * two_over_pi;
    q = q + magic;
    q = q - magic;
    float r = sm_fmaf(q, pio2_hi, x);
    r = sm_fmaf(q, pio2_med, r);
    r = sm_fmaf(q, pio2_lo, r);
    float r2 = r * r;
    float c = sm_fmaf(0x1.98e616p-16f, r2, -0x1.6c06dcp-10f);
    c = sm_fmaf(c, r2, 0x1.55553cp-05f);
    c = sm_fmaf(c, r2, -0x1.000000p-01f);
    c = sm_fmaf(c, r2, 0x1.000000p+00f);
    float s = sm_fmaf(0x1.7d3bbcp-19f, r2, -0x1.a06bbap-13f);
    s = sm_fmaf(s, r2, 0x1.11119ap-07f);
    s = sm_fmaf(s, r2, -0x1.555556p-03f);
    s = s * r2;
    s = sm_fmaf(s, r, r);
    int iq = (int)q;
    /* sine: quadrant iq; cosine: quadrant iq+1 */
    float sv = (iq & 1) ? c : s;
    if (iq & 2) sv = -sv;
    int iqc = iq + 1;
    float cv = (iqc & 1) ? c : s;
    if (iqc & 2) cv = -cv;
    *s_out = sv;
    *c_out = cv;
}

/* ------------------------------------------------- fp64 sin/cos (fdlibm) */
/* The kernel polynomials' coefficients (fdlibm __kernel_sin / __kernel_cos).
 * Passed by value so that a hot loop can hand in a copy kept in VGPRs
 * (salp_device.h pin_params): gfx950 has no 64-bit literal operands, and
 * pinning each use separately costs a v_mov_b64 per coefficient per call. */
typedef struct {
    double S1, S2, S3, S4, S5, S6, C1, C2, C3, C4, C5, C6;
    double R_INV, R_P1, R_P1T;   /* sm_rem_pio2's common-path constants: 2/pi, pio2_1, pio2_1t */
} SmPoly;
SM_QUAL SmPoly sm_poly(void) {
    SmPoly k = {-1.66666666666666324348e-01, 8.33333333332248946124e-03, -1.98412698298579493134e-04,
                2.75573137070700676789e-06,  -2.50507602534068634195e-08, 1.58969099521155010221e-10,
                4.16666666666666019037e-02,  -1.38888888888741095749e-03, 2.48015872894767294178e-05,
                -2.75573143513906633035e-07, 2.08757232129817482790e-09,  -1.13596475577881948265e-11,
                6.36619772367581382433e-01,  1.57079632673412561417e+00,  6.07710050650619224932e-11};
    return k;
}
/* fdlibm's kernels with the polynomial steps written as sm_mad: with
 * SALP_FMA = 0 each line is fdlibm's expression exactly
 * (r = S2 + z*(S3 + z*S4) + z*w*(S5 + z*S6), ...). */
SM_QUAL double sm_ksin_r(double z, double w, SmPoly K) {
    return sm_mad(z * w, sm_mad(z, K.S6, K.S5), sm_mad(z, sm_mad(z, K.S4, K.S3), K.S2));
}
/* x - ((z*(0.5*y - v*r) - y) - v*S1) */
SM_QUAL double sm_ksin_tail(double x, double y, double z, double v, double r, SmPoly K) {
    return x - sm_mad(-v, K.S1, sm_mad(z, sm_mad(-v, r, 0.5 * y), -y));
}
SM_QUAL double sm_ksin_p(double x, double y, int iy, SmPoly K) {
    double z = x * x, w = z * z;
    double r = sm_ksin_r(z, w, K);
    double v = z * x;
    if (iy == 0) return sm_mad(v, sm_mad(z, r, K.S1), x);
    return sm_ksin_tail(x, y, z, v, r, K);
}
SM_QUAL double sm_kcos_p(double x, double y, SmPoly K) {
    double z = x * x, w = z * z;
    /* z*(C1 + z*(C2 + z*C3)) + w*w*(C4 + z*(C5 + z*C6)) */
    double r = sm_mad(z, sm_mad(z, sm_mad(z, K.C3, K.C2), K.C1), (w * w) * sm_mad(z, sm_mad(z, K.C6, K.C5), K.C4));
    double hz = 0.5 * z;
    w = 1.0 - hz;
    return w + (((1.0 - w) - hz) + sm_mad(z, r, -(x * y)));
}
SM_QUAL double sm_ksin(double x, double y, int iy) { return sm_ksin_p(x, y, iy, sm_poly()); }
SM_QUAL double sm_kcos(double x, double y) { return sm_kcos_p(x, y, sm_poly()); }
/* Cody-Waite reduction for |x| < 2^20*pi/2 (fdlibm __ieee754_rem_pio2,
 * medium case).  Returns n with x = n*pi/2 + (y0 + y1). */
SM_QUAL int sm_rem_pio2_p(double x, double* y0, double* y1, SmPoly K) {
    const double invpio2 = K.R_INV, pio2_1 = K.R_P1, pio2_1t = K.R_P1T,
                 pio2_2 = 6.07710050630396597660e-11, pio2_2t = 2.02226624879595063154e-21,
                 pio2_3 = 2.02226624871116645580e-21, pio2_3t = 8.47842766036889956997e-32;
    double fn = rint(x * invpio2);
    /* fn * pio2_1 is exact while |fn| < 2^20 (33-bit pio2_1), so the unfused
     * and the fused form agree there; beyond (|x| > 1.6e6, tumbling or
     * diverging envs) only the fused one keeps the product exact, and the
     * unfused one lost ~ulp(x) of the angle (NumPy mode 1e-5 off the
     * reference at 1e10 rad, tests/test_oracle_tumble.py).  Fused in both
     * modes: this is libm's reduction, not a NumPy expression. */
    double r = sm_fma(-fn, pio2_1, x);
    double w = fn * pio2_1t;
    double y = r - w;
    int j = (sm_hi(x) >> 20) & 0x7ff;
    int i = j - ((sm_hi(y) >> 20) & 0x7ff);
    if (i > 16) {
        double t = r;
        w = fn * pio2_2;
        r = t - w;
        w = fn * pio2_2t - ((t - r) - w);
        y = r - w;
        i = j - ((sm_hi(y) >> 20) & 0x7ff);
        if (i > 49) {
            t = r;
            w = fn * pio2_3;
            r = t - w;
            w = fn * pio2_3t - ((t - r) - w);
            y = r - w;
        }
    }
    *y0 = y;
    *y1 = (r - y) - w;
    /* The quadrant fn mod 4, exactly, for every fn: (int)fn is undefined in C
     * (and saturates on the GPU) once |fn| >= 2^31, which a diverged env's
     * angle reaches (UBSan, tools/sanitize).  Callers only use n & 3; for
     * |fn| < 2^31 this is exactly (int)fn & 3.  (Beyond |x| = 2^20 pi/2 the
     * later stages' products are no longer exact, so the reduction loses
     * its guarantee, as fdlibm's medium branch does where fdlibm switches to
     * Payne-Hanek; measured against the reference up to 1e11 rad it stays
     * within the tumble fixtures' tolerances.) */
    const double q = fn - 4.0 * floor(fn * 0.25);
    return q == q ? (int)q : 0;
}
SM_QUAL int sm_rem_pio2(double x, double* y0, double* y1) { return sm_rem_pio2_p(x, y0, y1, sm_poly()); }
SM_QUAL void sm_sincos_p(double x, double* s_out, double* c_out, SmPoly K) {
    int32_t ix = sm_hi(x) & 0x7fffffff;
    /* |x| <= pi/4, or x is NaN: the kernels return NaN for it as the
     * reduction would, and a diverged env's NaN angle then does not drag its
     * whole wave through the reduction path (roll and pitch of every finite
     * env stay far below pi/4).  +-inf still takes the reduction (NaN). */
    if (ix <= 0x3fe921fb || x != x) {
        *s_out = sm_ksin_p(x, 0.0, 0, K);
        *c_out = sm_kcos_p(x, 0.0, K);
        return;
    }
    double y0, y1;
    int n = sm_rem_pio2_p(x, &y0, &y1, K);
    double s = sm_ksin_p(y0, y1, 1, K), c = sm_kcos_p(y0, y1, K);
    switch (n & 3) {
        case 0: *s_out = s; *c_out = c; break;
        case 1: *s_out = c; *c_out = -s; break;
        case 2: *s_out = -s; *c_out = -c; break;
        default: *s_out = -c; *c_out = s; break;
    }
}
/* sm_sincos_p without the |x| <= pi/4 branch: every lane runs the reduction,
 * lanes below pi/4 then take (x, 0, quadrant 0) and the iy == 0 form of the sin
 * kernel (the cos kernel with y = 0 is that form already: x * 0 is exact).
 * Bit-identical to sm_sincos_p; cheaper where a wave holds both kinds of
 * argument (the yaw, uniform over the circle), since the branchy version then
 * runs both paths. */
SM_QUAL void sm_sincos_nb_p(double x, double* s_out, double* c_out, SmPoly K) {
    const int small = (sm_hi(x) & 0x7fffffff) <= 0x3fe921fb;
    double y0, y1;
    int n = sm_rem_pio2_p(x, &y0, &y1, K);
    if (small) { y0 = x; y1 = 0.0; n = 0; }
    const double z = y0 * y0, w = z * z;
    const double r = sm_ksin_r(z, w, K);
    const double v = z * y0;
    const double s = small ? sm_mad(v, sm_mad(z, r, K.S1), y0) : sm_ksin_tail(y0, y1, z, v, r, K);
    const double c = sm_kcos_p(y0, y1, K);
    const int q = n & 3;
    const double a = (q & 1) ? c : s, b = (q & 1) ? s : c;
    *s_out = (q & 2) ? -a : a;
    *c_out = ((q + 1) & 2) ? -b : b;
}
SM_QUAL void sm_sincos(double x, double* s_out, double* c_out) { sm_sincos_p(x, s_out, c_out, sm_poly()); }

/* ------------------------- the tick's sin/cos (round 5, SALP_FMA = 1) */
/* The physics tick takes sin and cos of the three Euler angles every tick
 * (src/dynamics.py:20-58): 21 % of k_rollout's executed instructions
 * (profiles/r5a_ablation.json).  In the product mode (SALP_FMA = 1) the tick,
 * the world-frame rotation and the Euler-rate map use the two functions below
 * on both sides (device and oracle include this header), so the device still
 * equals the oracle bit for bit; SALP_FMA = 0 keeps fdlibm's sm_sincos_p for
 * every angle.  Both are within one ulp of sin / cos (tests/test_math.py), so
 * the oracle stays inside the golden tolerances against the reference's own
 * NumPy (glibc) sin / cos (tests/test_oracle_golden.py). */

/* sin / cos of roll x0 and pitch x1 together (round 6): the yaw's
 * branch-free sm_sincos_yaw_p for both, whatever their size (fdlibm's
 * sm_sincos_p without SALP_FMA).  Round 5 ran fdlibm's first four kernel terms
 * while both |x| <= 1/16 and the yaw's function otherwise; in the steady state ~4 %
 * of the envs tumble (|roll| or |pitch| > 1/16) and they sit in ~965 of 1 024
 * waves (profiles/r5am_angle_census.json), so nearly every wave ran both
 * paths.  One path for every lane: +12 % steady state on the headline
 * (profiles/r5_experiments.md r5ao).  r5ao's split-invariance failure was NaN
 * signs only: a diverged lane's NaN carries a sign bit that depends on which
 * tick instance (full / steady / settled: negation modifiers on other
 * operands) the lane ran, i.e. on its wave; every value that is not NaN is
 * identical (profiles/r6c_split_probe_r5ao.json), and NaN signs and payloads
 * are not part of the reference's results (tests compare NaN as NaN). */
SM_QUAL void sm_sincos_yaw_p(double x, double* s_out, double* c_out, SmPoly K);
SM_QUAL void sm_sincos_rp2(double x0, double x1, double* s0, double* c0, double* s1, double* c1, SmPoly K) {
    sm_sincos_yaw_p(x0, s0, c0, K);
    sm_sincos_yaw_p(x1, s1, c1, K);
}
/* sin / cos of the yaw (any size: the heading is uniform over the circle).
 * fdlibm's reduction and kernels, streamlined for a SIMD lane (every step is
 * branch-free):
 *  - fn = rint(x 2/pi) and the quadrant come from one add of 1.5 * 2^52:
 *    fn is in the low bits of x 2/pi + 1.5 * 2^52 (exact for |fn| < 2^51);
 *  - one Cody-Waite stage (pio2_1, pio2_1t).  fdlibm adds a second and third
 *    stage when more than 16 bits cancel (x within |x| 2^-16 of a multiple of
 *    pi/2); the fused first stage keeps fn * pio2_1 exact for every fn, so
 *    the absolute error is below 1.5e-26 |fn| (pio2_1t's own truncation):
 *    within one ulp unless |y| < |fn| 1e-10 for |x| <= 2^20 pi/2, within
 *    1.5e-26 |fn| + ulp(1) up to |x| < 2^51 pi/2 (~3.5e15).  Beyond that the
 *    magic-add quadrant breaks and the result is not sin / cos (values up
 *    to 1e176, NaN from ~1e100): only an env whose state is already
 *    diverging gets there (finite angles seen: <= 3.9e11), the device still
 *    equals the oracle, and the reference's pin reaches 1e11 rad
 *    (tests/test_math.py test_tick_yaw_sincos_large_angles,
 *    tests/test_oracle_tumble.py);
 *  - the tail forms of the kernels for every argument (y1 = 0 when fn = 0);
 *  - quadrant swap as selects, the two signs as bit flips.
 * Differs from sm_sincos_p by at most an ulp. */
SM_QUAL void sm_sincos_yaw_p(double x, double* s_out, double* c_out, SmPoly K) {
#if SALP_FMA
    const double magic = 0x1.8p52;
    const double t = x * K.R_INV + magic;
    const double fn = t - magic;
    const uint32_t q = (uint32_t)sm_d2u(t) & 3u;
    const double r = sm_mad(-fn, K.R_P1, x);   /* the fused product is exact for every fn */
    const double w = fn * K.R_P1T;
    const double y0 = r - w;
    const double y1 = (r - y0) - w;
    const double z = y0 * y0, zz = z * z;
    const double s = sm_ksin_tail(y0, y1, z, z * y0, sm_ksin_r(z, zz, K), K);
    const double c = sm_kcos_p(y0, y1, K);
    const double a = (q & 1u) ? c : s, b = (q & 1u) ? s : c;
    *s_out = sm_u2d(sm_d2u(a) ^ ((uint64_t)(q & 2u) << 62));
    *c_out = sm_u2d(sm_d2u(b) ^ ((uint64_t)((q + 1u) & 2u) << 62));
#else
    sm_sincos_p(x, s_out, c_out, K);
#endif
}

/* R v for R = Rz(psi) Ry(theta) Rx(phi) (src/dynamics.py:34-58), given the
 * sin / cos of the three angles.  SALP_FMA = 1: the three plane rotations
 * applied in turn, Rz (Ry (Rx v)), 12 operations, each component one product
 * fused into a sum; the same vector up to rounding as NumPy's (R_z @ R_y @
 * R_x) @ v, which builds the matrix first (the oracle's SALP_FMA = 0 path). */
SM_QUAL void sm_world_frame(double sp, double cp, double st, double ct, double ss, double cs, double v0,
                            double v1, double v2, double* o) {
    const double x1 = sm_fma(cp, v1, -(sp * v2)), x2 = sm_fma(sp, v1, cp * v2);   /* Rx v */
    const double y0 = sm_fma(ct, v0, st * x2), y2 = sm_fma(-st, v0, ct * x2);     /* Ry (Rx v) */
    o[0] = sm_fma(cs, y0, -(ss * x1));                                          /* Rz (Ry (Rx v)) */
    o[1] = sm_fma(ss, y0, cs * x1);
    o[2] = y2;
}
SM_QUAL double sm_sin(double x) { double s, c; sm_sincos(x, &s, &c); return s; }
SM_QUAL double sm_cos(double x) { double s, c; sm_sincos(x, &s, &c); return c; }
SM_QUAL double sm_tan(double x) { double s, c; sm_sincos(x, &s, &c); return s / c; }

/* ----------------------------------------------------- atan family */
/* fdlibm's atan: the branchy original (sm_atan_ref, kept as the test's
 * reference) and the form the product uses, with its five argument ranges
 * chosen by selects and ONE division instead of a branch per range (a wave
 * whose lanes span the ranges ran every range's path: env-step boundaries
 * take five atan2 per env, src/robot.py:79-93, src/salp_robot_env.py:370,
 * 668).  Every operation is the original's on the same operands (x / 1 is
 * exact), so the two are equal bit for bit (tests/test_math.py). */
SM_QUAL double sm_atan(double x) {
    const double atanhi0 = 4.63647609000806093515e-01, atanhi1 = 7.85398163397448278999e-01,
                 atanhi2 = 9.82793723247329054082e-01, atanhi3 = 1.57079632679489655800e+00;
    const double atanlo0 = 2.26987774529616870924e-17, atanlo1 = 3.06161699786838301793e-17,
                 atanlo2 = 1.39033110312309984516e-17, atanlo3 = 6.12323399573676603587e-17;
    const double aT0 = 3.33333333333329318027e-01, aT1 = -1.99999999998764832476e-01,
                 aT2 = 1.42857142725034663711e-01, aT3 = -1.11111104054623557880e-01,
                 aT4 = 9.09088713343650656196e-02, aT5 = -7.69187620504482999495e-02,
                 aT6 = 6.66107313738753120669e-02, aT7 = -5.83357013379057348645e-02,
                 aT8 = 4.97687799461593236017e-02, aT9 = -3.65315727442169155270e-02,
                 aT10 = 1.62858201153657823623e-02;
    const int32_t hx = sm_hi(x), ix = hx & 0x7fffffff;
    const double ax = fabs(x);
    const int small = ix < 0x3fdc0000;                  /* |x| < 0.4375: id -1, no reduction */
    const int r0 = ix < 0x3fe60000, r1 = ix < 0x3ff30000, r2 = ix < 0x40038000;
    /* id 0: (2x - 1) / (2 + x); 1: (x - 1) / (x + 1); 2: (x - 1.5) / (1 + 1.5x); 3: -1 / x */
    const double num = small ? x : r0 ? 2.0 * ax - 1.0 : r1 ? ax - 1.0 : r2 ? ax - 1.5 : -1.0;
    const double den = small ? 1.0 : r0 ? 2.0 + ax : r1 ? ax + 1.0 : r2 ? 1.0 + 1.5 * ax : ax;
    const double t = num / den;
    const double z = t * t, w = z * z;
    const double s1 = z * (aT0 + w * (aT2 + w * (aT4 + w * (aT6 + w * (aT8 + w * aT10)))));
    const double s2 = w * (aT1 + w * (aT3 + w * (aT5 + w * (aT7 + w * aT9))));
    const double hi = r0 ? atanhi0 : r1 ? atanhi1 : r2 ? atanhi2 : atanhi3;
    const double lo = r0 ? atanlo0 : r1 ? atanlo1 : r2 ? atanlo2 : atanlo3;
    const double zr = hi - ((t * (s1 + s2) - lo) - t);
    const double big = atanhi3 + atanlo3;               /* |x| >= 2^66 */
    double r = small ? (ix < 0x3e400000 ? x : t - t * (s1 + s2)) : (hx < 0 ? -zr : zr);
    if (ix >= 0x44100000) r = hx < 0 ? -big : big;
    return r;
}
SM_QUAL double sm_atan_ref(double x) {
    const double atanhi[4] = {4.63647609000806093515e-01, 7.85398163397448278999e-01,
                              9.82793723247329054082e-01, 1.57079632679489655800e+00};
    const double atanlo[4] = {2.26987774529616870924e-17, 3.06161699786838301793e-17,
                              1.39033110312309984516e-17, 6.12323399573676603587e-17};
    const double aT0 = 3.33333333333329318027e-01, aT1 = -1.99999999998764832476e-01,
                 aT2 = 1.42857142725034663711e-01, aT3 = -1.11111104054623557880e-01,
                 aT4 = 9.09088713343650656196e-02, aT5 = -7.69187620504482999495e-02,
                 aT6 = 6.66107313738753120669e-02, aT7 = -5.83357013379057348645e-02,
                 aT8 = 4.97687799461593236017e-02, aT9 = -3.65315727442169155270e-02,
                 aT10 = 1.62858201153657823623e-02;
    int32_t hx = sm_hi(x), ix = hx & 0x7fffffff;
    int id;
    if (ix >= 0x44100000) { /* |x| >= 2^66 */
        double z = atanhi[3] + atanlo[3];
        return hx < 0 ? -z : z;
    }
    if (ix < 0x3fdc0000) { /* |x| < 0.4375 */
        if (ix < 0x3e400000) return x;
        id = -1;
    } else {
        x = fabs(x);
        if (ix < 0x3ff30000) {
            if (ix < 0x3fe60000) { id = 0; x = (2.0 * x - 1.0) / (2.0 + x); }
            else { id = 1; x = (x - 1.0) / (x + 1.0); }
        } else {
            if (ix < 0x40038000) { id = 2; x = (x - 1.5) / (1.0 + 1.5 * x); }
            else { id = 3; x = -1.0 / x; }
        }
    }
    double z = x * x, w = z * z;
    double s1 = z * (aT0 + w * (aT2 + w * (aT4 + w * (aT6 + w * (aT8 + w * aT10)))));
    double s2 = w * (aT1 + w * (aT3 + w * (aT5 + w * (aT7 + w * aT9))));
    if (id < 0) return x - x * (s1 + s2);
    z = atanhi[id] - ((x * (s1 + s2) - atanlo[id]) - x);
    return hx < 0 ? -z : z;
}
SM_QUAL double sm_atan2(double y, double x) {
    const double pi = 3.1415926535897931160e+00, pi_o_2 = 1.5707963267948965580e+00,
                 pi_lo = 1.2246467991473531772e-16;
    if (x != x || y != y) return x + y;
    if (x == 1.0) return sm_atan(y);
    int32_t hx = sm_hi(x), hy = sm_hi(y);
    int m = ((hy >> 31) & 1) | ((hx >> 30) & 2);
    if (y == 0.0) {
        switch (m) {
            case 0: case 1: return y;
            case 2: return pi;
            default: return -pi;
        }
    }
    if (x == 0.0) return hy < 0 ? -pi_o_2 : pi_o_2;
    int32_t ix = hx & 0x7fffffff, iy = hy & 0x7fffffff;
    int k = (iy - ix) >> 20;
    double z;
    if (k > 60) { z = pi_o_2 + 0.5 * pi_lo; m &= 1; }
    else if (hx < 0 && k < -60) z = 0.0;
    else z = sm_atan(fabs(y / x));
    switch (m) {
        case 0: return z;
        case 1: return -z;
        case 2: return pi - (z - pi_lo);
        default: return (z - pi_lo) - pi;
    }
}
/* ------------------------------------------------------------------ log */
/* fdlibm __ieee754_log (e_log.c): argument reduction to [sqrt(2)/2, sqrt(2)]
 * and the Lg1..Lg7 minimax polynomial in s = f / (2 + f).  Used by the
 * Box-Muller draws of the disturbance noise (device and oracle alike). */
SM_QUAL double sm_log(double x) {
    const double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10,
                 two54 = 1.80143985094819840000e+16, Lg1 = 6.666666666666735130e-01,
                 Lg2 = 3.999999999940941908e-01, Lg3 = 2.857142874366239149e-01,
                 Lg4 = 2.222219843214978396e-01, Lg5 = 1.818357216161805012e-01,
                 Lg6 = 1.531383769920937332e-01, Lg7 = 1.479819860511658591e-01;
    uint64_t u = sm_d2u(x);
    int32_t hx = (int32_t)(u >> 32);
    uint32_t lx = (uint32_t)u;
    int k = 0;
    if (hx < 0x00100000) {                          /* x < 2^-1022 */
        if (((hx & 0x7fffffff) | lx) == 0) return -INFINITY;
        if (hx < 0) return NAN;
        k -= 54;
        x *= two54;
        u = sm_d2u(x);
        hx = (int32_t)(u >> 32);
    }
    if (hx >= 0x7ff00000) return x + x;
    k += (hx >> 20) - 1023;
    hx &= 0x000fffff;
    int32_t i = (hx + 0x95f64) & 0x100000;
    x = sm_u2d(((uint64_t)(uint32_t)(hx | (i ^ 0x3ff00000)) << 32) | (sm_d2u(x) & 0xffffffffu));
    k += (i >> 20);
    double f = x - 1.0;
    double dk;
    if ((0x000fffff & (2 + hx)) < 3) {              /* |f| < 2^-20 */
        if (f == 0.0) {
            if (k == 0) return 0.0;
            dk = (double)k;
            return dk * ln2_hi + dk * ln2_lo;
        }
        double R = f * f * (0.5 - 0.33333333333333333 * f);
        if (k == 0) return f - R;
        dk = (double)k;
        return dk * ln2_hi - ((R - dk * ln2_lo) - f);
    }
    double s = f / (2.0 + f);
    dk = (double)k;
    double z = s * s;
    i = hx - 0x6147a;
    double w = z * z;
    int32_t j = 0x6b851 - hx;
    double t1 = w * (Lg2 + w * (Lg4 + w * Lg6));
    double t2 = z * (Lg1 + w * (Lg3 + w * (Lg5 + w * Lg7)));
    i |= j;
    double R = t2 + t1;
    if (i > 0) {
        double hfsq = 0.5 * f * f;
        if (k == 0) return f - (hfsq - s * (hfsq + R));
        return dk * ln2_hi - ((hfsq - (s * (hfsq + R) + dk * ln2_lo)) - f);
    }
    if (k == 0) return f - s * (f - R);
    return dk * ln2_hi - ((s * (f - R) - dk * ln2_lo) - f);
}

SM_QUAL double sm_asin(double x) { return sm_atan2(x, sqrt((1.0 - x) * (1.0 + x))); }
SM_QUAL double sm_acos(double x) { return sm_atan2(sqrt((1.0 - x) * (1.0 + x)), x); }

#endif /* SALP_MATH_H */
