/*
 * salp_device.h — per-lane SALP physics for gfx950 (one env per lane).
 *
 * Restates the reference hot path (Avielstein/GRASP_LAB_SALP src/robot.py,
 * src/dynamics.py, src/geometry.py, src/salp_robot_env.py) for registers:
 *
 *  - Every 3x3 matrix the reference builds is diagonal, a rotation with known
 *    zeros, or x-only (center of mass, jet moment arm).  The products below keep
 *    the reference's (NumPy/OpenBLAS) evaluation order of every NON-zero term
 *    and drop the terms that are exact zeros (x*0, x+0), so results equal the
 *    full-matrix evaluation bit for bit (signed zeros aside).  The CPU oracle
 *    (oracle/salp_oracle.c) evaluates the full matrices; tests compare the two
 *    exactly.
 *  - fp64 throughout (the reference is NumPy fp64); the few float32 operations
 *    are the ones NumPy 2 performs in float32 (NEP 50: float32 action ->
 *    contraction -> body geometry while REFILL runs past refill_time).
 *  - Quantities that only depend on (length, width, volume, prev volume) are
 *    recomputed at the start of each tick instead of being stored, which is
 *    what Robot.update_properties computes one call earlier.
 *
 * Hot state lives in registers for the whole breathing cycle (~700 ticks);
 * cold env state (targets, obstacles, episode trackers) is read/written in the
 * struct-of-arrays state buffer only at env-step boundaries.
 */
#ifndef SALP_DEVICE_H
#define SALP_DEVICE_H

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/salp.h"
#include "salp_math.h"
#include "salp_philox.h"
#include "salp_random.h"

#pragma clang fp contract(off)

/* The device implements the product arithmetic mode only (salp_math.h
 * SALP_FMA = 1: fused product-sums, the tick's sin / cos, world-frame
 * rotation, Euler-rate map and reciprocal quotients); the oracle implements
 * both, SALP_FMA = 0 being NumPy's own evaluation order. */
static_assert(SALP_FMA, "libsalp.so is built in the product arithmetic mode (salp_math.h)");

#define SD static __device__ __forceinline__
#define SD_MEMBER __device__ __forceinline__
#define SD_HOST_DEV static __host__ __device__ __forceinline__

namespace salp {

constexpr double DT = 0.01;                                /* src/robot.py:293 */
constexpr double PI = 3.141592653589793;
constexpr double COS_GAMMA = 0x1.6a09e667f3bcdp-1;         /* np.cos(np.pi/4) */
constexpr double SIN_GAMMA = 0x1.6a09e667f3bccp-1;         /* np.sin(np.pi/4) */
constexpr double REFILL_C0 = -0x1.f3ffffffffffcp+8, REFILL_C1 = 0x1.5bffffffffffcp+6,
                 REFILL_C2 = -0x1.ccccccccccccbp-2;       /* np.polyfit, src/geometry.py:6-10 */
constexpr double PROPUL_C0 = -0x1.f400000000001p+7, PROPUL_C1 = 0x1.97ffffffffffep+4,
                 PROPUL_C2 = -0x1.0000000000003p-3;       /* src/geometry.py:18-22 */
constexpr double BUOY_MASS = 0.195, SKIN_MASS = 0.145, TUBE_MASS = 0.414; /* src/robot.py:286-288 */
constexpr double CD = 0.3, DRAG_FORCE_RATIO = 0.25, DRAG_TORQUE_RATIO = 0.1; /* :300-302 */
constexpr double AMF0 = 0.5, AMF1 = 0.6, AMF2 = 0.6, AMRF = 0.2;  /* :303-304 */
constexpr double AMT0 = 0.3, AMT1 = 0.6, AMT2 = 0.6;              /* :305 */
enum { REFILL = 0, JET = 1, COAST = 2, REST = 3 };

/* Launch-invariant constants derived on the host from SalpParams (kernel arg,
 * read through the scalar cache). */
struct Params {
    double L0, W0, maxc, dry_mass, nozzle_mass, density, nozzle_area;
    double mid_x;            /* nozzle middle position x = -(length1 + length2) */
    double tube_volume;      /* src/robot.py:295 */
    double tube_volume_I;    /* src/geometry.py:140 (different pi literal) */
    double net_tube_mass;    /* src/geometry.py:157 */
    double com_mass_sum;     /* tube + nozzle + buoy + skin masses */
    double P1000tv;          /* 1000 * tube_volume (src/geometry.py:198) */
    double init_aspect, end_aspect, aspect_den;
    double angle_speed;      /* 31*pi/30 */
    double obstacle_radius, x_min, x_max, y_min, y_max, sep;
    double init_angle1, init_angle2;
    SmPoly sk;               /* sin/cos kernel coefficients (pinned with the rest) */
    int32_t num_obstacles, max_cycles, obs_dim;
    /* randomisation switches (SalpParams; salp_random.h) */
    int32_t rand_dyn, rand_dist, rand_act, rand_obs, latency;
    int64_t n;               /* envs on this device (SoA stride) */
    int64_t cold_off;        /* first double of the env-major cold block (state layout below) */
    int64_t env_offset;      /* global id of env 0 */
    uint64_t seed;
};

/* The launch constants the tick reads, moved into VGPRs for the tick loop.
 * gfx950 has no 64-bit literal operands, so every fp64 constant otherwise lives
 * in an SGPR pair; the tick loop needs more of them than there are SGPRs and
 * the compiler then re-materialises them (two s_mov_b32 per use) inside the
 * loop.  The empty asm makes each value opaque once, before the loop, so it
 * stays in its VGPR pair.  Values unchanged. */
SD Params pin_params(const Params& P) {
    Params v = P;
    asm volatile("" : "+v"(v.L0), "+v"(v.W0), "+v"(v.dry_mass), "+v"(v.nozzle_mass), "+v"(v.density),
                 "+v"(v.nozzle_area), "+v"(v.mid_x), "+v"(v.tube_volume), "+v"(v.net_tube_mass),
                 "+v"(v.com_mass_sum), "+v"(v.P1000tv), "+v"(v.end_aspect), "+v"(v.aspect_den));
    asm volatile("" : "+v"(v.sk.S1), "+v"(v.sk.S2), "+v"(v.sk.S3), "+v"(v.sk.S4), "+v"(v.sk.S5),
                 "+v"(v.sk.S6), "+v"(v.sk.C1), "+v"(v.sk.C2), "+v"(v.sk.C3), "+v"(v.sk.C4), "+v"(v.sk.C5),
                 "+v"(v.sk.C6), "+v"(v.sk.R_INV), "+v"(v.sk.R_P1), "+v"(v.sk.R_P1T));
    return v;
}

/* ----------------------------------------------------------- helpers */
SD double pymax(double a, double b) { return b > a ? b : a; }
/* x / DT, correctly rounded, in 4 instructions instead of the ~11 of a general
 * division: 1/0.01 rounds to exactly 100 with relative error 2^-55.4, so
 * q0 = x*100 is within 1 ulp of x/DT and one FMA correction with the exact
 * remainder yields the correctly rounded quotient (Markstein); div_fixup
 * supplies the sign of zero and the inf/NaN cases.  Checked against x / 0.01
 * on 4e8 random operands (tests/test_divdt.py keeps a sample). */
SD double div_dt(double x) {
    const double q0 = x * 100.0;
    const double q = sm_fma(sm_fma(-DT, q0, x), 100.0, q0);
    return __builtin_amdgcn_div_fixup(q, DT, x);
}
/* x / d with the divisor's reciprocal shared between quotients.  The
 * compiler's f64 division is: v_div_scale of both operands (the identity
 * unless an operand lies near the exponent limits), v_rcp_f64 and two Newton
 * steps (a function of d alone), q0 = x * r, one FMA remainder correction
 * (v_div_fmas: an FMA when nothing was scaled) and v_div_fixup.  Rcp is the
 * refined reciprocal, computed once per divisor; qdiv is the per-quotient
 * tail, 4 instructions instead of 10 and no VCC hazard.  Equal to x / d bit
 * for bit unless v_div_scale would rescale (|x| within 2^53 of the double
 * range limits or of the denormals): the masses, inertias, cosines, lengths
 * and constants the tick divides by are far from both (math selftest row 11
 * checks it against the oracle's C division). */
struct Rcp { double d, r; };
SD Rcp rcp_of(double d) {
    double r = __builtin_amdgcn_rcp(d);
    r = sm_fma(r, sm_fma(-d, r, 1.0), r);
    r = sm_fma(r, sm_fma(-d, r, 1.0), r);
    return Rcp{d, r};
}
SD double qdiv(double x, Rcp k) {
    const double q0 = x * k.r;
    const double q = sm_fma(sm_fma(-k.d, q0, x), k.r, q0);
    return __builtin_amdgcn_div_fixup(q, k.d, x);
}
/* One component a*b - c*d of np.cross (the reference multiplies, then
 * subtracts), the product a*b fused into the difference in the SALP_FMA
 * build (salp_math.h sm_mad; the oracle's cross() is the same expression). */
SD double cross_c(double a, double b, double c, double d) { return sm_mad(a, b, -(c * d)); }
SD float sqf(float x) { return (float)((double)x * (double)x); }
SD float cubef(float x) {
    double p = (double)x * (double)x;
    double h = p * (double)x, e = sm_fma(p, (double)x, -h);
    float r = (float)h;
    double d = h - (double)r;
    float nb = nextafterf(r, d > 0 ? INFINITY : -INFINITY);
    double ulp = (double)nb - (double)r;
    if (d != 0.0 && fabs(d) * 2.0 == fabs(ulp) && e != 0.0) r = ((e > 0) == (d > 0)) ? nb : r;
    return r;
}

/* Rotation R = Rz(psi) Ry(theta) Rx(phi) (src/dynamics.py:34-58) from the
 * dgemm-order product with its zeros removed. */
struct Rot { double r[3][3]; };
SD Rot rot_sc(double sp, double cp, double st, double ct, double ss, double cs) {
    /* A = Rz @ Ry */
    double a00 = cs * ct, a01 = -ss, a02 = cs * st;
    double a10 = ss * ct, a11 = cs, a12 = ss * st;
    double a20 = -st, a22 = ct;
    Rot R;
    R.r[0][0] = a00; R.r[0][1] = sm_fma(a02, sp, a01 * cp); R.r[0][2] = sm_fma(a02, cp, a01 * -sp);
    R.r[1][0] = a10; R.r[1][1] = sm_fma(a12, sp, a11 * cp); R.r[1][2] = sm_fma(a12, cp, a11 * -sp);
    R.r[2][0] = a20; R.r[2][1] = a22 * sp;                   R.r[2][2] = a22 * cp;
    return R;
}
SD Rot rot_zyx(double phi, double theta, double psi) {
    double sp, cp, st, ct, ss, cs;
    sm_sincos(phi, &sp, &cp);
    sm_sincos(theta, &st, &ct);
    sm_sincos(psi, &ss, &cs);
    return rot_sc(sp, cp, st, ct, ss, cs);
}
/* to_world_frame_jit (src/dynamics.py:34-58) of v at the angles (e0, e1, e2)
 * as the tick computes it (salp_math.h: the roll / pitch pair and yaw sin /
 * cos, three plane rotations); finish_step and the trace use it too, so that
 * every world-frame vector equals the oracle's to_world_frame. */
SD void world_frame(double e0, double e1, double e2, double v0, double v1, double v2, double* o, SmPoly K) {
    double sp, cp, st, ct, ss, cs;
    sm_sincos_rp2(e0, e1, &sp, &cp, &st, &ct, K);
    sm_sincos_yaw_p(e2, &ss, &cs, K);
    sm_world_frame(sp, cp, st, ct, ss, cs, v0, v1, v2, o);
}
/* R.T @ (d0, d1, 0) (transposed view order), components 0 and 1 */
SD void rot_body_xy(const Rot& R, double d0, double d1, double* b0, double* b1) {
    *b0 = sm_fma(R.r[1][0], d1, R.r[0][0] * d0);
    *b1 = sm_fma(R.r[1][1], d1, R.r[0][1] * d0);
}

/* ---------------------------------------------- geometry (src/geometry.py) */
/* NumPy 2 performs some geometry operations in float32 (see the file header).
 * Both dtypes run through ONE branch-free code path: every operation is done
 * in fp64 and, in float32 mode, rounded to float32 right after (r32).  For
 * float32 operands this equals the float32 operation exactly (double rounding
 * is innocuous for + - * / sqrt when the wide format has >= 2p+2 bits, 53 >=
 * 50).  Constants that NumPy converts to float32 are selected per lane (sel).
 * No lane-divergent branch, so a wave never executes both dtype variants. */
SD double r32(double x, bool f) { return f ? (double)(float)x : x; }
SD double sel(bool f, double c) { return f ? (double)(float)c : c; }

/* f32 / f64 x**3 (NumPy: float32 ** 3 -> powf, float64 ** 3 -> pow; both
 * correctly rounded here).  For float32 x the double-double cube (h, lo) is
 * exact and rounding h to float32 only needs fixing when h is a float32 tie. */
SD double cube_sel(double x, bool f) {
    double p = x * x, pe = sm_fma(x, x, -p);
    double h = p * x, he = sm_fma(p, x, -h);
    double lo = sm_fma(pe, x, he);
    double c64 = h + lo;
    float r = (float)h;
    double d = h - (double)r;
    float nb = nextafterf(r, d > 0 ? INFINITY : -INFINITY);
    double ulp = (double)nb - (double)r;
    bool tie = d != 0.0 && fabs(d) * 2.0 == fabs(ulp) && lo != 0.0;
    float r2 = (tie && ((lo > 0) == (d > 0))) ? nb : r;
    return f ? (double)r2 : c64;
}

/* Shared pieces of compute_water_volume_jit / compute_inertia_matrix_jit /
 * compute_center_of_mass_jit for one (length, width) */
struct Core {
    double lh, wh, lh2, wh2, t;   /* L/2, W/2, (L/2)^2, (W/2)^2, L/2 - 0.08 */
    double vell, wme;             /* ellipsoid water volume, 1000 * vell */
};
SD Core core(double L, double W, bool f) {
    Core c;
    c.lh = L / 2.0;
    c.wh = W / 2.0;
    c.lh2 = r32(c.lh * c.lh, f);
    c.wh2 = r32(c.wh * c.wh, f);
    c.t = r32(c.lh - sel(f, 0.08), f);
    c.vell = r32(r32(sel(f, (4.0 / 3.0) * PI) * c.lh, f) * c.wh2, f);   /* src/geometry.py:78-81 */
    c.wme = r32(1000.0 * c.vell, f);
    return c;
}
/* Robot._get_water_volume (src/robot.py:1055-1056) */
SD double water_volume(const Params& P, const Core& c, bool f) {
    return r32(c.vell - sel(f, P.tube_volume), f);
}
/* water mass = density * volume (src/robot.py:1058-1063) */
SD double water_mass(const Params& P, double V, bool f) { return r32(sel(f, P.density) * V, f); }

/* compute_center_of_mass_jit (src/geometry.py:186-203), x component */
SD double center_of_mass(const Params& P, const Core& c, double wm, bool f) {
    double pbx = c.lh, ptx = c.t;
    double pnx = r32(r32(-c.lh - sel(f, 0.025), f) + sel(f, 0.05), f);
    double num = c.wme * 0.0 - P.P1000tv * ptx;
    double den = r32(c.wme - sel(f, P.P1000tv), f);
    double pwx = qdiv(num, rcp_of(den));
    double total = r32(sel(f, P.com_mass_sum) + wm, f);
    return qdiv(TUBE_MASS * ptx + P.nozzle_mass * pnx + BUOY_MASS * pbx + SKIN_MASS * 0.0 + wm * pwx,
                rcp_of(total));
}

/* Everything the next tick's dynamics needs from (length, width, volume,
 * prev volume): computed once in update_properties and carried in registers. */
struct Geo {
    double m, mr;                 /* total mass, water-mass rate */
    double I0, I1;                /* inertia diag xx, yy (= zz) */
    double kc0, kc1;              /* drag force: (-0.5 rho A) * C_t per axis (y = z) */
    double ra0, ra1;              /* drag torque: C_r * (-0.5 rho) * A per axis (y = z) */
    double dimx, dimy;            /* width**3, length**3 */
    double speed;                 /* jet speed (V - V_prev) / dt / A_nozzle */
    double rx;                    /* jet moment arm x */
    double rm, rI0, rI1;          /* correctly rounded 1/m, 1/I0, 1/I1 (geo_recips) */
};
/* compute_cross_sectional_area_jit (src/geometry.py:67-75): A0 = area[0],
 * A1 = area[1] = area[2]; compute_drag_coefficient_jit (src/geometry.py:
 * 104-123): the clipped interpolation ratio nr of the coefficient ranges. */
struct Shape { double A0, A1, nr; };
/* compute_jet_moment_arm_jit (src/geometry.py:126-130), x component */
SD double jet_arm(const Params& P, double L) { return P.mid_x + -L / 2.0; }
SD Shape shape_of(const Params& P, const Core& c, double L, double W, bool f) {
    Shape s;
    double pi = sel(f, PI);
    s.A0 = r32(r32(pi * c.wh, f) * c.wh, f);
    s.A1 = r32(r32(pi * c.lh, f) * c.wh, f);
    double aspect = r32(qdiv(L, rcp_of(W)), f);
    double nr = r32(qdiv(r32(aspect - sel(f, P.end_aspect), f), rcp_of(sel(f, P.aspect_den))), f);
    nr = nr < 0.0 ? 0.0 : nr;
    s.nr = nr > 1.0 ? 1.0 : nr;
    return s;
}
/* trans / rot drag-coefficient ranges (src/robot.py:415-434) at ratio nr */
SD double tcd_x(double nr) { return 2.5 - nr * (2.5 - 1.5); }
SD double tcd_y(double nr) { return 1.5 - nr * (1.5 - 2.5); }
SD double rcd_x(double nr) { return 0.3 - nr * (0.3 - 0.1); }
SD double rcd_y(double nr) { return 0.2 - nr * (0.2 - 0.5); }
/* get_mass (src/robot.py:1061-1066); wm = water mass */
SD double geo_mass(const Params& P, double wm, bool f) {
    return r32(r32(sel(f, P.dry_mass) + wm, f) + sel(f, P.nozzle_mass), f);
}
/* Everything of make_geo_shape but the mass: drag coefficients, body cubes,
 * inertia and jet moment arm (the shape side, which k_rollout_pair's B wave
 * computes while the A wave does the mass side). */
SD void geo_shape(const Params& P, const Core& c, double L, double W, bool f, Geo& g) {
    const Shape sh = shape_of(P, c, L, W, f);
    const double A0 = sh.A0, A1 = sh.A1, nr = sh.nr;
    /* compute_drag_force_jit / compute_drag_torque_jit coefficients
     * (src/dynamics.py:110-128; ranges src/robot.py:415-434) */
    const double k = -0.5 * P.density;
    double tcd0 = tcd_x(nr), tcd1 = tcd_y(nr);
    double rcd0 = rcd_x(nr), rcd1 = rcd_y(nr);
    g.kc0 = r32(A0 * k, f) * tcd0;
    g.kc1 = r32(A1 * k, f) * tcd1;
    g.ra0 = rcd0 * k * A0;
    g.ra1 = rcd1 * k * A1;
    g.dimx = cube_sel(W, f);
    g.dimy = cube_sel(L, f);
    /* compute_inertia_matrix_jit (src/geometry.py:133-183) */
    double p1 = sel(f, 1.0 / 3.0 * SKIN_MASS);
    double sx = r32(c.wh2 + c.wh2, f), sy = r32(c.lh2 + c.wh2, f);
    double kw = r32(sel(f, 0.2) * c.wme, f);
    double t8 = r32(c.t * c.t, f);
    double n = r32(c.lh + sel(f, 0.025), f);
    double n25 = r32(n * n, f);
    g.I0 = r32(p1 * sx, f) + r32(kw * sx, f);
    g.I1 = BUOY_MASS * c.lh2 + P.net_tube_mass * t8 + r32(p1 * sy, f) + r32(kw * sy, f) +
           P.nozzle_mass * n25;
    /* compute_jet_moment_arm_jit (src/geometry.py:126-130) */
    g.rx = jet_arm(P, L);
}
SD Geo make_geo_shape(const Params& P, const Core& c, double L, double W, double wm, bool f) {
    Geo g;
    g.m = geo_mass(P, wm, f);
    geo_shape(P, c, L, W, f, g);
    return g;
}
/* get_mass_rate (src/robot.py:651-654) and compute_jet_velocity_jit speed
 * (src/dynamics.py:87-94); float32 only when both volumes are float32. */
SD void jet_rates(const Params& P, double V, double pV, double wm, bool g32, bool pv32, Geo& g) {
    const bool b32 = g32 && pv32;
    double pwm = r32(sel(pv32, P.density) * pV, pv32);
    g.mr = div_dt(wm - pwm);
    g.speed = qdiv(div_dt(V - pV), rcp_of(P.nozzle_area));
    /* The float32 arm only where a lane of the wave holds the float32 body on
     * two ticks in a row (REFILL past refill_time, ~2.5 % of the ticks).  A
     * float32 quotient is the float64 quotient of the float32 operands rounded
     * to float32 (double rounding is exact here: 53 >= 2*24 + 2), so it
     * shares the float64 reciprocals. */
    if (__any(b32)) {
        const Rcp rdt32 = rcp_of(sel(true, DT)), ra32 = rcp_of(sel(true, P.nozzle_area));
        const double mr32 = r32(qdiv(r32(wm - pwm, true), rdt32), true);
        const double sp32 = r32(qdiv(r32(qdiv(r32(V - pV, true), rdt32), true), ra32), true);
        g.mr = b32 ? mr32 : g.mr;
        g.speed = b32 ? sp32 : g.speed;
    }
}
/* The correctly rounded reciprocals 1/m, 1/I0, 1/I1 of the dynamics' two
 * solves (F/m, tau/I; product mode: F * (1/m), the oracle's robot_newton /
 * robot_euler): computed with the geometry, so that a tick whose geometry is
 * kept (steady body) keeps them too. */
SD double rcr(double d) { return qdiv(1.0, rcp_of(d)); }
SD void geo_recips(Geo& g) {
    g.rm = rcr(g.m);
    g.rI0 = rcr(g.I0);
    g.rI1 = rcr(g.I1);
}
SD Geo make_geo(const Params& P, const Core& c, double L, double W, double V, double pV, bool g32,
                bool pv32, double wm) {
    Geo g = make_geo_shape(P, c, L, W, wm, g32);
    jet_rates(P, V, pV, wm, g32, pv32, g);
    geo_recips(g);
    return g;
}

/* Float32-mode geometry of the current cycle.  While REFILL runs past
 * refill_time the body is the float32 contracted shape (init_length -
 * contraction, init_width + contraction) for every tick, so everything NumPy
 * computes in float32 there is a per-cycle constant: computed once per cycle
 * (begin_step / kernel start) into LDS, read back by the ticks whose lane is in
 * that mode.  Ticks compute the float64 geometry only: no dtype selects. */
enum { C32_V, C32_WM, C32_COM, C32_M, C32_I0, C32_I1, C32_KC0, C32_KC1, C32_RA0, C32_RA1, C32_DIMX,
       C32_DIMY, C32_N };
constexpr int LANES = 256;   /* workgroup size of every ticking kernel (LDS stride) */
struct Cache32 {
    double* p;               /* this lane's column of a [C32_N][stride] LDS array */
    int stride = LANES;      /* slots of the array: LANES, or k_rollout_pair's envs per workgroup */
    SD_MEMBER double& operator[](int k) const { return p[k * stride]; }
};
SD void fill_cache32(const Params& P, double contraction, Cache32 c32) {
    const double L = (double)((float)P.L0 - (float)contraction);
    const double W = (double)((float)P.W0 + (float)contraction);
    const Core c = core(L, W, true);
    const double V = water_volume(P, c, true);
    const double wm = water_mass(P, V, true);
    const Geo g = make_geo_shape(P, c, L, W, wm, true);
    c32[C32_V] = V; c32[C32_WM] = wm; c32[C32_COM] = center_of_mass(P, c, wm, true);
    c32[C32_M] = g.m; c32[C32_I0] = g.I0; c32[C32_I1] = g.I1;
    c32[C32_KC0] = g.kc0; c32[C32_KC1] = g.kc1; c32[C32_RA0] = g.ra0; c32[C32_RA1] = g.ra1;
    c32[C32_DIMX] = g.dimx; c32[C32_DIMY] = g.dimy;
}

/* compute_length_jit / compute_width_jit (src/geometry.py:39-64).  With an
 * np.float32 contraction (c32, the env path) `init_length - contraction` is
 * np.float32: in REFILL past refill_time the body is float32, in JET that
 * float32 difference is the first operand of a float64 sum.  With a Python
 * float contraction everything is float64. */
SD void body_lw(const Params& P, int phase, double ct, double refill, double mx, double c,
                double cr, double rr, bool c32, double* L, double* W, bool* f32) {
    const bool fill = phase == REFILL, jet = phase == JET, early = ct < refill;
    const double Lc = c32 ? (double)((float)P.L0 - (float)c) : P.L0 - c;
    const double Wc = c32 ? (double)((float)P.W0 + (float)c) : P.W0 + c;
    const double x = (ct - mx) * rr;
    /* every arm computed, then flat selects (no branches in the tick) */
    const double Le = P.L0 - ct * cr, We = P.W0 + ct * cr, Lj = Lc + x, Wj = Wc - x;
    const double Lf = early ? Le : Lc, Wf = early ? We : Wc;
    const double Lo = jet ? Lj : P.L0, Wo = jet ? Wj : P.W0;
    *L = fill ? Lf : Lo;
    *W = fill ? Wf : Wo;
    *f32 = fill && !early && c32;
}

/* ---------------------------------------------------- per-lane state */
struct Hot {
    double v0, v1, v2, w0, w1, w2, a0, a1, a2, al0, al1, al2;   /* vel, ang vel, acc, ang acc */
    double e0, e1, e2, p0, p1, p2, q0, q1, q2, g0, g1, g2;        /* euler, pos world, position, angle */
    double L, W, V, pV, com, comr, coma, pI0, pI1, pI2;
    double ct, time;
    double refill, jet, coast, c, cr, rr, turn;                /* cycle constants */
    double mx, b1, b2;                                         /* phase boundaries */
    double d0, d1, d2;                                         /* nozzle direction */
    double sp, cp, st, cth;                                    /* sin/cos of roll, pitch */
    Geo geo;                                                   /* geometry of (L, W, V, pV) */
    int phase;
    bool g32, pv32, c32;
    /* randomised kernels only (RAND): this cycle's coefficients, the OU
     * disturbance states that survive the reference's zeroing (force x, y;
     * torque z) and the per-env tick counter of the noise stream */
    struct Rnd {
        double cd, dfr, dtr, amf0, amf1, amf2, amrf0, amrf1, amrf2, amt0, amt1, amt2;
        double ouf0, ouf1, out2, tick;
    } rnd;
    uint64_t env_id;
};

/* An env whose two-wave cycle could not finish (a partner wait gave up): its
 * motion state becomes NaN, the state a diverged env carries. */
SD_HOST_DEV void poison_motion(Hot& h) {
    const double nan = __builtin_nan("");
    h.v0 = h.v1 = h.v2 = h.w0 = h.w1 = h.w2 = nan;
    h.a0 = h.a1 = h.a2 = h.al0 = h.al1 = h.al2 = nan;
    h.e0 = h.e1 = h.e2 = h.p0 = h.p1 = h.p2 = nan;
    h.sp = h.cp = h.st = h.cth = nan;
}

/* Fields store_hot writes (the tick's state); every other field is "cold":
 * touched only at env-step boundaries.  RAND kernels also carry Hot::Rnd. */
SD_HOST_DEV constexpr bool is_rnd(int f) {
    return (f >= SALP_F_CD && f <= SALP_F_DTR) || (f >= SALP_F_AMF0 && f <= SALP_F_AMRF2) ||
           (f >= SALP_F_AMT0 && f <= SALP_F_AMT2) || f == SALP_F_OUF0 || f == SALP_F_OUF1 ||
           f == SALP_F_OUT2 || f == SALP_F_RNG_TICK;
}
template <bool RAND>
SD_HOST_DEV constexpr bool is_hot(int f) {
    return (f >= SALP_F_V0 && f <= SALP_F_ANG2) || (f >= SALP_F_LENGTH && f <= SALP_F_PVOL32) ||
           (f >= SALP_F_CYCLE_TIME && f <= SALP_F_PHASE) || f == SALP_F_CONTR32 || f == SALP_F_TURN_TIME ||
           (RAND && is_rnd(f));
}
/* One env's cold fields into registers with all loads in flight at once. */
template <bool RAND>
SD_HOST_DEV constexpr bool is_cached(int f) { return !is_hot<RAND>(f) && (RAND || f < SALP_F_CD); }

/* ------------------------------------------------ state layout in HBM */
/* The ABI's state is field-major, state[f * n + i] (salp_get_state and
 * salp_set_state convert).  In HBM a handle keeps two regions:
 *   rows:  every field but the cold ones, field-major [kLayout.n_rows][n]: a
 *          wave's load of one field is one contiguous 512-B access (kernel
 *          start and end; the RAND kernels' coefficient / OU fields);
 *   block: the cold fields (is_cached<false>: read and written only at
 *          env-step boundaries), env-major [n][COLD_SLOTS] from P.cold_off
 *          (a multiple of 16 doubles): a lane that ends an env-step moves its
 *          cold state as 16-B loads / stores within 4 whole 128-B lines,
 *          instead of 55 scattered 8-B pieces of 55 rows.
 * Every field has exactly one home (row or slot); field ids are compile-time
 * constants at almost every access, so the lookups fold away. */
#ifndef SALP_COLD_BLOCK
#define SALP_COLD_BLOCK 1   /* 0: every field field-major (the round-1 layout; A/B builds) */
#endif
constexpr int COLD_SLOTS = 64;   /* 512 B per env: 4 lines, line-aligned */
struct Layout {
    int16_t row[SALP_NUM_FIELDS];    /* row of a field-major field, else -1 */
    int16_t slot[SALP_NUM_FIELDS];   /* slot in the env's cold block, else -1 */
    int n_rows, n_cold;
};
constexpr Layout make_layout() {
    Layout L{};
    int r = 0, c = 0;
    for (int f = 0; f < SALP_NUM_FIELDS; ++f) {
        if (SALP_COLD_BLOCK && is_cached<false>(f)) {
            L.slot[f] = (int16_t)c++;
            L.row[f] = -1;
        } else {
            L.row[f] = (int16_t)r++;
            L.slot[f] = -1;
        }
    }
    L.n_rows = r;
    L.n_cold = c;
    return L;
}
constexpr Layout kLayout = make_layout();
static_assert(kLayout.n_cold <= COLD_SLOTS && (!SALP_COLD_BLOCK || kLayout.n_cold % 2 == 1),
              "cold block: 16-B pairs + one tail");
static_assert(kLayout.n_rows + kLayout.n_cold == SALP_NUM_FIELDS, "every field has one home");
/* Offset of the cold block and total doubles of a handle's state (host). */
SD_HOST_DEV constexpr int64_t layout_cold_off(int64_t n) { return ((int64_t)kLayout.n_rows * n + 15) / 16 * 16; }
SD_HOST_DEV constexpr int64_t layout_doubles(int64_t n) {
    return layout_cold_off(n) + (SALP_COLD_BLOCK ? (int64_t)COLD_SLOTS * n : 0);
}

/* State access.  The env-step functions below are templates over the state
 * they read and write: the struct-of-arrays buffer in HBM (double*), or a
 * register copy of one env's row (ColdRegs*, the rollout boundary) so that the
 * env-step epilogue/prologue issues all its loads at once instead of one
 * dependent HBM round trip per read-modify-write. */
/* RAND = false: the randomisation fields (SALP_F_CD and after) are not
 * cached; the plain kernels only ever store constants into them (coefficient
 * means, calm OU states), so they pass straight through to HBM and cost no
 * registers. */
template <bool RAND>
struct ColdRegs {
    double v[SALP_NUM_FIELDS];
    double* g;   /* this env's column of the HBM state: g[f * n] */
    int64_t n;
};
SD size_t state_index(const Params& P, int64_t i, int f) {
    return kLayout.row[f] >= 0 ? (size_t)kLayout.row[f] * (size_t)P.n + (size_t)i
                               : (size_t)P.cold_off + (size_t)i * COLD_SLOTS + (size_t)kLayout.slot[f];
}
SD double& sref(double* S, const Params& P, int64_t i, int f) { return S[state_index(P, i, f)]; }
SD const double& sref(const double* S, const Params& P, int64_t i, int f) { return S[state_index(P, i, f)]; }
template <bool RAND>
SD double& sref(ColdRegs<RAND>* C, const Params&, int64_t, int f) {
    /* plain kernels: the randomisation fields live in rows, read in place */
    return (!RAND && f >= SALP_F_CD) ? C->g[(size_t)kLayout.row[f] * (size_t)C->n] : C->v[f];
}
#define SF(f) sref(S, P, i, (f))

/* Register-resident values derived from the stored state: geometry of the
 * current body and sin/cos of roll and pitch. */
SD void refresh_derived(Hot& h, const Params& P) {
    const Core c = core(h.L, h.W, h.g32);
    h.geo = make_geo(P, c, h.L, h.W, h.V, h.pV, h.g32, h.pv32, water_mass(P, h.V, h.g32));
    sm_sincos_rp2(h.e0, h.e1, &h.sp, &h.cp, &h.st, &h.cth, sm_poly());
}

/* the RAND-only part of Hot (set_control / the tick read and write it) */
SD void load_rnd(Hot& h, const double* S, const Params& P, int64_t i) {
    Hot::Rnd& r = h.rnd;
    r.cd = SF(SALP_F_CD); r.dfr = SF(SALP_F_DFR); r.dtr = SF(SALP_F_DTR);
    r.amf0 = SF(SALP_F_AMF0); r.amf1 = SF(SALP_F_AMF1); r.amf2 = SF(SALP_F_AMF2);
    r.amrf0 = SF(SALP_F_AMRF0); r.amrf1 = SF(SALP_F_AMRF1); r.amrf2 = SF(SALP_F_AMRF2);
    r.amt0 = SF(SALP_F_AMT0); r.amt1 = SF(SALP_F_AMT1); r.amt2 = SF(SALP_F_AMT2);
    r.ouf0 = SF(SALP_F_OUF0); r.ouf1 = SF(SALP_F_OUF1); r.out2 = SF(SALP_F_OUT2);
    r.tick = SF(SALP_F_RNG_TICK);
}
SD void store_rnd(const Hot& h, double* S, const Params& P, int64_t i) {
    const Hot::Rnd& r = h.rnd;
    SF(SALP_F_CD) = r.cd; SF(SALP_F_DFR) = r.dfr; SF(SALP_F_DTR) = r.dtr;
    SF(SALP_F_AMF0) = r.amf0; SF(SALP_F_AMF1) = r.amf1; SF(SALP_F_AMF2) = r.amf2;
    SF(SALP_F_AMRF0) = r.amrf0; SF(SALP_F_AMRF1) = r.amrf1; SF(SALP_F_AMRF2) = r.amrf2;
    SF(SALP_F_AMT0) = r.amt0; SF(SALP_F_AMT1) = r.amt1; SF(SALP_F_AMT2) = r.amt2;
    SF(SALP_F_OUF0) = r.ouf0; SF(SALP_F_OUF1) = r.ouf1; SF(SALP_F_OUT2) = r.out2;
    SF(SALP_F_RNG_TICK) = r.tick;
}

template <bool RAND = false>
SD void load_hot(Hot& h, const double* S, const Params& P, int64_t i, bool derived = true) {
    h.env_id = (uint64_t)(P.env_offset + i);
    if (RAND) load_rnd(h, S, P, i);
    h.v0 = SF(SALP_F_V0); h.v1 = SF(SALP_F_V1); h.v2 = SF(SALP_F_V2);
    h.w0 = SF(SALP_F_W0); h.w1 = SF(SALP_F_W1); h.w2 = SF(SALP_F_W2);
    h.a0 = SF(SALP_F_ACC0); h.a1 = SF(SALP_F_ACC1); h.a2 = SF(SALP_F_ACC2);
    h.al0 = SF(SALP_F_ALPHA0); h.al1 = SF(SALP_F_ALPHA1); h.al2 = SF(SALP_F_ALPHA2);
    h.e0 = SF(SALP_F_ETA0); h.e1 = SF(SALP_F_ETA1); h.e2 = SF(SALP_F_ETA2);
    h.p0 = SF(SALP_F_PW0); h.p1 = SF(SALP_F_PW1); h.p2 = SF(SALP_F_PW2);
    h.q0 = SF(SALP_F_POS0); h.q1 = SF(SALP_F_POS1); h.q2 = SF(SALP_F_POS2);
    h.g0 = SF(SALP_F_ANG0); h.g1 = SF(SALP_F_ANG1); h.g2 = SF(SALP_F_ANG2);
    h.L = SF(SALP_F_LENGTH); h.W = SF(SALP_F_WIDTH); h.V = SF(SALP_F_VOLUME);
    h.pV = SF(SALP_F_PREV_VOLUME); h.com = SF(SALP_F_COM); h.comr = SF(SALP_F_COM_RATE);
    h.coma = SF(SALP_F_COM_ACC);
    h.pI0 = SF(SALP_F_PREV_I0); h.pI1 = SF(SALP_F_PREV_I1); h.pI2 = SF(SALP_F_PREV_I2);
    h.g32 = SF(SALP_F_GEOM32) != 0.0; h.pv32 = SF(SALP_F_PVOL32) != 0.0;
    h.ct = SF(SALP_F_CYCLE_TIME); h.time = SF(SALP_F_TIME);
    h.refill = SF(SALP_F_REFILL_TIME); h.jet = SF(SALP_F_JET_TIME); h.coast = SF(SALP_F_COAST_TIME);
    h.c = SF(SALP_F_CONTRACTION); h.cr = SF(SALP_F_CONTRACT_RATE); h.rr = SF(SALP_F_RELEASE_RATE);
    h.turn = SF(SALP_F_TURN_TIME);
    h.phase = (int)SF(SALP_F_PHASE);
    h.c32 = SF(SALP_F_CONTR32) != 0.0;
    if (derived) refresh_derived(h, P);
}
template <bool RAND = false>
SD void store_hot(const Hot& h, double* S, const Params& P, int64_t i) {
    if (RAND) store_rnd(h, S, P, i);
    SF(SALP_F_V0) = h.v0; SF(SALP_F_V1) = h.v1; SF(SALP_F_V2) = h.v2;
    SF(SALP_F_W0) = h.w0; SF(SALP_F_W1) = h.w1; SF(SALP_F_W2) = h.w2;
    SF(SALP_F_ACC0) = h.a0; SF(SALP_F_ACC1) = h.a1; SF(SALP_F_ACC2) = h.a2;
    SF(SALP_F_ALPHA0) = h.al0; SF(SALP_F_ALPHA1) = h.al1; SF(SALP_F_ALPHA2) = h.al2;
    SF(SALP_F_ETA0) = h.e0; SF(SALP_F_ETA1) = h.e1; SF(SALP_F_ETA2) = h.e2;
    SF(SALP_F_PW0) = h.p0; SF(SALP_F_PW1) = h.p1; SF(SALP_F_PW2) = h.p2;
    SF(SALP_F_POS0) = h.q0; SF(SALP_F_POS1) = h.q1; SF(SALP_F_POS2) = h.q2;
    SF(SALP_F_ANG0) = h.g0; SF(SALP_F_ANG1) = h.g1; SF(SALP_F_ANG2) = h.g2;
    SF(SALP_F_LENGTH) = h.L; SF(SALP_F_WIDTH) = h.W; SF(SALP_F_VOLUME) = h.V;
    SF(SALP_F_PREV_VOLUME) = h.pV; SF(SALP_F_COM) = h.com; SF(SALP_F_COM_RATE) = h.comr;
    SF(SALP_F_COM_ACC) = h.coma;
    SF(SALP_F_PREV_I0) = h.pI0; SF(SALP_F_PREV_I1) = h.pI1; SF(SALP_F_PREV_I2) = h.pI2;
    SF(SALP_F_GEOM32) = h.g32 ? 1.0 : 0.0; SF(SALP_F_PVOL32) = h.pv32 ? 1.0 : 0.0;
    SF(SALP_F_CYCLE_TIME) = h.ct; SF(SALP_F_TIME) = h.time;
    SF(SALP_F_REFILL_TIME) = h.refill; SF(SALP_F_JET_TIME) = h.jet; SF(SALP_F_COAST_TIME) = h.coast;
    SF(SALP_F_CONTRACTION) = h.c; SF(SALP_F_CONTRACT_RATE) = h.cr; SF(SALP_F_RELEASE_RATE) = h.rr;
    SF(SALP_F_TURN_TIME) = h.turn;
    SF(SALP_F_PHASE) = (double)h.phase;
    SF(SALP_F_CONTR32) = h.c32 ? 1.0 : 0.0;
}

/* Nozzle.get_nozzle_direction (src/robot.py:138-150): R_br @ R_mb @ R_nm @
 * [cos g, 0, sin g] with the matrices of _get_rotation_matrices (:187-208). */
SD void nozzle_direction(double angle1, double angle2, double* d) {
    const double cg = COS_GAMMA, sg = SIN_GAMMA;
    double s1, c1, s2, c2;
    sm_sincos(angle1, &s1, &c1);
    sm_sincos(angle2, &s2, &c2);
    /* R_nm = R_theta_fixed @ R_nozzle: columns 0 and 2 are all that is used */
    double n00 = cg * c2, n10 = s2, n20 = sg * c2;
    double n02 = -sg, n12 = 0.0, n22 = cg;
    /* C = (R_br @ R_mb) @ R_nm ; rows of R_br@R_mb: (-0,-0,-1), (s1,c1,0), (c1,-s1,0) */
    double c00 = -n20, c02 = -n22;
    double c10 = sm_fma(c1, n10, s1 * n00), c12 = sm_fma(c1, n12, s1 * n02);
    double c20 = sm_fma(-s1, n10, c1 * n00), c22 = sm_fma(-s1, n12, c1 * n02);
    d[0] = sm_fma(c02, sg, c00 * cg);
    d[1] = sm_fma(c12, sg, c10 * cg);
    d[2] = sm_fma(c22, sg, c20 * cg);
}
/* phase boundaries of update_state / step_through_cycle (src/robot.py:640-649, 742) */
SD void cycle_bounds(Hot& h) {
    h.mx = pymax(h.refill, h.turn);
    h.b1 = h.mx + h.jet;
    h.b2 = h.b1 + h.coast;
}

/* --------------------------------------------------- steady body */
/* Will the next tick's body be the steady one?  In COAST and REST the body is
 * (init_length, init_width) in float64 (body_lw), 70 % of the ticks under
 * random actions.  If the previous geometry was computed for that body too,
 * the next tick's update_properties reproduces it bit for bit, and
 * tick<STEADY> keeps it instead of recomputing (~43 % of a tick;
 * profiles/r2_experiments.md r2j).  The phase only moves forward within a
 * cycle, so a lane steady for one tick stays steady until the cycle ends.
 * The next phase is COAST or REST iff the next cycle_time exceeds both mx and
 * mx + jet (update_state's chain in tick): the reference's polynomial gives
 * small contractions a negative jet (and refill) time, so mx + jet < mx
 * happens (tests/test_gpu_parity.py::test_steady_body_with_negative_phase_times). */
/* The first tick of a cycle is always a full one (h.ct > 0): after a reset
 * the geometry in the state is Robot.reset's, not update_properties' (its
 * centre of mass differs in the last bits), so "the previous tick computed this
 * body" only holds once a tick of the cycle has run.  A cycle whose very first
 * tick is already in COAST/REST (contraction 0: negative refill and jet times)
 * right after a reset showed it: tests/test_gpu_parity.py::
 * test_steady_first_tick_after_reset. */
SD bool next_tick_steady(const Hot& h, const Params& P) {
    const double ct = h.ct + DT;
    return h.ct > 0.0 && h.L == P.L0 && h.W == P.W0 && !h.g32 && ct > h.b1 && ct > h.mx;
}

/* The dynamics of one tick (src/robot.py:854-875: _newton_equations,
 * _euler_equations, _update_motion_states) on the geometry the lane holds
 * (h.geo, centre of mass and its rates, phase, width): everything of Robot.step
 * before cycle_time / update_state / update_properties, in three parts (PARTS
 * bits): TD_FORCES the forces and the velocity integration, TD_KINEMATICS the
 * Euler-angle rates at the current angles, the new angles, their sin / cos
 * (kept for the next tick) and the world-frame velocity into the world
 * position, TD_POSITIONS the body-frame position and angle.  The forces never
 * read the angles or the world position, so the kinematics only follow them
 * (k_step_wave runs them on a second wave).  SETTLED: see tick. */
enum { TD_FORCES = 1, TD_KINEMATICS = 2, TD_POSITIONS = 4, TD_ALL = 7 };
/* The angle chain of a tick (TD_KINEMATICS) on explicit values: the Euler
 * angles, world position and roll / pitch sin / cos it carries, and this
 * tick's integrated v and w (k_rollout_split's B wave runs it alone). */
struct Kin { double e0, e1, e2, p0, p1, p2, sp, cp, st, cth; };
SD void kinematics(Kin& k, double v0, double v1, double v2, double w0, double w1, double w2, const Params& P,
                   double* rates) {
    {   /* to_euler_angle_rate_jit (src/dynamics.py:20-31) at the current angles;
         * product mode (the oracle's to_euler_angle_rate): u = sin(phi) w1 +
         * cos(phi) w2, g = u / cos(theta) is row 2 and tan(theta) u = sin(theta) g
         * row 0's tail */
        const double u = sm_fma(k.cp, w2, k.sp * w1);
        const double g2 = qdiv(u, rcp_of(k.cth));
        const double r0 = sm_fma(k.st, g2, w0);
        const double r1 = sm_fma(-k.sp, w2, k.cp * w1);
        const double r2 = g2;
        k.e0 = sm_mad(r0, DT, k.e0); k.e1 = sm_mad(r1, DT, k.e1); k.e2 = sm_mad(r2, DT, k.e2);
        rates[0] = r0; rates[1] = r1; rates[2] = r2;
    }
    {   /* to_world_frame_jit (src/dynamics.py:34-58) at the new angles (world_frame;
         * roll / pitch sin / cos kept for the next tick's Euler-rate map) */
        double ss, cs;
        sm_sincos_rp2(k.e0, k.e1, &k.sp, &k.cp, &k.st, &k.cth, P.sk);
        sm_sincos_yaw_p(k.e2, &ss, &cs, P.sk);
        double vw[3];
        sm_world_frame(k.sp, k.cp, k.st, k.cth, ss, cs, v0, v1, v2, vw);
        k.p0 = sm_mad(vw[0], DT, k.p0); k.p1 = sm_mad(vw[1], DT, k.p1); k.p2 = sm_mad(vw[2], DT, k.p2);
    }
}
template <bool REC, bool RAND, bool SETTLED, int PARTS = TD_ALL>
SD void tick_dynamics(Hot& h, const Params& P, double* rec, int64_t rs) {
    if (PARTS & TD_FORCES) {
        const Geo& g = h.geo;
        const double m = g.m;
        /* coefficients of this cycle: the reference's means, or (RAND) the
         * Robot._randomize_parameters draw of set_control */
        const double cd = RAND ? h.rnd.cd : CD, dfr = RAND ? h.rnd.dfr : DRAG_FORCE_RATIO,
                     dtr = RAND ? h.rnd.dtr : DRAG_TORQUE_RATIO;
        const double cam0 = RAND ? h.rnd.amf0 : AMF0, cam1 = RAND ? h.rnd.amf1 : AMF1,
                     cam2 = RAND ? h.rnd.amf2 : AMF2;
        const double car0 = RAND ? h.rnd.amrf0 : AMRF, car1 = RAND ? h.rnd.amrf1 : AMRF,
                     car2 = RAND ? h.rnd.amrf2 : AMRF;
        const double cat0 = RAND ? h.rnd.amt0 : AMT0, cat1 = RAND ? h.rnd.amt1 : AMT1,
                     cat2 = RAND ? h.rnd.amt2 : AMT2;
        /* OUDisturbance.sample (src/robot.py:233-242) of the force (x, y kept) and
         * torque (z kept) processes, src/robot.py:796-800, 834-838 */
        double nf0 = 0.0, nf1 = 0.0, nt2 = 0.0;
        if (RAND && P.rand_dist) {
            double z0, z1, z2;
            sr_normals3(P.seed, h.env_id, (uint64_t)h.rnd.tick, &z0, &z1, &z2);
            h.rnd.tick += 1.0;
            h.rnd.ouf0 = sr_ou_step(h.rnd.ouf0, SR_OU_FORCE_THETA, SR_OU_FORCE_SIGMA, z0);
            h.rnd.ouf1 = sr_ou_step(h.rnd.ouf1, SR_OU_FORCE_THETA, SR_OU_FORCE_SIGMA, z1);
            h.rnd.out2 = sr_ou_step(h.rnd.out2, SR_OU_TORQUE_THETA, SR_OU_TORQUE_SIGMA, z2);
            nf0 = h.rnd.ouf0; nf1 = h.rnd.ouf1; nt2 = h.rnd.out2;
        }
        /* ---------------- Newton ---------------- */
        /* Coriolis force -w x (M v)  (src/dynamics.py:159-162) */
        double mv0 = m * h.v0, mv1 = m * h.v1, mv2 = m * h.v2;
        double cf0 = -cross_c(h.w1, mv2, h.w2, mv1), cf1 = -cross_c(h.w2, mv0, h.w0, mv2),
               cf2 = -cross_c(h.w0, mv1, h.w1, mv0);
        /* drag force (src/dynamics.py:110-116); product mode: (k C v) (|v| + ratio) */
        const double vnr = np_norm3(h.v0, h.v1, h.v2) + dfr;
        double df0 = (g.kc0 * h.v0) * vnr;
        double df1 = (g.kc1 * h.v1) * vnr;
        double df2 = (g.kc1 * h.v2) * vnr;
        /* jet force, JET phase only (src/robot.py:937-951, src/dynamics.py:87-101) */
        const bool jet = !SETTLED && h.phase == JET;
        double jf0 = jet ? g.mr * (h.d0 * g.speed) * -cd : 0.0;
        double jf1 = jet ? g.mr * (h.d1 * g.speed) * -cd : 0.0;
        double jf2 = jet ? g.mr * (h.d2 * g.speed) * -cd : 0.0;
        /* added-mass force (src/dynamics.py:131-141) */
        const double mr = SETTLED ? 0.0 : g.mr;
        double am0 = m * cam0, am1 = m * cam1, am2 = m * cam2;
        double amr0 = mr * car0, amr1 = mr * car1, amr2 = mr * car2;
        double amv0 = am0 * h.v0, amv1 = am1 * h.v1, amv2 = am2 * h.v2;
        double af0 = -sm_mad(amr0, h.v0, sm_mad(am0, h.a0, cross_c(h.w1, amv2, h.w2, amv1)));
        double af1 = -sm_mad(amr1, h.v1, sm_mad(am1, h.a1, cross_c(h.w2, amv0, h.w0, amv2)));
        double af2 = -sm_mad(amr2, h.v2, sm_mad(am2, h.a2, cross_c(h.w0, amv1, h.w1, amv0)));
        /* fictitious forces of the moving center of mass (src/robot.py:806-810);
         * com = (cx, 0, 0) */
        const double cx = h.com, crx = SETTLED ? 0.0 : h.comr;
        double acc_y = (h.w0 * (h.w1 * cx) + (h.w2 * crx) * 2.0) + h.al2 * cx;
        double acc_z = (h.w0 * (h.w2 * cx) + -(h.w1 * crx) * 2.0) + -(h.al1 * cx);
        double acc_x = cross_c(h.w1, -(h.w1 * cx), h.w2, h.w2 * cx) + (SETTLED ? 0.0 : h.coma);
        /* total force and linear acceleration (src/dynamics.py:5-10) */
        /* F * (1/m) (product mode; src/dynamics.py:5-10 solves diag(m) a = F) */
        double na0, na1, na2;
        const double rm = g.rm;
        if (RAND) {   /* + force noise (z: zero) */
            na0 = sm_mad(acc_x, m, (((jf0 + df0) + af0) + cf0) + nf0) * rm;
            na1 = sm_mad(acc_y, m, (((jf1 + df1) + af1) + cf1) + nf1) * rm;
            na2 = sm_mad(acc_z, m, (((jf2 + df2) + af2) + cf2) + 0.0) * rm;
        } else {
            na0 = sm_mad(acc_x, m, ((jf0 + df0) + af0) + cf0) * rm;
            na1 = sm_mad(acc_y, m, ((jf1 + df1) + af1) + cf1) * rm;
            na2 = sm_mad(acc_z, m, ((jf2 + df2) + af2) + cf2) * rm;
        }
        /* ---------------- Euler ---------------- */
        const double I0 = g.I0, I1 = g.I1;
        /* Coriolis torque -w x (I w) (src/dynamics.py:165-168) */
        double iw0 = I0 * h.w0, iw1 = I1 * h.w1, iw2 = I1 * h.w2;
        double ct0 = -cross_c(h.w1, iw2, h.w2, iw1), ct1 = -cross_c(h.w2, iw0, h.w0, iw2),
               ct2 = -cross_c(h.w0, iw1, h.w1, iw0);
        /* drag torque (src/dynamics.py:119-128); product mode: (C k A w) (|w| dims + width ratio) */
        const double wn = np_norm3(h.w0, h.w1, h.w2), wr = h.W * dtr;
        const double sx = sm_fma(wn, g.dimx, wr), sy = sm_fma(wn, g.dimy, wr);
        double dt0 = (g.ra0 * h.w0) * sx;
        double dt1 = (g.ra1 * h.w1) * sy;
        double dt2 = (g.ra1 * h.w2) * sy;
        /* jet torque r x F, r = (mid_x - L/2, 0, 0) (src/robot.py:931-935) */
        double jt1 = -(g.rx * jf2), jt2 = g.rx * jf1;
        /* deformation torque -(dI/dt) w; prev_I <- I (src/robot.py:888-896) */
        double ir0 = 0.0, ir1 = 0.0, ir2 = 0.0;   /* settled: (I - prev_I) / dt = +0 / dt */
        if (!SETTLED) {
            ir0 = div_dt(I0 - h.pI0);
            ir1 = div_dt(I1 - h.pI1);
            ir2 = ir1;
            if (h.pI2 != h.pI1) ir2 = div_dt(I1 - h.pI2);   /* prev_I[1,1] == prev_I[2,2] always */
            h.pI0 = I0; h.pI1 = I1; h.pI2 = I1;
        }
        double dft0 = -(ir0 * h.w0), dft1 = -(ir1 * h.w1), dft2 = -(ir2 * h.w2);
        /* added-mass torque, I_rate term identically zero (src/dynamics.py:144-156) */
        double at0 = I0 * cat0, at1 = I1 * cat1, at2 = I1 * cat2;
        double atw0 = at0 * h.w0, atw1 = at1 * h.w1, atw2 = at2 * h.w2;
        double amt0 = -(sm_mad(at0, h.al0, cross_c(h.w1, atw2, h.w2, atw1)) + cross_c(h.v1, amv2, h.v2, amv1));
        double amt1 = -(sm_mad(at1, h.al1, cross_c(h.w2, atw0, h.w0, atw2)) + cross_c(h.v2, amv0, h.v0, amv2));
        double amt2 = -(sm_mad(at2, h.al2, cross_c(h.w0, atw1, h.w1, atw0)) + cross_c(h.v0, amv1, h.v1, amv0));
        /* total torque and angular acceleration (src/dynamics.py:13-17) */
        /* tau * (1/I) (product mode; src/dynamics.py:13-17) */
        double nal0, nal1, nal2;
        const double rI0 = g.rI0, rI1 = g.rI1;
        if (RAND) {   /* + torque noise (x, y: zero) */
            nal0 = ((sm_mad(-ir0, h.w0, dt0 + ct0) + amt0) + 0.0) * rI0;
            nal1 = ((sm_mad(-ir1, h.w1, (jt1 + dt1) + ct1) + amt1) + 0.0) * rI1;
            nal2 = ((sm_mad(-ir2, h.w2, (jt2 + dt2) + ct2) + amt2) + nt2) * rI1;
        } else {
            nal0 = (sm_mad(-ir0, h.w0, dt0 + ct0) + amt0) * rI0;
            nal1 = (sm_mad(-ir1, h.w1, (jt1 + dt1) + ct1) + amt1) * rI1;
            nal2 = (sm_mad(-ir2, h.w2, (jt2 + dt2) + ct2) + amt2) * rI1;
        }
        if (REC) {
            const double z = 0.0;
            auto put = [&](int col, double x) { rec[(int64_t)col * rs] = x; };
            put(SALP_T_JETV0, jet ? h.d0 * g.speed : 0.0);
            put(SALP_T_JETV1, jet ? h.d1 * g.speed : 0.0);
            put(SALP_T_JETV2, jet ? h.d2 * g.speed : 0.0);
            put(SALP_T_JETF0, jf0); put(SALP_T_JETF1, jf1); put(SALP_T_JETF2, jf2);
            put(SALP_T_JETT0, z * jf2 - z * jf1); put(SALP_T_JETT1, jt1); put(SALP_T_JETT2, jt2);
            put(SALP_T_DRAGF0, df0); put(SALP_T_DRAGF1, df1); put(SALP_T_DRAGF2, df2);
            put(SALP_T_DRAGT0, dt0); put(SALP_T_DRAGT1, dt1); put(SALP_T_DRAGT2, dt2);
            put(SALP_T_CORF0, cf0); put(SALP_T_CORF1, cf1); put(SALP_T_CORF2, cf2);
            put(SALP_T_CORT0, ct0); put(SALP_T_CORT1, ct1); put(SALP_T_CORT2, ct2);
            put(SALP_T_AMF0, af0); put(SALP_T_AMF1, af1); put(SALP_T_AMF2, af2);
            put(SALP_T_AMT0, amt0); put(SALP_T_AMT1, amt1); put(SALP_T_AMT2, amt2);
            put(SALP_T_DEFT0, dft0); put(SALP_T_DEFT1, dft1); put(SALP_T_DEFT2, dft2);
            put(SALP_T_ACCF0, acc_x * m); put(SALP_T_ACCF1, acc_y * m); put(SALP_T_ACCF2, acc_z * m);
        }
        h.a0 = na0; h.a1 = na1; h.a2 = na2;
        h.al0 = nal0; h.al1 = nal1; h.al2 = nal2;
        /* ---------------- integrate (semi-implicit Euler) ---------------- */
        h.v0 = sm_mad(na0, DT, h.v0); h.v1 = sm_mad(na1, DT, h.v1); h.v2 = sm_mad(na2, DT, h.v2);
        h.w0 = sm_mad(nal0, DT, h.w0); h.w1 = sm_mad(nal1, DT, h.w1); h.w2 = sm_mad(nal2, DT, h.w2);
    }
    if (PARTS & TD_KINEMATICS) {
        Kin k{h.e0, h.e1, h.e2, h.p0, h.p1, h.p2, h.sp, h.cp, h.st, h.cth};
        double r[3];
        kinematics(k, h.v0, h.v1, h.v2, h.w0, h.w1, h.w2, P, r);
        h.e0 = k.e0; h.e1 = k.e1; h.e2 = k.e2; h.p0 = k.p0; h.p1 = k.p1; h.p2 = k.p2;
        h.sp = k.sp; h.cp = k.cp; h.st = k.st; h.cth = k.cth;
        if (REC) {
            rec[(int64_t)SALP_T_ETAR0 * rs] = r[0];
            rec[(int64_t)SALP_T_ETAR1 * rs] = r[1];
            rec[(int64_t)SALP_T_ETAR2 * rs] = r[2];
        }
    }
    if (PARTS & TD_POSITIONS) {
        h.q0 = sm_mad(h.v0, DT, h.q0); h.q1 = sm_mad(h.v1, DT, h.q1); h.q2 = sm_mad(h.v2, DT, h.q2);
        h.g0 = sm_mad(h.w0, DT, h.g0); h.g1 = sm_mad(h.w1, DT, h.g1); h.g2 = sm_mad(h.w2, DT, h.g2);
    }
}

/* --------------------------------------------------- one physics tick */
/* Robot.step (src/robot.py:670-678): update_dynamics (:854-858) with
 * _newton_equations (:789-823), _euler_equations (:825-851),
 * _update_motion_states (:860-875); then cycle_time, update_state,
 * update_properties (:640-668). */
/* Recording (REC): rec points at this env's column of a trace sample,
 * rec[col * rs] (include/salp.h SalpTraceBuffer); the force columns are
 * written here, the state columns by record_state after the tick. */
/* LATE32: read the cycle's float32-mode geometry from LDS only inside the
 * branch that uses it, not at the top of the tick (no register round trip;
 * faster in k_rollout, slower in the lock-step kernels: A/B in
 * profiles/r1f_experiments.md). */
/* SETTLED (with STEADY): the tick after a steady tick that ended settled
 * (tick's return value): the values that are then exactly +0 are used as
 * the constants they are — centre-of-mass rate and acceleration, water-mass
 * rate and jet speed (settled), the inertia rate I - prev_I (a steady tick
 * set prev_I = I and kept I), and the jet force (the previous steady tick's
 * update_state gave COAST or REST) — and the arithmetic that produced them is
 * skipped.  Every remaining operation is the same, so the results are bit
 * for bit those of the plain steady tick; and the tick ends settled again.
 * Returns, for a STEADY tick, whether this lane is settled after it. */
/* PARTS: the tick_dynamics parts this tick runs (k_rollout_split's A wave runs
 * TD_FORCES | TD_POSITIONS and leaves TD_KINEMATICS to its B wave). */
template <bool REC = false, bool RAND = false, bool LATE32 = false, bool STEADY = false, bool SETTLED = false,
          int PARTS = TD_ALL>
SD bool tick(Hot& h, const Params& P, Cache32 c32, double* rec = nullptr, int64_t rs = 0) {
    static_assert(!SETTLED || STEADY, "a settled tick is a steady one");
    /* this cycle's float32-mode geometry, used at the end if the lane is in
     * that mode (issued first so that the LDS latency hides under the tick) */
    double k32[C32_N];
    if (!LATE32 && !STEADY)
        for (int k = 0; k < C32_N; ++k) k32[k] = c32[k];
    tick_dynamics<REC, RAND, SETTLED, PARTS>(h, P, rec, rs);
    /* ---------------- clocks, phase, properties ---------------- */
    h.ct += DT;
    h.time += DT;
    if (STEADY) {
        /* A steady tick's cycle_time is past mx and mx + jet (next_tick_steady
         * checked this very sum), so update_state gives COAST or REST and
         * body_lw the float64 rest body (init_length, init_width) the lane
         * already holds (next_tick_steady: L == L0, W == W0, !g32). */
        h.phase = h.ct <= h.b2 ? COAST : REST;
        h.pV = h.V;
        h.pv32 = false;
    } else {
        /* update_state's if-chain as flat selects, lowest priority first */
        int ph = h.ct <= h.b2 ? COAST : REST;
        ph = h.ct <= h.b1 ? JET : ph;
        h.phase = h.ct <= h.mx ? REFILL : ph;
        h.pV = h.V;
        h.pv32 = h.g32;
        bool f;
        body_lw(P, h.phase, h.ct, h.refill, h.mx, h.c, h.cr, h.rr, h.c32, &h.L, &h.W, &f);
        h.g32 = f;
    }
    if (STEADY) {
        /* Steady body (see next_tick_steady): update_properties recomputes
         * the previous tick's volume, water mass, centre of mass, mass,
         * inertia and drag coefficients bit for bit, so they are kept; what
         * depends on the previous tick is evaluated by the expressions below
         * with the same operands (the volume and centre-of-mass differences
         * are +0). */
        /* From the second steady tick on these are all +0 and recompute as +0
         * (V == pV, pv32 == false, com - com = +0, and div_dt / qdiv of +0 is
         * +0), so a wave whose lanes are all there skips them. */
        if (SETTLED) return true;
        const auto zero = [&] {
            return (__double_as_longlong(h.comr) | __double_as_longlong(h.coma) | __double_as_longlong(h.geo.mr) |
                    __double_as_longlong(h.geo.speed)) == 0;
        };
        if (!__all(zero())) {
            const double comr = div_dt(h.com - h.com);
            h.coma = div_dt(comr - h.comr);
            h.comr = comr;
            /* jet_rates with g32 = false: its float64 arm */
            const double pwm = r32(sel(h.pv32, P.density) * h.pV, h.pv32);
            h.geo.mr = div_dt(water_mass(P, h.V, false) - pwm);
            h.geo.speed = qdiv(div_dt(h.V - h.pV), rcp_of(P.nozzle_area));
        }
        return zero();
    }
    /* float64 geometry (bitwise the f = false instance of the shared code),
     * replaced by the cycle's float32 geometry where the lane is in that mode */
    const Core c = core(h.L, h.W, false);
    double V = water_volume(P, c, false);
    double wm = water_mass(P, V, false);
    double com = center_of_mass(P, c, wm, false);
    Geo ng = make_geo_shape(P, c, h.L, h.W, wm, false);
    const bool f = h.g32;
    if (f) {
        if (LATE32)
            for (int k = 0; k < C32_N; ++k) k32[k] = c32[k];
        V = k32[C32_V]; wm = k32[C32_WM]; com = k32[C32_COM];
        ng.m = k32[C32_M]; ng.I0 = k32[C32_I0]; ng.I1 = k32[C32_I1];
        ng.kc0 = k32[C32_KC0]; ng.kc1 = k32[C32_KC1]; ng.ra0 = k32[C32_RA0]; ng.ra1 = k32[C32_RA1];
        ng.dimx = k32[C32_DIMX]; ng.dimy = k32[C32_DIMY];
    }
    h.V = V;
    double comr = div_dt(com - h.com);
    h.coma = div_dt(comr - h.comr);
    h.com = com;
    h.comr = comr;
    jet_rates(P, V, h.pV, wm, f, h.pv32, ng);
    geo_recips(ng);
    h.geo = ng;
    return false;
}

/* ------------------------------------------- Nozzle / Robot control */
/* Nozzle.set_yaw_angle + Nozzle.solve_angles (src/robot.py:62-98).  yaw32:
 * the yaw is an np.float32 (env path, src/salp_robot_env.py:207), so np.cos /
 * np.sin run in float32; otherwise in float64. */
/* The angles solve_angles computes for a yaw (no state touched). */
SD void nozzle_ik(double yaw, bool yaw32, double* an1_out, double* an2_out) {
    double sy, cy;
    if (yaw32) {
        float s, c;
        sm_np_sincosf((float)yaw, &s, &c);
        sy = s; cy = c;
    } else {
        sm_sincos(yaw, &sy, &cy);
    }
    /* R_br.T @ -[cos, sin, 0] = [-0, -sin, cos] */
    double t1 = -sy, t2 = cy;
    double val2 = 2.0 * t2 - 1.0;
    if (val2 < -1.0) val2 = -1.0;
    if (val2 > 1.0) val2 = 1.0;
    double an2 = sm_acos(val2), an1;
    if (an2 <= -PI) an2 += 2 * PI;
    else if (an2 > PI) an2 -= 2 * PI;
    if (an2 == 0.0) {
        an1 = 0.0;
    } else {
        double s2, c2;
        sm_sincos(an2, &s2, &c2);
        double a = 0.5 * (c2 - 1.0);
        double b = sqrt(2.0) * s2 / 2.0;
        double val1 = t1 / sqrt(a * a + b * b);
        if (val1 < -1.0) val1 = -1.0;
        if (val1 > 1.0) val1 = 1.0;
        an1 = sm_asin(val1) - sm_atan2(b, a);
    }
    if (an1 <= -PI) an1 += 2 * PI;
    else if (an1 > PI) an1 -= 2 * PI;
    *an1_out = an1;
    *an2_out = an2;
}
template <class ST>
SD void nozzle_solve(ST S, const Params& P, int64_t i, double yaw, bool yaw32) {
    SF(SALP_F_PREV_YAW) = SF(SALP_F_YAW);
    SF(SALP_F_YAW) = yaw;
    SF(SALP_F_PREV_ANGLE1) = SF(SALP_F_ANGLE1);
    SF(SALP_F_PREV_ANGLE2) = SF(SALP_F_ANGLE2);
    double an1, an2;
    nozzle_ik(yaw, yaw32, &an1, &an2);
    SF(SALP_F_ANGLE1) = an1;
    SF(SALP_F_ANGLE2) = an2;
}

/* Length in ticks of the breathing cycle an env-step with float32 action
 * (a0, a1, a2) will run, from the current nozzle angles (which it updates in
 * *ang1 / *ang2 for a following step): begin_step's control arithmetic
 * (src/salp_robot_env.py:166-210, src/robot.py:544-592, 740-757) without
 * touching the state.  ceil(total / dt) is within one tick of the
 * accumulated-clock count; it only orders envs for the lock-step launch. */
SD int predict_cycle_ticks(const Params& P, float a0, float a1, float a2, double* ang1, double* ang2) {
    const float r0 = a0 * 0.06f, r1 = a1 * 10.0f, r2 = a2 * (float)(PI / 2);
    double an1, an2;
    nozzle_ik((double)r2, true, &an1, &an2);
    const double turn = fabs(an1 - *ang1) / P.angle_speed + fabs(an2 - *ang2) / P.angle_speed;
    *ang1 = an1;
    *ang2 = an2;
    const double c = (double)r0, sq = (double)sqf(r0);
    const double refill = REFILL_C0 * sq + REFILL_C1 * c + REFILL_C2;
    const double jet = PROPUL_C0 * sq + PROPUL_C1 * c + PROPUL_C2;
    const double total = pymax(refill, turn) + jet + (double)r1;
    if (!(total > 0.0)) return 0;
    const double t = ceil(total / DT);
    return t > 60000.0 ? 60000 : (int)t;
}

/* Nozzle.set_angles -> _nozzle_turn_time (src/robot.py:50-60, 173-185) */
template <class ST>
SD double nozzle_set_angles(ST S, const Params& P, int64_t i, double a1, double a2) {
    SF(SALP_F_ANGLE1) = a1;
    SF(SALP_F_ANGLE2) = a2;
    const double turn = fabs(a1 - SF(SALP_F_PREV_ANGLE1)) / P.angle_speed +
                        fabs(a2 - SF(SALP_F_PREV_ANGLE2)) / P.angle_speed;
    SF(SALP_F_TURN_TIME) = turn;
    return turn;
}

/* Robot.set_control (src/robot.py:544-592, geometry.py:14-26); c32: the
 * contraction is an np.float32 (contraction**2 is then float32). */
/* this cycle's coefficients: Robot._randomize_parameters (src/robot.py:
 * 594-628) when dynamics randomisation is on, else the means (:553-561).
 * The plain kernels run only with every switch off, when the stored
 * coefficients are the means already (salp_set_randomization restores them
 * when the switch goes off), so they skip this. */
template <bool RAND, class ST>
SD void set_coefficients(Hot& h, ST S, const Params& P, int64_t i) {
    if (!RAND) return;
    SrCoef k;
    if (RAND && P.rand_dyn) {
        sr_draw_coefs(P.seed, h.env_id, (uint64_t)SF(SALP_F_RNG_CTL), &k);
        SF(SALP_F_RNG_CTL) = SF(SALP_F_RNG_CTL) + 1.0;
    } else {
        sr_coef_means(&k);
    }
    SF(SALP_F_CD) = k.cd; SF(SALP_F_DFR) = k.dfr; SF(SALP_F_DTR) = k.dtr;
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        SF(SALP_F_AMF0 + j) = k.amf[j]; SF(SALP_F_AMRF0 + j) = k.amrf[j];
        SF(SALP_F_AMT0 + j) = k.amt[j]; SF(SALP_F_AMRT0 + j) = k.amrt[j];
    }
    h.rnd.cd = k.cd; h.rnd.dfr = k.dfr; h.rnd.dtr = k.dtr;
    h.rnd.amf0 = k.amf[0]; h.rnd.amf1 = k.amf[1]; h.rnd.amf2 = k.amf[2];
    h.rnd.amrf0 = k.amrf[0]; h.rnd.amrf1 = k.amrf[1]; h.rnd.amrf2 = k.amrf[2];
    h.rnd.amt0 = k.amt[0]; h.rnd.amt1 = k.amt[1]; h.rnd.amt2 = k.amt[2];
}

template <bool RAND = false, class ST>
SD void set_control(Hot& h, ST S, const Params& P, int64_t i, double contraction, double coast,
                    double a1, double a2, bool c32) {
    set_coefficients<RAND>(h, S, P, i);
    SF(SALP_F_AVGV0) = 0.0; SF(SALP_F_AVGV1) = 0.0; SF(SALP_F_AVGV2) = 0.0;
    SF(SALP_F_AVGW0) = 0.0; SF(SALP_F_AVGW1) = 0.0; SF(SALP_F_AVGW2) = 0.0;
    h.c = contraction;
    h.coast = coast;
    h.c32 = c32;
    h.turn = nozzle_set_angles(S, P, i, a1, a2);
    nozzle_direction(a1, a2, &h.d0);
    SF(SALP_F_CYCLE) = SF(SALP_F_CYCLE) + 1.0;
    h.ct = 0.0;
    const double sq = c32 ? (double)sqf((float)h.c) : h.c * h.c;
    h.refill = REFILL_C0 * sq + REFILL_C1 * h.c + REFILL_C2;
    h.jet = PROPUL_C0 * sq + PROPUL_C1 * h.c + PROPUL_C2;
    h.cr = h.refill > 0 ? h.c / h.refill : 0.0;
    h.rr = h.jet > 0 ? h.c / h.jet : 0.0;
    cycle_bounds(h);
}

/* Robot.step_through_cycle prologue (src/robot.py:740-748): the previous
 * cycle's displacement over this cycle's total time. */
template <class ST>
SD void cycle_prologue(const Hot& h, ST S, const Params& P, int64_t i) {
    const double total = h.b2;
    double pq0 = SF(SALP_F_PPOS0), pq1 = SF(SALP_F_PPOS1), pq2 = SF(SALP_F_PPOS2);
    double pg0 = SF(SALP_F_PANG0), pg1 = SF(SALP_F_PANG1), pg2 = SF(SALP_F_PANG2);
    SF(SALP_F_AVGV0) = (h.q0 - pq0) / total; SF(SALP_F_AVGV1) = (h.q1 - pq1) / total;
    SF(SALP_F_AVGV2) = (h.q2 - pq2) / total;
    SF(SALP_F_AVGW0) = (h.g0 - pg0) / total; SF(SALP_F_AVGW1) = (h.g1 - pg1) / total;
    SF(SALP_F_AVGW2) = (h.g2 - pg2) / total;
    SF(SALP_F_PPOS0) = h.q0; SF(SALP_F_PPOS1) = h.q1; SF(SALP_F_PPOS2) = h.q2;
    SF(SALP_F_PANG0) = h.g0; SF(SALP_F_PANG1) = h.g1; SF(SALP_F_PANG2) = h.g2;
    SF(SALP_F_PENDING) = 1.0;
}

/* ------------------------------------------------ env-step prologue */
/* SalpRobotEnv.step up to step_through_cycle's loop (src/salp_robot_env.py:
 * 196-210): float32 action rescale, IK, set_control, cycle prologue. */
template <bool RAND = false, class ST>
SD void begin_step(Hot& h, ST S, const Params& P, int64_t i, float a0, float a1, float a2,
                   Cache32 c32) {
    SF(SALP_F_ACT0) = a0; SF(SALP_F_ACT1) = a1; SF(SALP_F_ACT2) = a2;
    /* _rescale_action in float32 (src/salp_robot_env.py:166-174) */
    float r0 = a0 * 0.06f, r1 = a1 * 10.0f, r2 = a2 * (float)(PI / 2);
    if (RAND && P.rand_act) {
        /* _randomize_actions (:176-181): Python floats from here on, so the
         * IK and the body geometry run in float64 */
        const float rr[3] = {r0, r1, r2};
        double ra[3];
        sr_randomize_action(P.seed, h.env_id, (uint64_t)SF(SALP_F_STEP_COUNT), rr, ra);
        nozzle_solve(S, P, i, ra[2], false);
        set_control<RAND>(h, S, P, i, ra[0], ra[1], SF(SALP_F_ANGLE1), SF(SALP_F_ANGLE2), false);
    } else {
        nozzle_solve(S, P, i, (double)r2, true);
        set_control<RAND>(h, S, P, i, (double)r0, (double)r1, SF(SALP_F_ANGLE1), SF(SALP_F_ANGLE2), true);
    }
    fill_cache32(P, h.c, c32);
    cycle_prologue(h, S, P, i);
}

/* Trace sample: the state columns (src/robot.py:687-716) of the current
 * state.  first: sample 0 of a cycle, whose force / rate columns are NaN. */
template <class ST>
SD void record_state(const Hot& h, const Params& P, ST S, int64_t i, double* rec,
                     int64_t rs, bool first) {
    auto put = [&](int col, double x) { rec[(int64_t)col * rs] = x; };
    put(SALP_T_STATE, (double)h.phase);
    put(SALP_T_PW0, h.p0); put(SALP_T_PW1, h.p1); put(SALP_T_PW2, h.p2);
    put(SALP_T_V0, h.v0); put(SALP_T_V1, h.v1); put(SALP_T_V2, h.v2);
    put(SALP_T_ACC0, h.a0); put(SALP_T_ACC1, h.a1); put(SALP_T_ACC2, h.a2);
    put(SALP_T_ETA0, h.e0); put(SALP_T_ETA1, h.e1); put(SALP_T_ETA2, h.e2);
    put(SALP_T_W0, h.w0); put(SALP_T_W1, h.w1); put(SALP_T_W2, h.w2);
    put(SALP_T_ALPHA0, h.al0); put(SALP_T_ALPHA1, h.al1); put(SALP_T_ALPHA2, h.al2);
    put(SALP_T_LENGTH, h.L); put(SALP_T_WIDTH, h.W);
    const Core c = core(h.L, h.W, h.g32);
    const Shape sh = shape_of(P, c, h.L, h.W, h.g32);
    put(SALP_T_AREA0, sh.A0); put(SALP_T_AREA1, sh.A1); put(SALP_T_AREA2, sh.A1);
    put(SALP_T_VOLUME, h.V);
    put(SALP_T_MASS, h.geo.m);
    put(SALP_T_MASS_RATE, h.geo.mr);
    put(SALP_T_I0, h.geo.I0); put(SALP_T_I1, h.geo.I1); put(SALP_T_I2, h.geo.I1);
    put(SALP_T_TCD0, tcd_x(sh.nr)); put(SALP_T_TCD1, tcd_y(sh.nr)); put(SALP_T_TCD2, tcd_y(sh.nr));
    put(SALP_T_RCD0, rcd_x(sh.nr)); put(SALP_T_RCD1, rcd_y(sh.nr)); put(SALP_T_RCD2, rcd_y(sh.nr));
    put(SALP_T_COM, h.com); put(SALP_T_COM_RATE, h.comr); put(SALP_T_COM_ACC, h.coma);
    /* get_front_position_world_frame (src/robot.py:924-928) */
    double fw[3];
    world_frame(h.e0, h.e1, h.e2, h.L / 2, 0.0, 0.0, fw, sm_poly());
    put(SALP_T_FRONT_W0, fw[0]); put(SALP_T_FRONT_W1, fw[1]); put(SALP_T_FRONT_W2, fw[2]);
    if (first) {
        for (int k = SALP_T_FIRST_FORCE; k < SALP_TRACE_DIM; ++k) put(k, NAN);
        put(SALP_T_ETAR0, NAN); put(SALP_T_ETAR1, NAN); put(SALP_T_ETAR2, NAN);
        put(SALP_T_NOZZLE_YAW, NAN);
    } else {
        /* Nozzle.step(cycle_time) (src/robot.py:101-108) */
        const double yaw = SF(SALP_F_YAW), pyaw = SF(SALP_F_PREV_YAW);
        put(SALP_T_NOZZLE_YAW, h.ct < h.turn ? pyaw + (h.ct / h.turn) * (yaw - pyaw) : yaw);
    }
}

/* Resume an in-flight cycle: derived per-cycle values from stored ones. */
template <class ST>
SD void resume_cycle(Hot& h, ST S, const Params& P, int64_t i) {
    cycle_bounds(h);
    nozzle_direction(SF(SALP_F_ANGLE1), SF(SALP_F_ANGLE2), &h.d0);
}

/* ------------------------------------------------------ observation */
/* _get_observation (src/salp_robot_env.py:651-670) */
template <class ST>
SD void observation(const Hot& h, const Rot& R, ST S, const Params& P, int64_t i,
                    float* obs) {
    double tx = SF(SALP_F_TARGET0), ty = SF(SALP_F_TARGET1);
    double b0, b1;
    rot_body_xy(R, tx - h.p0, ty - h.p1, &b0, &b1);
    double heading = sm_atan2(b1, b0);
    obs[0] = (float)b0; obs[1] = (float)b1;
    obs[2] = (float)h.v0; obs[3] = (float)h.v1;
    obs[4] = (float)h.w2; obs[5] = (float)heading;
    const int nob = (int)SF(SALP_F_N_OBST);
#pragma unroll
    for (int k = 0; k < SALP_MAX_OBSTACLES; ++k) {
        if (k >= P.num_obstacles) break;
        if (k < nob) {
            obs[6 + 2 * k] = (float)(SF(SALP_F_OBST0 + 2 * k) - h.p0);
            obs[7 + 2 * k] = (float)(SF(SALP_F_OBST0 + 2 * k + 1) - h.p1);
        } else {
            obs[6 + 2 * k] = 0.0f;
            obs[7 + 2 * k] = 0.0f;
        }
    }
}

struct StepOut {
    double reward;
    bool terminated, truncated, hit;
};

/* ------------------------------------------------ env-step epilogue */
/* SalpRobotEnv.step after the cycle (src/salp_robot_env.py:237-299), reward
 * (:349-397), collision (:561-568), episode metrics (:399-447). */
template <bool RAND = false, class ST>
SD StepOut finish_step(Hot& h, ST S, const Params& P, int64_t i, float* obs,
                       double* info) {
    StepOut out;
    const Rot R = rot_zyx(h.e0, h.e1, h.e2);   /* the body frame of the observation and the reward */
    double vw[3];
    world_frame(h.e0, h.e1, h.e2, h.v0, h.v1, h.v2, vw, sm_poly());
    const double px = h.p0, py = h.p1;
    /* episode_positions / episode_velocities */
    double path = SF(SALP_F_PATH_LEN) + np_norm2(px - SF(SALP_F_LAST_PX), py - SF(SALP_F_LAST_PY));
    SF(SALP_F_PATH_LEN) = path;
    SF(SALP_F_LAST_PX) = px; SF(SALP_F_LAST_PY) = py;
    double svel = SF(SALP_F_SUM_VEL) + np_norm2(vw[0], vw[1]);
    SF(SALP_F_SUM_VEL) = svel;
    const double tx = SF(SALP_F_TARGET0), ty = SF(SALP_F_TARGET1);
    const double dx = px - tx, dy = py - ty;
    const double dist = np_norm2(dx, dy);
    /* reward components */
    double comp[7];
    comp[0] = (-dist + SF(SALP_F_PREV_DIST)) * 100;
    SF(SALP_F_PREV_DIST) = dist;
    double b0, b1;
    rot_body_xy(R, dx, dy, &b0, &b1);
    comp[1] = -0.5 * fabs(sm_atan2(-b1, -b0));
    const float a2 = (float)SF(SALP_F_ACT2);
    const double ep_len = SF(SALP_F_EP_LEN);
    if (ep_len == 0.0) {
        double ch = (double)a2 - SF(SALP_F_PREV_A2);
        comp[2] = -1.0 * (ch * ch);
    } else {
        float ch = a2 - (float)SF(SALP_F_PREV_A2);
        comp[2] = (double)(-(ch * ch));
    }
    comp[3] = -10.0 * fabs(SF(SALP_F_AVGW2));
    comp[4] = -0.1;
    comp[5] = -100.0 * fabs(SF(SALP_F_AVGV1));
    comp[6] = 0.0;
    const int nob = (int)SF(SALP_F_N_OBST);
    double md = 0.0;
#pragma unroll
    for (int k = 0; k < SALP_MAX_OBSTACLES; ++k) {
        if (k >= nob) break;
        double d = np_norm2(px - SF(SALP_F_OBST0 + 2 * k), py - SF(SALP_F_OBST0 + 2 * k + 1));
        if (k == 0 || d < md) md = d;
    }
    if (nob > 0) {
        double danger = 2.0 * P.obstacle_radius;
        if (md < danger) comp[6] = -1.0 * (1.0 - md / danger);
    }
    double reward = comp[0] + comp[1] + comp[2] + comp[3] + comp[4] + comp[5] + comp[6];
    observation(h, R, S, P, i, obs);
    /* _randomize_observations (src/salp_robot_env.py:183-194, 253-254) */
    if (RAND && P.rand_obs) sr_randomize_obs(P.seed, h.env_id, (uint64_t)SF(SALP_F_STEP_COUNT), obs);
    /* _check_obstacle_collision with get_current_length() */
    bool l32;
    double Lc, Wc;
    body_lw(P, h.phase, h.ct, h.refill, h.mx, h.c, h.cr, h.rr, h.c32, &Lc, &Wc, &l32);
    double thr = l32 ? (double)((float)P.obstacle_radius + (float)Lc / 2.0f)
                     : P.obstacle_radius + Lc / 2;
    bool hit = false;
#pragma unroll
    for (int k = 0; k < SALP_MAX_OBSTACLES; ++k) {
        if (k >= nob) break;
        double d = np_norm2(px - SF(SALP_F_OBST0 + 2 * k), py - SF(SALP_F_OBST0 + 2 * k + 1));
        if (d < thr) hit = true;
    }
    bool done = false, trunc = false;
    if (dist < 0.2) { done = true; reward += 500.0; }
    else if (dist > 5.0) { trunc = true; reward -= 200.0; }
    if (hit) { trunc = true; reward -= 200.0; }
    if (SF(SALP_F_CYCLE) >= (double)P.max_cycles) { trunc = true; reward -= 50.0; }
    /* episode accumulators */
    const double nlen = ep_len + 1.0;
    SF(SALP_F_EP_LEN) = nlen;
    const double ret = SF(SALP_F_EP_RETURN) + reward;
    SF(SALP_F_EP_RETURN) = ret;
    const double sa0 = SF(SALP_F_SUM_A0) + (double)(float)SF(SALP_F_ACT0);
    const double sa1 = SF(SALP_F_SUM_A1) + (double)(float)SF(SALP_F_ACT1);
    const double sa2 = SF(SALP_F_SUM_ABS_A2) + (double)fabsf(a2);
    SF(SALP_F_SUM_A0) = sa0; SF(SALP_F_SUM_A1) = sa1; SF(SALP_F_SUM_ABS_A2) = sa2;
    double sr[7];
#pragma unroll
    for (int k = 0; k < 7; ++k) {
        sr[k] = SF(SALP_F_SUM_R0 + k) + comp[k];
        SF(SALP_F_SUM_R0 + k) = sr[k];
    }
    if (info) {
        for (int k = 0; k < SALP_INFO_DIM; ++k) info[k] = 0.0;
        for (int k = 0; k < 7; ++k) info[SALP_INFO_R_TRACK + k] = comp[k];
        info[SALP_INFO_EP_RETURN] = ret;
        info[SALP_INFO_EP_LEN] = nlen;
        info[SALP_INFO_HIT_OBSTACLE] = hit ? 1.0 : 0.0;
        if (done || trunc) {
            double dd = np_norm2(px - 0.0, py - 0.0);
            info[SALP_INFO_HAS_METRICS] = 1.0;
            info[SALP_INFO_PATH_LENGTH] = path;
            info[SALP_INFO_DIRECT_DISTANCE] = dd;
            info[SALP_INFO_PATH_EFFICIENCY] = path > 0 ? dd / path : 0.0;
            info[SALP_INFO_FINAL_DISTANCE] = dist;
            info[SALP_INFO_INITIAL_DISTANCE] = SF(SALP_F_INIT_DIST);
            info[SALP_INFO_AVG_COMPRESSION] = sa0 / nlen;
            info[SALP_INFO_AVG_COAST_TIME] = sa1 / nlen;
            info[SALP_INFO_AVG_NOZZLE_ANGLE] = sa2 / nlen;
            info[SALP_INFO_AVG_VELOCITY] = svel / (nlen + 1.0);
            for (int k = 0; k < 7; ++k) info[SALP_INFO_AVG_R_TRACK + k] = sr[k] / nlen;
        }
    }
    SF(SALP_F_PREV_A2) = (double)a2;
    SF(SALP_F_PENDING) = 0.0;
    if (RAND && P.latency) {
        /* latency (src/salp_robot_env.py:292-297): set_control(contraction=0,
         * coast_time=U(0, 0.1), current nozzle angles) without a cycle */
        const double lat = sr_latency(P.seed, h.env_id, (uint64_t)SF(SALP_F_STEP_COUNT));
        set_control<RAND>(h, S, P, i, 0.0, lat, SF(SALP_F_ANGLE1), SF(SALP_F_ANGLE2), false);
    }
    out.reward = reward;
    out.terminated = done;
    out.truncated = trunc;
    out.hit = hit;
    return out;
}

/* ---------------------------------------------------------- reset */
/* Philox draws replacing np.random in generate_target_point("random") and
 * _generate_obstacles (src/salp_robot_env.py:449-559). */
SD int draw_reset(const Params& P, uint64_t env_id, uint64_t episode, float* tgt, float* obst) {
    double u0, u1;
    sp_reset_pair(P.seed, env_id, episode, 0u, &u0, &u1);
    double tx = P.x_min + (P.x_max - P.x_min) * u0, ty = P.y_min + (P.y_max - P.y_min) * u1;
    if (tx < P.x_min) tx = P.x_min;
    if (tx > P.x_max) tx = P.x_max;
    if (ty < P.y_min) ty = P.y_min;
    if (ty > P.y_max) ty = P.y_max;
    tgt[0] = (float)tx; tgt[1] = (float)ty;
    int n = 0;
    for (int k = 0; k < P.num_obstacles; ++k) {
        for (int att = 0; att < 200; ++att) {
            sp_reset_pair(P.seed, env_id, episode, (uint32_t)(1 + k * 200 + att), &u0, &u1);
            float px = (float)(P.x_min + (P.x_max - P.x_min) * u0);
            float py = (float)(P.y_min + (P.y_max - P.y_min) * u1);
            float ds = sqrtf(sm_fmaf(py, py, px * px));
            float ex = px - tgt[0], ey = py - tgt[1];
            float dtg = sqrtf(sm_fmaf(ey, ey, ex * ex));
            bool close = false;
            for (int j = 0; j < n; ++j) {
                float fx = px - obst[2 * j], fy = py - obst[2 * j + 1];
                if ((double)sqrtf(sm_fmaf(fy, fy, fx * fx)) < P.sep) close = true;
            }
            if ((double)ds > 0.5 && (double)dtg > 0.5 && !close) {
                obst[2 * n] = px; obst[2 * n + 1] = py; ++n;
                break;
            }
        }
    }
    return n;
}

/* Robot.reset (src/robot.py:452-501): kinematics zeroed, body back to the
 * initial shape; the center of mass is taken from the PREVIOUS geometry
 * (get_center_of_mass runs before length/width are reset); nozzle angles are
 * not reset. */
template <class ST>
SD void robot_reset(Hot& h, ST S, const Params& P, int64_t i) {
    h.time = 0.0; h.ct = 0.0; h.phase = REST;
    SF(SALP_F_CYCLE) = 0.0;
    h.v0 = h.v1 = h.v2 = 0.0; h.w0 = h.w1 = h.w2 = 0.0;
    h.a0 = h.a1 = h.a2 = 0.0; h.al0 = h.al1 = h.al2 = 0.0;
    h.e0 = h.e1 = h.e2 = 0.0; h.p0 = h.p1 = h.p2 = 0.0;
    h.q0 = h.q1 = h.q2 = 0.0; h.g0 = h.g1 = h.g2 = 0.0;
    SF(SALP_F_PPOS0) = 0.0; SF(SALP_F_PPOS1) = 0.0; SF(SALP_F_PPOS2) = 0.0;
    SF(SALP_F_PANG0) = 0.0; SF(SALP_F_PANG1) = 0.0; SF(SALP_F_PANG2) = 0.0;
    {
        const Core old = core(h.L, h.W, h.g32);
        h.com = center_of_mass(P, old, water_mass(P, h.V, h.g32), h.g32);
    }
    h.comr = (h.com - h.com) / DT;
    h.coma = (h.comr - h.comr) / DT;
    h.L = P.L0; h.W = P.W0; h.g32 = false;
    const Core c0 = core(h.L, h.W, false);
    h.V = water_volume(P, c0, false);
    h.pV = h.V; h.pv32 = false;
    refresh_derived(h, P);
    h.pI0 = h.geo.I0; h.pI1 = h.geo.I1; h.pI2 = h.geo.I1;
    /* force_disturbance.reset(), torque_disturbance.reset() (src/robot.py:454-455);
     * with disturbances off the processes are calm already (salp_set_randomization) */
    if (P.rand_dist) {
        SF(SALP_F_OUF0) = 0.0; SF(SALP_F_OUF1) = 0.0; SF(SALP_F_OUF2) = 0.0;
        SF(SALP_F_OUT0) = 0.0; SF(SALP_F_OUT1) = 0.0; SF(SALP_F_OUT2) = 0.0;
        h.rnd.ouf0 = 0.0; h.rnd.ouf1 = 0.0; h.rnd.out2 = 0.0;
    }
    SF(SALP_F_PENDING) = 0.0;
}

/* SalpRobotEnv.reset with the target / obstacles given (src/salp_robot_env.py:
 * 114-155) -> Robot.reset. */
template <class ST>
SD void reset_env(Hot& h, ST S, const Params& P, int64_t i, const float* tgt,
                  const float* obst, int nob, float* obs) {
    SF(SALP_F_TARGET0) = tgt[0]; SF(SALP_F_TARGET1) = tgt[1];
#pragma unroll
    for (int k = 0; k < SALP_MAX_OBSTACLES; ++k) {
        SF(SALP_F_OBST0 + 2 * k) = k < nob ? (double)obst[2 * k] : 0.0;
        SF(SALP_F_OBST0 + 2 * k + 1) = k < nob ? (double)obst[2 * k + 1] : 0.0;
    }
    SF(SALP_F_N_OBST) = nob;
    robot_reset(h, S, P, i);
    /* env trackers */
    const double d0 = h.p0 - (double)tgt[0], d1 = h.p1 - (double)tgt[1];
    const double dist = np_norm2(d0, d1);
    SF(SALP_F_PREV_DIST) = dist;
    SF(SALP_F_PREV_A2) = 0.0;
    SF(SALP_F_ACT0) = 0.0; SF(SALP_F_ACT1) = 0.0; SF(SALP_F_ACT2) = 0.0;
    SF(SALP_F_EP_LEN) = 0.0; SF(SALP_F_EP_RETURN) = 0.0; SF(SALP_F_PATH_LEN) = 0.0;
    SF(SALP_F_LAST_PX) = h.p0; SF(SALP_F_LAST_PY) = h.p1;
    SF(SALP_F_SUM_A0) = 0.0; SF(SALP_F_SUM_A1) = 0.0; SF(SALP_F_SUM_ABS_A2) = 0.0;
    SF(SALP_F_SUM_VEL) = np_norm2(0.0, 0.0);
    SF(SALP_F_INIT_DIST) = dist;
#pragma unroll
    for (int k = 0; k < 7; ++k) SF(SALP_F_SUM_R0 + k) = 0.0;
    SF(SALP_F_EPISODE) = SF(SALP_F_EPISODE) + 1.0;
    SF(SALP_F_PENDING) = 0.0;
    if (obs) {
        Rot R = rot_zyx(h.e0, h.e1, h.e2);
        observation(h, R, S, P, i, obs);
    }
}

template <class ST>
SD void reset_env_philox(Hot& h, ST S, const Params& P, int64_t i, float* obs) {
    float tgt[2], obst[2 * SALP_MAX_OBSTACLES];
    int nob = draw_reset(P, (uint64_t)(P.env_offset + i), (uint64_t)SF(SALP_F_EPISODE), tgt, obst);
    reset_env(h, S, P, i, tgt, obst, nob, obs);
}

/* ------------------------------------- rollout boundary: LDS + registers */
/* One env's cold block as 16-B loads (all in flight at once), plus, in the
 * RAND kernels, the randomisation fields they cache from their rows. */
template <bool RAND>
SD void load_cold(ColdRegs<RAND>& C, double* S, const Params& P, int64_t i) {
    C.g = S + i;
    C.n = P.n;
    if (!SALP_COLD_BLOCK) {
#pragma unroll
        for (int f = 0; f < SALP_NUM_FIELDS; ++f)
            if (is_cached<RAND>(f)) C.v[f] = S[(size_t)f * (size_t)P.n + (size_t)i];
        return;
    }
    const double2* blk = reinterpret_cast<const double2*>(S + P.cold_off + (size_t)i * COLD_SLOTS);
    double v[kLayout.n_cold + 1];
#pragma unroll
    for (int k = 0; k < (kLayout.n_cold + 1) / 2; ++k) {
        const double2 x = blk[k];
        v[2 * k] = x.x;
        v[2 * k + 1] = x.y;
    }
#pragma unroll
    for (int f = 0; f < SALP_NUM_FIELDS; ++f) {
        if (kLayout.slot[f] >= 0) C.v[f] = v[kLayout.slot[f]];
        else if (is_cached<RAND>(f)) C.v[f] = S[(size_t)kLayout.row[f] * (size_t)P.n + (size_t)i];
    }
}
template <bool RAND>
SD void store_cold(const ColdRegs<RAND>& C, double* S, const Params& P, int64_t i) {
    if (!SALP_COLD_BLOCK) {
#pragma unroll
        for (int f = 0; f < SALP_NUM_FIELDS; ++f)
            if (is_cached<RAND>(f)) S[(size_t)f * (size_t)P.n + (size_t)i] = C.v[f];
        return;
    }
    double v[kLayout.n_cold + 1];
#pragma unroll
    for (int f = 0; f < SALP_NUM_FIELDS; ++f) {
        if (kLayout.slot[f] >= 0) v[kLayout.slot[f]] = C.v[f];
        else if (is_cached<RAND>(f)) S[(size_t)kLayout.row[f] * (size_t)P.n + (size_t)i] = C.v[f];
    }
    v[kLayout.n_cold] = 0.0;   /* padding slot of the last 16-B pair */
    double2* blk = reinterpret_cast<double2*>(S + P.cold_off + (size_t)i * COLD_SLOTS);
#pragma unroll
    for (int k = 0; k < (kLayout.n_cold + 1) / 2; ++k) blk[k] = make_double2(v[2 * k], v[2 * k + 1]);
}

/* A lane's slot of a workgroup LDS array [SPILL_N][LANES]: the whole Hot
 * state parks here while the wave runs an env-step boundary.  Plain kernels
 * park the geometry and roll/pitch sin/cos too (nothing recomputed on
 * reload); RAND kernels park Hot::Rnd in those slots instead and recompute
 * the geometry on reload. */
constexpr int SPILL_N = 63;
struct SpillSlot {
    double* p;
    int stride = LANES;
    SD_MEMBER double& operator[](int k) const { return p[k * stride]; }
};
template <bool RAND>
SD void spill(const Hot& h, SpillSlot s) {
    const Hot::Rnd& r = h.rnd;
    const double v[SPILL_N] = {
        h.v0, h.v1, h.v2, h.w0, h.w1, h.w2, h.a0, h.a1, h.a2, h.al0, h.al1, h.al2,
        h.e0, h.e1, h.e2, h.p0, h.p1, h.p2, h.q0, h.q1, h.q2, h.g0, h.g1, h.g2,
        h.L, h.W, h.V, h.pV, h.com, h.comr, h.coma, h.pI0, h.pI1, h.pI2, h.ct, h.time,
        h.refill, h.jet, h.coast, h.c, h.cr, h.rr, h.turn, h.d0, h.d1, h.d2,
        (double)(h.phase | (h.g32 ? 4 : 0) | (h.pv32 ? 8 : 0) | (h.c32 ? 16 : 0)),
        RAND ? r.cd : h.sp, RAND ? r.dfr : h.cp, RAND ? r.dtr : h.st, RAND ? r.amf0 : h.cth,
        RAND ? r.amf1 : h.geo.m, RAND ? r.amf2 : h.geo.mr, RAND ? r.amrf0 : h.geo.I0,
        RAND ? r.amrf1 : h.geo.I1, RAND ? r.amrf2 : h.geo.kc0, RAND ? r.amt0 : h.geo.kc1,
        RAND ? r.amt1 : h.geo.ra0, RAND ? r.amt2 : h.geo.ra1, RAND ? r.ouf0 : h.geo.dimx,
        RAND ? r.ouf1 : h.geo.dimy, RAND ? r.out2 : h.geo.speed, RAND ? r.tick : h.geo.rx};
#pragma unroll
    for (int k = 0; k < SPILL_N; ++k) s[k] = v[k];
}
template <bool RAND>
SD void unspill(Hot& h, SpillSlot s, const Params& P, uint64_t env_id) {
    double v[SPILL_N];
#pragma unroll
    for (int k = 0; k < SPILL_N; ++k) v[k] = s[k];
    h.v0 = v[0]; h.v1 = v[1]; h.v2 = v[2]; h.w0 = v[3]; h.w1 = v[4]; h.w2 = v[5];
    h.a0 = v[6]; h.a1 = v[7]; h.a2 = v[8]; h.al0 = v[9]; h.al1 = v[10]; h.al2 = v[11];
    h.e0 = v[12]; h.e1 = v[13]; h.e2 = v[14]; h.p0 = v[15]; h.p1 = v[16]; h.p2 = v[17];
    h.q0 = v[18]; h.q1 = v[19]; h.q2 = v[20]; h.g0 = v[21]; h.g1 = v[22]; h.g2 = v[23];
    h.L = v[24]; h.W = v[25]; h.V = v[26]; h.pV = v[27]; h.com = v[28]; h.comr = v[29]; h.coma = v[30];
    h.pI0 = v[31]; h.pI1 = v[32]; h.pI2 = v[33]; h.ct = v[34]; h.time = v[35];
    h.refill = v[36]; h.jet = v[37]; h.coast = v[38]; h.c = v[39]; h.cr = v[40]; h.rr = v[41];
    h.turn = v[42]; h.d0 = v[43]; h.d1 = v[44]; h.d2 = v[45];
    const int fl = (int)v[46];
    h.phase = fl & 3; h.g32 = (fl & 4) != 0; h.pv32 = (fl & 8) != 0; h.c32 = (fl & 16) != 0;
    h.env_id = env_id;
    if (RAND) {
        Hot::Rnd& r = h.rnd;
        r.cd = v[47]; r.dfr = v[48]; r.dtr = v[49]; r.amf0 = v[50]; r.amf1 = v[51]; r.amf2 = v[52];
        r.amrf0 = v[53]; r.amrf1 = v[54]; r.amrf2 = v[55]; r.amt0 = v[56]; r.amt1 = v[57];
        r.amt2 = v[58]; r.ouf0 = v[59]; r.ouf1 = v[60]; r.out2 = v[61]; r.tick = v[62];
        refresh_derived(h, P);
    } else {
        h.sp = v[47]; h.cp = v[48]; h.st = v[49]; h.cth = v[50];
        h.geo.m = v[51]; h.geo.mr = v[52]; h.geo.I0 = v[53]; h.geo.I1 = v[54]; h.geo.kc0 = v[55];
        h.geo.kc1 = v[56]; h.geo.ra0 = v[57]; h.geo.ra1 = v[58]; h.geo.dimx = v[59]; h.geo.dimy = v[60];
        h.geo.speed = v[61]; h.geo.rx = v[62];
        geo_recips(h.geo);
    }
    cycle_bounds(h);
}

/* Switching a randomisation feature off (an extension: the reference only
 * has enable_*): coefficients back to the means, OU processes calm. */
SD void calm_env(double* S, const Params& P, int64_t i, bool coefficients, bool ou) {
    if (coefficients) {
        SrCoef k;
        sr_coef_means(&k);
        SF(SALP_F_CD) = k.cd; SF(SALP_F_DFR) = k.dfr; SF(SALP_F_DTR) = k.dtr;
        for (int j = 0; j < 3; ++j) {
            SF(SALP_F_AMF0 + j) = k.amf[j]; SF(SALP_F_AMRF0 + j) = k.amrf[j];
            SF(SALP_F_AMT0 + j) = k.amt[j]; SF(SALP_F_AMRT0 + j) = k.amrt[j];
        }
    }
    if (ou)
        for (int j = 0; j < 3; ++j) { SF(SALP_F_OUF0 + j) = 0.0; SF(SALP_F_OUT0 + j) = 0.0; }
}

/* Robot / Nozzle / SalpRobotEnv constructors (src/robot.py:20-47, 261-412) */
SD void construct_env(double* S, const Params& P, int64_t i) {
    for (int f = 0; f < SALP_NUM_FIELDS; ++f) SF(f) = 0.0;
    if (SALP_COLD_BLOCK)
        for (int k = kLayout.n_cold; k < COLD_SLOTS; ++k) S[P.cold_off + (size_t)i * COLD_SLOTS + k] = 0.0;
    const Core c0 = core(P.L0, P.W0, false);
    const double V = water_volume(P, c0, false);
    const Geo g = make_geo(P, c0, P.L0, P.W0, V, V, false, false, water_mass(P, V, false));
    SF(SALP_F_LENGTH) = P.L0; SF(SALP_F_WIDTH) = P.W0;
    SF(SALP_F_VOLUME) = V; SF(SALP_F_PREV_VOLUME) = V;
    SF(SALP_F_PREV_I0) = g.I0; SF(SALP_F_PREV_I1) = g.I1; SF(SALP_F_PREV_I2) = g.I1;
    /* Robot.__init__ runs before set_environment: density 1000 */
    SF(SALP_F_COM) = center_of_mass(P, c0, 1000.0 * V, false);
    SF(SALP_F_PHASE) = REST;
    /* make_env: nozzle.set_angles(init angles) */
    SF(SALP_F_ANGLE1) = P.init_angle1; SF(SALP_F_ANGLE2) = P.init_angle2;
    SF(SALP_F_TURN_TIME) = fabs(P.init_angle1 - 0.0) / P.angle_speed +
                           fabs(P.init_angle2 - 0.0) / P.angle_speed;
    SrCoef k;
    sr_coef_means(&k);
    SF(SALP_F_CD) = k.cd; SF(SALP_F_DFR) = k.dfr; SF(SALP_F_DTR) = k.dtr;
    for (int j = 0; j < 3; ++j) {
        SF(SALP_F_AMF0 + j) = k.amf[j]; SF(SALP_F_AMRF0 + j) = k.amrf[j];
        SF(SALP_F_AMT0 + j) = k.amt[j]; SF(SALP_F_AMRT0 + j) = k.amrt[j];
    }
}

#undef SF
}  // namespace salp

#endif /* SALP_DEVICE_H */
