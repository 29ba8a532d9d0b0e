/*
 * oracle/salp_oracle.c — CPU restatement of the SALP hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This is the checker, never the product: only
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it
 * (through oracle/oracle.py).  The product path (libsalp.so) never links it.
 *
 * It restates, literally and object-per-env, the reference Python code of
 * Avielstein/GRASP_LAB_SALP:
 *   src/dynamics.py   — Newton/Euler solves, frame maps, force/torque models
 *   src/geometry.py   — cycle-time fits, body geometry, mass properties
 *   src/robot.py      — Nozzle IK, Robot state machine and integrator
 *   src/salp_robot_env.py — reset / step / reward / observation / metrics
 * keeping every 3x3 matrix the reference builds and the evaluation order of
 * NumPy 2.2 + OpenBLAS (salp_math.h np_* helpers), in fp64, with
 * -ffp-contract=off.  Each function cites the reference lines it follows.
 *
 * Parity is pinned against the reference itself: tests/golden/ fixtures were
 * produced by running /root/reference/src under the stand-ins of
 * tests/golden/make_golden.py, and tests/test_oracle_golden.py checks this file
 * against them.  Randomness the reference takes from the global np.random
 * (targets, obstacles) is injected (oracle_reset_to) or, for batched
 * rollouts, drawn from the same Philox mapping the device uses.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/salp.h"
#include "../grasp_lab_salp_amd/csrc/salp_math.h"
#include "../grasp_lab_salp_amd/csrc/salp_philox.h"
#include "../grasp_lab_salp_amd/csrc/salp_random.h"

#ifdef _OPENMP
#include <omp.h>
#endif

/* ------------------------------------------------------------------ types */
typedef struct { double v[3]; } V3;
typedef struct { double m[3][3]; } M3;

static V3 v3(double a, double b, double c) { V3 r; r.v[0] = a; r.v[1] = b; r.v[2] = c; return r; }
static V3 vzero(void) { return v3(0.0, 0.0, 0.0); }
static V3 vadd(V3 a, V3 b) { return v3(a.v[0] + b.v[0], a.v[1] + b.v[1], a.v[2] + b.v[2]); }
static V3 vsub(V3 a, V3 b) { return v3(a.v[0] - b.v[0], a.v[1] - b.v[1], a.v[2] - b.v[2]); }
static V3 vneg(V3 a) { return v3(-a.v[0], -a.v[1], -a.v[2]); }
static V3 vmuls(V3 a, double s) { return v3(a.v[0] * s, a.v[1] * s, a.v[2] * s); }
static V3 vmul(V3 a, V3 b) { return v3(a.v[0] * b.v[0], a.v[1] * b.v[1], a.v[2] * b.v[2]); }
static V3 vdivs(V3 a, double s) { return v3(a.v[0] / s, a.v[1] / s, a.v[2] / s); }
static V3 vdiv(V3 a, V3 b) { return v3(a.v[0] / b.v[0], a.v[1] / b.v[1], a.v[2] / b.v[2]); }
static M3 mzero(void) { M3 r; memset(&r, 0, sizeof r); return r; }
static M3 mdiag(double a, double b, double c) { M3 r = mzero(); r.m[0][0] = a; r.m[1][1] = b; r.m[2][2] = c; return r; }
static M3 madd(M3 a, M3 b) { M3 r; for (int i = 0; i < 3; ++i) for (int j = 0; j < 3; ++j) r.m[i][j] = a.m[i][j] + b.m[i][j]; return r; }
static M3 msub(M3 a, M3 b) { M3 r; for (int i = 0; i < 3; ++i) for (int j = 0; j < 3; ++j) r.m[i][j] = a.m[i][j] - b.m[i][j]; return r; }
static M3 mdivs(M3 a, double s) { M3 r; for (int i = 0; i < 3; ++i) for (int j = 0; j < 3; ++j) r.m[i][j] = a.m[i][j] / s; return r; }
static M3 msmul(double s, M3 a) { M3 r; for (int i = 0; i < 3; ++i) for (int j = 0; j < 3; ++j) r.m[i][j] = s * a.m[i][j]; return r; }
/* A @ B (dgemm order) */
static M3 mmul(M3 a, M3 b) {
    M3 r;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j)
            r.m[i][j] = np_dot_fwd(a.m[i][0], a.m[i][1], a.m[i][2], b.m[0][j], b.m[1][j], b.m[2][j]);
    return r;
}
/* A @ v, A C-contiguous (dgemv order) */
static V3 mvec(M3 a, V3 x) {
    V3 r;
    for (int i = 0; i < 3; ++i)
        r.v[i] = np_matvec_row(a.m[i][0], a.m[i][1], a.m[i][2], x.v[0], x.v[1], x.v[2]);
    return r;
}
/* A.T @ v (transposed view) */
static V3 mTvec(M3 a, V3 x) {
    V3 r;
    for (int i = 0; i < 3; ++i)
        r.v[i] = np_dot_fwd(a.m[0][i], a.m[1][i], a.m[2][i], x.v[0], x.v[1], x.v[2]);
    return r;
}
/* np.cross: multiply then subtract, per component (the first product fused
 * into the difference in the SALP_FMA build, salp_math.h sm_mad) */
static V3 cross(V3 a, V3 b) {
    return v3(sm_mad(a.v[1], b.v[2], -(a.v[2] * b.v[1])), sm_mad(a.v[2], b.v[0], -(a.v[0] * b.v[2])),
              sm_mad(a.v[0], b.v[1], -(a.v[1] * b.v[0])));
}
/* a * s + b per component (b + a * s of the reference, fused with SALP_FMA) */
static V3 vmad(V3 a, double s, V3 b) {
    return v3(sm_mad(a.v[0], s, b.v[0]), sm_mad(a.v[1], s, b.v[1]), sm_mad(a.v[2], s, b.v[2]));
}
/* a * b + c per component */
static V3 vmadv(V3 a, V3 b, V3 c) {
    return v3(sm_mad(a.v[0], b.v[0], c.v[0]), sm_mad(a.v[1], b.v[1], c.v[1]), sm_mad(a.v[2], b.v[2], c.v[2]));
}
static double norm3(V3 a) { return np_norm3(a.v[0], a.v[1], a.v[2]); }
static double pymax(double a, double b) { return b > a ? b : a; } /* Python max(a, b) */

/* NumPy 2 / NEP 50: a Python float combined with an np.float32 is converted
 * to float32 and the operation is done in float32.  `contraction` is an
 * np.float32 (the float32 action times 0.06), so in REFILL past refill_time the
 * body length/width and everything computed from them are float32 values.
 * These helpers are the float32 building blocks (C float arithmetic, one
 * rounding per operation, FLT_EVAL_METHOD 0). */
static float sqf(float x) { return (float)((double)x * (double)x); } /* f32 ** 2 */
static float cubef(float x) {                                          /* f32 ** 3 */
    double p = (double)x * (double)x;          /* exact */
    double h = p * (double)x, e = sm_fma(p, (double)x, -h);
    float r = (float)h;
    double d = h - (double)r;
    double ulp = (double)nextafterf(r, d > 0 ? INFINITY : -INFINITY) - (double)r;
    if (d != 0.0 && fabs(d) * 2.0 == fabs(ulp) && e != 0.0) /* tie broken by the tail */
        r = ((e > 0) == (d > 0)) ? nextafterf(r, d > 0 ? INFINITY : -INFINITY) : r;
    return r;
}

/* ------------------------------------------------------------- constants */
#define DT 0.01                                    /* src/robot.py:293 */
#define PI 3.141592653589793
static const double COS_GAMMA = 0x1.6a09e667f3bcdp-1; /* np.cos(np.pi/4), glibc */
static const double SIN_GAMMA = 0x1.6a09e667f3bccp-1; /* np.sin(np.pi/4), glibc */
/* np.polyfit fits of src/geometry.py:6-25, exact fp64 outputs */
static const double REFILL_C[3] = {-0x1.f3ffffffffffcp+8, 0x1.5bffffffffffcp+6, -0x1.ccccccccccccbp-2};
static const double PROPUL_C[3] = {-0x1.f400000000001p+7, 0x1.97ffffffffffep+4, -0x1.0000000000003p-3};
enum { REFILL = 0, JET = 1, COAST = 2, REST = 3 };  /* src/robot.py:252-257 */

/* ---------------------------------------------------------------- Nozzle */
typedef struct {
    double length1, length2, length3, area, mass;
    double angle1, angle2, prev_angle1, prev_angle2;
    double yaw, prev_yaw, current_yaw;
    double angle_speed, turn_time;
    M3 R_nm, R_mb, R_br;
} Nozzle;

/* src/robot.py:187-208 */
static void nozzle_rotation_matrices(Nozzle* n) {
    M3 rt = mzero(), rn = mzero(), rm = mzero(), rb = mzero();
    rt.m[0][0] = COS_GAMMA; rt.m[0][2] = -SIN_GAMMA; rt.m[1][1] = 1.0;
    rt.m[2][0] = SIN_GAMMA; rt.m[2][2] = COS_GAMMA;
    double s2, c2, s1, c1;
    sm_sincos(n->angle2, &s2, &c2);
    sm_sincos(n->angle1, &s1, &c1);
    rn.m[0][0] = c2; rn.m[0][1] = -s2; rn.m[1][0] = s2; rn.m[1][1] = c2; rn.m[2][2] = 1.0;
    rm.m[0][0] = c1; rm.m[0][1] = -s1; rm.m[1][0] = s1; rm.m[1][1] = c1; rm.m[2][2] = 1.0;
    rb.m[0][2] = -1.0; rb.m[1][1] = 1.0; rb.m[2][0] = 1.0;
    n->R_nm = mmul(rt, rn);
    n->R_mb = rm;
    n->R_br = rb;
}
/* src/robot.py:173-185 */
static double nozzle_turn_time(const Nozzle* n) {
    double d1 = fabs(n->angle1 - n->prev_angle1), d2 = fabs(n->angle2 - n->prev_angle2);
    return d1 / n->angle_speed + d2 / n->angle_speed;
}
/* src/robot.py:50-60 */
static void nozzle_set_angles(Nozzle* n, double a1, double a2) {
    n->angle1 = a1; n->angle2 = a2;
    n->turn_time = nozzle_turn_time(n);
    nozzle_rotation_matrices(n);
}
/* src/robot.py:62-69 */
static void nozzle_set_yaw_angle(Nozzle* n, double yaw) { n->prev_yaw = n->yaw; n->yaw = yaw; }
/* src/robot.py:71-98; yaw32: the yaw is an np.float32 (env path), so np.cos /
 * np.sin run in float32 */
static void nozzle_solve_angles(Nozzle* n, int yaw32) {
    n->prev_angle1 = n->angle1;
    n->prev_angle2 = n->angle2;
    double sy, cy;
    if (yaw32) {
        float s, c;
        sm_np_sincosf((float)n->yaw, &s, &c);        /* np.cos/np.sin of a float32 */
        sy = s; cy = c;
    } else {
        sm_sincos(n->yaw, &sy, &cy);
    }
    V3 td = vneg(v3(cy, sy, 0.0));                   /* -np.array([cos, sin, 0]) */
    td = mTvec(n->R_br, td);                         /* R_br.transpose() @ td */
    double val2 = 2.0 * td.v[2] - 1.0;
    if (val2 < -1.0) val2 = -1.0;
    if (val2 > 1.0) val2 = 1.0;
    n->angle2 = sm_acos(val2);
    if (n->angle2 <= -PI) n->angle2 += 2 * PI;
    else if (n->angle2 > PI) n->angle2 -= 2 * PI;
    if (n->angle2 == 0.0) {
        n->angle1 = 0.0;
    } else {
        double s2, c2;
        sm_sincos(n->angle2, &s2, &c2);
        double a = 0.5 * (c2 - 1.0);
        double b = sqrt(2.0) * s2 / 2.0;
        double c = td.v[1];
        double val1 = c / sqrt(a * a + b * b);
        if (val1 < -1.0) val1 = -1.0;
        if (val1 > 1.0) val1 = 1.0;
        n->angle1 = sm_asin(val1) - sm_atan2(b, a);
    }
    if (n->angle1 <= -PI) n->angle1 += 2 * PI;
    else if (n->angle1 > PI) n->angle1 -= 2 * PI;
}
/* src/robot.py:101-108 (cosmetic yaw interpolation, kept for completeness) */
static void nozzle_step(Nozzle* n, double time) {
    if (time < n->turn_time) {
        double ratio = time / n->turn_time;
        n->current_yaw = n->prev_yaw + ratio * (n->yaw - n->prev_yaw);
    } else {
        n->current_yaw = n->yaw;
    }
}
/* src/robot.py:138-150 */
static V3 nozzle_direction(const Nozzle* n) {
    V3 d = v3(COS_GAMMA, 0.0, SIN_GAMMA);
    return mvec(mmul(mmul(n->R_br, n->R_mb), n->R_nm), d);
}
/* src/robot.py:152-170 */
static V3 nozzle_middle_position(const Nozzle* n) {
    V3 base = v3(0.0, 0.0, n->length1), mid = v3(0.0, 0.0, n->length2);
    return mvec(n->R_br, vadd(base, mvec(n->R_mb, mid)));
}

/* ------------------------------------------------------- Robot + Env object */
typedef struct {
    Nozzle nz;
    /* physical parameters src/robot.py:285-295 */
    double dry_mass, buoy_mass, skin_mass, tube_mass, init_length, init_width, max_contraction;
    double density, tube_volume;
    /* coefficients src/robot.py:300-308 (means, or the draw of
     * Robot._randomize_parameters :594-628 when dynamics randomisation is on) */
    double discharge_coefficient, drag_force_ratio, drag_torque_ratio;
    M3 amf, amrf, amt, amrt;
    /* randomisation switches (SalpParams) and their Philox stream
     * (grasp_lab_salp_amd/csrc/salp_random.h): seed, global env id, the
     * set_control and tick counters, OUDisturbance states src/robot.py:210-242 */
    int rand_dyn, rand_dist, rand_act, rand_obs, latency;
    uint64_t seed, env_id;
    double rng_ctl, rng_tick;
    V3 ou_force, ou_torque;
    double trans_range[3][2], rot_range[3][2];
    /* control src/robot.py:311-316 */
    double contraction, contract_rate, release_rate, refill_time, jet_time, coast_time;
    int c32; /* contraction is an np.float32 (env path) rather than a Python float */
    int phase, cycle;
    double time, cycle_time;
    /* dynamic properties; g32: length/width/area/volume/water_mass/mass are
     * np.float32 values, pv32: prev_water_volume/prev_water_mass are */
    int g32, pv32;
    double length, width, volume, water_mass, prev_water_volume, prev_water_mass;
    V3 area;
    M3 mass, mass_rate, prev_I;
    V3 com, prev_com, com_rate, prev_com_rate, com_acc;
    V3 jet_velocity, jet_force, jet_torque, drag_force, drag_torque, coriolis_force,
        coriolis_torque, added_mass_force, added_mass_torque, asymmetry_torque, deform_torque,
        acceleration_force, tcd, rcd;
    V3 pw, pos, ppos, v, vw, avg_v, acc, eta, eta_rate, w, avg_w, alpha, ang, pang;
    /* env */
    int width_px, height_px, num_obstacles, max_cycles;
    double obstacle_radius, target_radius, tank_margin;
    float target[2];
    float obst[SALP_MAX_OBSTACLES][2];
    int n_obst;
    double prev_dist;
    float action[3];
    double prev_a2; /* prev_action[2] (float32 value, or 0.0 fp64 right after reset) */
    /* episode trackers, kept as running sums */
    double ep_len, ep_return, path_len, last_px, last_py, sum_a0, sum_a1, sum_abs_a2, sum_vel,
        init_dist, sum_r[7];
    /* in-flight env-step + RNG counters */
    int pending;
    double step_count, episode;
} Obj;

/* ------------------------------------------------ geometry.py restated */
/* src/geometry.py:14-15, 25-26.  c32: the compression is an np.float32 (env
 * path), so compression**2 is float32; a Python float squares in float64. */
static double poly_time(double c, int c32, const double* k) {
    double sq = c32 ? (double)((float)c * (float)c) : c * c;
    return k[0] * sq + k[1] * c + k[2];
}
/* src/geometry.py:39-50; with an np.float32 contraction (c32) `L0 - c` is a
 * py float - np.float32 = np.float32 */
static double compute_length(int st, double ct, double refill, double turn, double L0, double c,
                             double cr, double rr, int c32, int* is32) {
    *is32 = 0;
    double Lc = c32 ? (double)((float)L0 - (float)c) : L0 - c;
    if (st == REFILL) {
        if (ct < refill) return L0 - ct * cr;
        *is32 = c32;
        return Lc;
    }
    if (st == JET) return Lc + (ct - pymax(refill, turn)) * rr;
    return L0;
}
/* src/geometry.py:53-64 */
static double compute_width(int st, double ct, double refill, double turn, double W0, double c,
                            double cr, double rr, int c32, int* is32) {
    *is32 = 0;
    double Wc = c32 ? (double)((float)W0 + (float)c) : W0 + c;
    if (st == REFILL) {
        if (ct < refill) return W0 + ct * cr;
        *is32 = c32;
        return Wc;
    }
    if (st == JET) return Wc - (ct - pymax(refill, turn)) * rr;
    return W0;
}
/* src/geometry.py:67-75 */
static V3 compute_csa(double L, double W, int f32) {
    if (f32) {
        float wh = (float)W / 2.0f, lh = (float)L / 2.0f, pi = (float)PI;
        return v3((double)(pi * wh * wh), (double)(pi * lh * wh), (double)(pi * lh * wh));
    }
    double wh = W / 2.0, lh = L / 2.0;
    return v3(PI * wh * wh, PI * lh * wh, PI * lh * wh);
}
/* src/geometry.py:78-81 */
static double compute_water_volume(double L, double W, int f32) {
    if (f32) {
        float lh = (float)L / 2.0f, wh = (float)W / 2.0f;
        return (double)((float)((4.0 / 3.0) * PI) * lh * sqf(wh));
    }
    double wh = W / 2.0;
    return (4.0 / 3.0) * PI * (L / 2.0) * (wh * wh);
}
/* src/geometry.py:104-123 */
static V3 compute_drag_coefficient(double L, double W, double L0, double W0, double maxc,
                                   const double rg[3][2], int f32) {
    double init_aspect = L0 / W0;
    double cl = L0 - maxc, cw = L0 - cl + W0;
    double end_aspect = cl / cw;
    double nr;
    if (f32) {
        float aspect = (float)L / (float)W;
        nr = (double)((aspect - (float)end_aspect) / (float)(init_aspect - end_aspect));
    } else {
        double aspect = L / W;
        nr = (aspect - end_aspect) / (init_aspect - end_aspect);
    }
    if (nr < 0.0) nr = 0.0;
    if (nr > 1.0) nr = 1.0;
    V3 r;
    for (int i = 0; i < 3; ++i) r.v[i] = rg[i][1] - nr * (rg[i][1] - rg[i][0]);
    return r;
}
/* src/geometry.py:133-183 (mass_scalar and jet_moment_arm are unused there) */
static M3 compute_inertia_matrix_f32(double L, double W, double nozzle_mass) {
    const double mass_buoy = 0.195, skin_mass = 0.145, tube_mass = 0.414;
    const double tube_volume = 3.14159265358979 * (0.029 * 0.029) * 0.15;
    const double density = 1000.0;
    float lh = (float)L / 2.0f, wh = (float)W / 2.0f;
    float lh2 = sqf(lh), wh2 = sqf(wh);
    M3 I_buoy = madd(mdiag(1.0 / 12.0 * mass_buoy * (0.0 + 0.0), 1.0 / 12.0 * mass_buoy * (0.0 + 0.0),
                           1.0 / 12.0 * mass_buoy * (0.0 + 0.0)),
                     msmul(mass_buoy, mdiag(0.0, (double)lh2, (double)lh2)));
    double net_tube_mass = tube_mass - tube_volume * density;
    float t8 = sqf(lh - 0.08f);
    M3 I_tube = madd(mdiag(0.5 * net_tube_mass * 0.0, 1.0 / 12.0 * net_tube_mass * (3.0 * 0.0 + 0.0),
                           1.0 / 12.0 * net_tube_mass * (3.0 * 0.0 + 0.0)),
                     msmul(net_tube_mass, mdiag(0.0, (double)t8, (double)t8)));
    float p1 = (float)(1.0 / 3.0 * skin_mass);
    M3 I_skin = mdiag((double)(p1 * (wh2 + wh2)), (double)(p1 * (lh2 + wh2)), (double)(p1 * (lh2 + wh2)));
    float wme = (float)density * (float)compute_water_volume(L, W, 1);
    float k = 0.2f * wme;
    M3 I_water = mdiag((double)(k * (wh2 + wh2)), (double)(k * (lh2 + wh2)), (double)(k * (lh2 + wh2)));
    float n25 = sqf(lh + 0.025f);
    M3 I_nozzle = madd(mdiag(1.0 / 12.0 * nozzle_mass * (0.0 + 0.0), 1.0 / 12.0 * nozzle_mass * (0.0 + 0.0),
                             1.0 / 12.0 * nozzle_mass * (0.0 + 0.0)),
                       msmul(nozzle_mass, mdiag(0.0, (double)n25, (double)n25)));
    return madd(madd(madd(madd(I_buoy, I_tube), I_skin), I_water), I_nozzle);
}
static M3 compute_inertia_matrix(double L, double W, double nozzle_mass, int f32) {
    if (f32) return compute_inertia_matrix_f32(L, W, nozzle_mass);
    const double mass_buoy = 0.195, skin_mass = 0.145, tube_mass = 0.414;
    const double tube_volume = 3.14159265358979 * (0.029 * 0.029) * 0.15; /* (0.058/2.0)**2 */
    const double density = 1000.0;
    double lh = L / 2.0, wh = W / 2.0;
    double lh2 = lh * lh, wh2 = wh * wh;
    M3 I_buoy = madd(mdiag(1.0 / 12.0 * mass_buoy * (0.0 + 0.0), 1.0 / 12.0 * mass_buoy * (0.0 + 0.0),
                           1.0 / 12.0 * mass_buoy * (0.0 + 0.0)),
                     msmul(mass_buoy, mdiag(0.0, lh2, lh2)));
    double net_tube_mass = tube_mass - tube_volume * density;
    double t8 = lh - 0.08;
    M3 I_tube = madd(mdiag(0.5 * net_tube_mass * 0.0, 1.0 / 12.0 * net_tube_mass * (3.0 * 0.0 + 0.0),
                           1.0 / 12.0 * net_tube_mass * (3.0 * 0.0 + 0.0)),
                     msmul(net_tube_mass, mdiag(0.0, t8 * t8, t8 * t8)));
    M3 I_skin = mdiag(1.0 / 3.0 * skin_mass * (wh2 + wh2), 1.0 / 3.0 * skin_mass * (lh2 + wh2),
                      1.0 / 3.0 * skin_mass * (lh2 + wh2));
    double wme = density * compute_water_volume(L, W, 0);
    M3 I_water = mdiag(0.2 * wme * (wh2 + wh2), 0.2 * wme * (lh2 + wh2), 0.2 * wme * (lh2 + wh2));
    double n25 = lh + 0.025;
    M3 I_nozzle = madd(mdiag(1.0 / 12.0 * nozzle_mass * (0.0 + 0.0), 1.0 / 12.0 * nozzle_mass * (0.0 + 0.0),
                             1.0 / 12.0 * nozzle_mass * (0.0 + 0.0)),
                       msmul(nozzle_mass, mdiag(0.0, n25 * n25, n25 * n25)));
    return madd(madd(madd(madd(I_buoy, I_tube), I_skin), I_water), I_nozzle);
}
/* src/geometry.py:186-203 (x component; y and z are exactly zero) */
static V3 compute_center_of_mass(double L, double W, double tube_volume, double nozzle_mass,
                                 double buoy_mass, double skin_mass, double tube_mass,
                                 double water_mass, int f32) {
    if (f32) {
        float Lf = (float)L;
        float pbx = Lf / 2.0f, ptx = Lf / 2.0f - 0.08f, pnx = -Lf / 2.0f - 0.025f + 0.05f;
        float wme = 1000.0f * (float)compute_water_volume(L, W, 1);
        double P = 1000.0 * tube_volume;
        double num = (double)wme * 0.0 - P * (double)ptx;
        float den = wme - (float)P;
        double pwx = num / (double)den;
        float total = (float)(tube_mass + nozzle_mass + buoy_mass + skin_mass) + (float)water_mass;
        double x = (tube_mass * (double)ptx + nozzle_mass * (double)pnx + buoy_mass * (double)pbx +
                    skin_mass * 0.0 + water_mass * pwx) / (double)total;
        return v3(x, 0.0, 0.0);
    }
    double pos_buoy = L / 2, pos_tube = L / 2 - 0.08, pos_nozzle = -L / 2 - 0.025 + 0.05;
    double wme = 1000.0 * compute_water_volume(L, W, 0);
    double pos_water = (wme * 0.0 - 1000.0 * tube_volume * pos_tube) / (wme - 1000.0 * tube_volume);
    double total_mass = tube_mass + nozzle_mass + buoy_mass + skin_mass + water_mass;
    double x = (tube_mass * pos_tube + nozzle_mass * pos_nozzle + buoy_mass * pos_buoy +
                skin_mass * 0.0 + water_mass * pos_water) / total_mass;
    return v3(x, 0.0, 0.0);
}

/* --------------------------------------------------- Robot getters */
/* src/robot.py:1051-1066 */
static V3 r_csa(const Obj* o) { return compute_csa(o->length, o->width, o->g32); }
static double r_water_volume(const Obj* o) {
    if (o->g32)
        return (double)((float)compute_water_volume(o->length, o->width, 1) - (float)o->tube_volume);
    return compute_water_volume(o->length, o->width, 0) - o->tube_volume;
}
static double r_water_mass(const Obj* o) {
    if (o->g32) return (double)((float)o->density * (float)r_water_volume(o));
    return o->density * r_water_volume(o);
}
static M3 r_get_mass(Obj* o) {
    o->water_mass = r_water_mass(o);
    double t = o->g32 ? (double)((float)o->dry_mass + (float)o->water_mass + (float)o->nz.mass)
                      : o->dry_mass + o->water_mass + o->nz.mass;
    return mdiag(t, t, t);
}
/* (water_mass - prev_water_mass) / dt: float32 only if both operands are */
static double mass_rate_value(const Obj* o) {
    if (o->g32 && o->pv32)
        return (double)(((float)o->water_mass - (float)o->prev_water_mass) / (float)DT);
    return (o->water_mass - o->prev_water_mass) / DT;
}
static M3 r_get_mass_rate(const Obj* o) {
    double rate = mass_rate_value(o);
    return mdiag(rate, rate, rate);
}
/* src/robot.py:881-896 */
static M3 r_get_inertia(const Obj* o) {
    return compute_inertia_matrix(o->length, o->width, o->nz.mass, o->g32);
}
static M3 r_get_inertia_rate(Obj* o) {
    M3 I_rate = mdivs(msub(r_get_inertia(o), o->prev_I), DT);
    o->prev_I = r_get_inertia(o);
    return I_rate;
}
/* src/robot.py:898-922 */
static V3 r_get_com(const Obj* o) {
    return compute_center_of_mass(o->length, o->width, o->tube_volume, o->nz.mass, o->buoy_mass,
                                  o->skin_mass, o->tube_mass, o->water_mass, o->g32);
}
static V3 r_get_com_rate(Obj* o) {
    V3 r = vdivs(vsub(r_get_com(o), o->prev_com), DT);
    o->prev_com = r_get_com(o);
    return r;
}
static V3 r_get_com_acc_rate(Obj* o) {
    V3 r = vdivs(vsub(o->com_rate, o->prev_com_rate), DT);
    o->prev_com_rate = o->com_rate;
    return r;
}
/* src/robot.py:931-932, src/geometry.py:126-130 */
static V3 r_jet_moment_arm(const Obj* o) {
    return vadd(nozzle_middle_position(&o->nz), v3(-o->length / 2.0, 0.0, 0.0));
}
/* src/robot.py:1028-1038 */
static double r_current_length(const Obj* o, int* is32) {
    return compute_length(o->phase, o->cycle_time, o->refill_time, o->nz.turn_time, o->init_length,
                          o->contraction, o->contract_rate, o->release_rate, o->c32, is32);
}
static double r_current_width(const Obj* o, int* is32) {
    return compute_width(o->phase, o->cycle_time, o->refill_time, o->nz.turn_time, o->init_width,
                         o->contraction, o->contract_rate, o->release_rate, o->c32, is32);
}
static V3 r_trans_cd(const Obj* o) {
    return compute_drag_coefficient(o->length, o->width, o->init_length, o->init_width,
                                    o->max_contraction, o->trans_range, o->g32);
}
static V3 r_rot_cd(const Obj* o) {
    return compute_drag_coefficient(o->length, o->width, o->init_length, o->init_width,
                                    o->max_contraction, o->rot_range, o->g32);
}

/* ----------------------------------------------------- dynamics.py restated */
/* src/dynamics.py:87-94 */
static V3 compute_jet_velocity(int st, double volume, double prev_volume, double dt,
                               double nozzle_area, V3 dir, int both32) {
    if (st != JET) return vzero();
    double jet_speed;
    if (both32) {
        float volume_rate = ((float)volume - (float)prev_volume) / (float)dt;
        jet_speed = (double)(volume_rate / (float)nozzle_area);
    } else {
        double volume_rate = (volume - prev_volume) / dt;
        jet_speed = volume_rate / nozzle_area;
    }
    return vmuls(dir, jet_speed);
}
/* src/dynamics.py:110-116 */
static V3 compute_drag_force(double density, V3 area, V3 cd, V3 vel, double ratio, int area32) {
    double vn = norm3(vel);
    double k = -0.5 * density;
    V3 ka = vmuls(area, k);
    if (area32) /* python float * float32 array -> float32 */
        for (int i = 0; i < 3; ++i) ka.v[i] = (double)((float)k * (float)area.v[i]);
#if SALP_FMA
    /* product mode (round 5): (ka cd v) (|v| + ratio), the device's form */
    V3 kv = vmul(vmul(ka, cd), vel);
    return vmuls(kv, vn + ratio);
#else
    V3 fq = vmul(vmuls(vmul(ka, cd), vn), vel);
    V3 fl = vmul(vmul(ka, cd), vel);
    return vmad(fl, ratio, fq);   /* fq + fl * ratio */
#endif
}
/* src/dynamics.py:119-128 */
static V3 compute_drag_torque(double density, V3 rcd, V3 area, V3 w, double width, double length,
                              double ratio, int f32) {
    double wn = norm3(w);
    V3 dims = f32 ? v3((double)cubef((float)width), (double)cubef((float)length), (double)cubef((float)length))
                  : v3(sm_cube(width), sm_cube(length), sm_cube(length));
    double k = -0.5 * density;
#if SALP_FMA
    /* product mode (round 5): (rcd k A w) (|w| dims + width ratio), the device's form */
    V3 aw = vmul(vmul(vmuls(rcd, k), area), w);
    const double wr = width * ratio;
    return v3(aw.v[0] * sm_fma(wn, dims.v[0], wr), aw.v[1] * sm_fma(wn, dims.v[1], wr),
              aw.v[2] * sm_fma(wn, dims.v[2], wr));
#else
    V3 tq = vmul(vmul(vmuls(vmul(vmuls(rcd, k), area), wn), w), dims);
    V3 tl = vmuls(vmul(vmul(vmuls(rcd, k), area), w), width);
    return vmad(tl, ratio, tq);   /* tq + tl * ratio */
#endif
}
/* src/dynamics.py:131-141 */
static V3 compute_added_mass_force(M3 mass, M3 amc, M3 mass_rate, M3 amrc, V3 acc, V3 w, V3 vel) {
    M3 am = mmul(mass, amc), amr = mmul(mass_rate, amrc);
#if SALP_FMA
    /* am and amr are products of diagonal matrices (exactly diagonal), so
     * t1 = am @ acc and t3 = amr @ vel are diag * vector, fused into the sums */
    V3 t2 = cross(w, mvec(am, vel));
    return vneg(vmadv(v3(amr.m[0][0], amr.m[1][1], amr.m[2][2]), vel,
                      vmadv(v3(am.m[0][0], am.m[1][1], am.m[2][2]), acc, t2)));
#else
    V3 t1 = mvec(am, acc), t2 = cross(w, mvec(am, vel)), t3 = mvec(amr, vel);
    return vneg(vadd(vadd(t1, t2), t3));
#endif
}
/* src/dynamics.py:144-156 */
static V3 compute_added_mass_torque(M3 I, M3 amct, M3 I_rate, M3 amrct, M3 mass, M3 amcf,
                                    V3 alpha, V3 w, V3 vel) {
    M3 am = mmul(I, amct), amr = mmul(I_rate, amrct), afm = mmul(mass, amcf);
    V3 t2 = cross(w, mvec(am, w)), t3 = mvec(amr, w);
    V3 t4 = cross(vel, mvec(afm, vel));
#if SALP_FMA
    /* am diagonal (I and amct are): t1 = am @ alpha fused into t1 + t2 */
    V3 t12 = vmadv(v3(am.m[0][0], am.m[1][1], am.m[2][2]), alpha, t2);
#else
    V3 t12 = vadd(mvec(am, alpha), t2);
#endif
    return vneg(vadd(vadd(t12, t3), t4));
}
/* src/dynamics.py:20-31 */
static V3 to_euler_angle_rate(V3 eta, V3 w) {
    double sp, cp, st, ct;
#if SALP_FMA
    /* product mode (salp_math.h, round 5): the tick's roll / pitch sin / cos,
     * and T @ w regrouped: u = sin(phi) w1 + cos(phi) w2 is both row 2 times
     * cos(theta) and, times tan(theta), row 0's tail, so one division
     * g = u / cos(theta) serves rows 0 and 2 (the device computes the same
     * expressions) */
    sm_sincos_rp2(eta.v[0], eta.v[1], &sp, &cp, &st, &ct, sm_poly());
    const double u = sm_fma(cp, w.v[2], sp * w.v[1]);
    const double g = u / ct;
    return v3(sm_fma(st, g, w.v[0]), sm_fma(-sp, w.v[2], cp * w.v[1]), g);
#endif
    sm_sincos(eta.v[0], &sp, &cp);
    sm_sincos(eta.v[1], &st, &ct);
    double tt = sm_tan(eta.v[1]);
    M3 T = mzero();
    T.m[0][0] = 1.0; T.m[0][1] = sp * tt; T.m[0][2] = cp * tt;
    T.m[1][1] = cp; T.m[1][2] = -sp;
    T.m[2][1] = sp / ct; T.m[2][2] = cp / ct;
    return mvec(T, w);
}
/* src/dynamics.py:34-58, 60-84: R = Rz @ Ry @ Rx */
static M3 rot_zyx(V3 eta) {
    double sp, cp, st, ct, ss, cs;
    sm_sincos(eta.v[0], &sp, &cp);
    sm_sincos(eta.v[1], &st, &ct);
    sm_sincos(eta.v[2], &ss, &cs);
    M3 Rx = mzero(), Ry = mzero(), Rz = mzero();
    Rx.m[0][0] = 1.0; Rx.m[1][1] = cp; Rx.m[1][2] = -sp; Rx.m[2][1] = sp; Rx.m[2][2] = cp;
    Ry.m[0][0] = ct; Ry.m[0][2] = st; Ry.m[1][1] = 1.0; Ry.m[2][0] = -st; Ry.m[2][2] = ct;
    Rz.m[0][0] = cs; Rz.m[0][1] = -ss; Rz.m[1][0] = ss; Rz.m[1][1] = cs; Rz.m[2][2] = 1.0;
    return mmul(mmul(Rz, Ry), Rx);
}
static V3 to_world_frame(V3 eta, V3 x) {
#if SALP_FMA
    /* product mode (salp_math.h, round 5): the tick's sin / cos and the three
     * plane rotations in turn, as the device's tick, finish_step and trace */
    double sp, cp, st, ct, ss, cs;
    sm_sincos_rp2(eta.v[0], eta.v[1], &sp, &cp, &st, &ct, sm_poly());
    sm_sincos_yaw_p(eta.v[2], &ss, &cs, sm_poly());
    V3 r;
    sm_world_frame(sp, cp, st, ct, ss, cs, x.v[0], x.v[1], x.v[2], r.v);
    return r;
#else
    return mvec(rot_zyx(eta), x);
#endif
}
static V3 to_body_frame(V3 eta, V3 x) { return mTvec(rot_zyx(eta), x); }

/* --------------------------------------------------------- Robot methods */
/* src/robot.py:261-412 (constructor, minus history buffers) */
static void robot_init(Obj* o, const SalpParams* p) {
    memset(o, 0, sizeof *o);
    Nozzle* n = &o->nz;
    n->length1 = p->nozzle_length1; n->length2 = p->nozzle_length2; n->length3 = p->nozzle_length3;
    n->area = p->nozzle_area; n->mass = p->nozzle_mass;
    n->angle_speed = 31 * PI / 30;
    nozzle_rotation_matrices(n);
    o->dry_mass = p->dry_mass; o->buoy_mass = 0.195; o->skin_mass = 0.145; o->tube_mass = 0.414;
    o->init_length = p->init_length; o->init_width = p->init_width;
    o->max_contraction = p->max_contraction;
    o->density = 1000.0;
    o->tube_volume = PI * (0.029 * 0.029) * 0.15; /* np.pi * (0.058 / 2)**2 * 0.15 */
    o->discharge_coefficient = 0.3; o->drag_force_ratio = 0.25; o->drag_torque_ratio = 0.1;
    o->amf = mdiag(0.5, 0.6, 0.6); o->amrf = mdiag(0.2, 0.2, 0.2);
    o->amt = mdiag(0.3, 0.6, 0.6); o->amrt = mdiag(0.2, 0.2, 0.2);
    const double tr[3][2] = {{1.5, 2.5}, {2.5, 1.5}, {2.5, 1.5}};
    const double rr[3][2] = {{0.1, 0.3}, {0.5, 0.2}, {0.5, 0.2}};
    memcpy(o->trans_range, tr, sizeof tr);
    memcpy(o->rot_range, rr, sizeof rr);
    o->phase = REST;
    o->length = o->init_length; o->width = o->init_width;
    o->area = r_csa(o);
    o->volume = r_water_volume(o);
    o->water_mass = r_water_mass(o);
    o->prev_water_volume = o->volume;
    o->prev_water_mass = o->water_mass;
    o->mass = r_get_mass(o);
    o->mass_rate = r_get_mass_rate(o);
    o->prev_I = r_get_inertia(o);
    o->com = r_get_com(o);
    o->prev_com = o->com;
    o->tcd = r_trans_cd(o);
    o->rcd = r_rot_cd(o);
    /* make_env: robot.nozzle.set_angles(...), robot.set_environment(density) */
    nozzle_set_angles(n, p->init_angle1, p->init_angle2);
    o->density = p->density;
    /* env constructor parameters src/salp_robot_env.py:35-56 */
    o->width_px = p->width; o->height_px = p->height;
    o->num_obstacles = p->num_obstacles; o->obstacle_radius = p->obstacle_radius;
    o->max_cycles = p->max_cycles;
    o->tank_margin = 50; o->target_radius = 0.2;
    o->rand_dyn = p->dynamics_randomization != 0; o->rand_dist = p->disturbances != 0;
    o->rand_act = p->action_randomization != 0; o->rand_obs = p->observation_randomization != 0;
    o->latency = p->latency != 0;
}

/* src/robot.py:452-501 */
static void robot_reset(Obj* o) {
    o->time = 0.0; o->cycle_time = 0.0; o->cycle = 0; o->phase = REST;
    o->pw = vzero(); o->pos = vzero(); o->ppos = vzero(); o->v = vzero(); o->vw = vzero();
    o->acc = vzero(); o->eta = vzero(); o->eta_rate = vzero(); o->w = vzero(); o->alpha = vzero();
    o->ang = vzero(); o->pang = vzero();
    o->com = r_get_com(o);          /* geometry of the previous episode */
    o->prev_com = o->com;
    o->com_rate = r_get_com_rate(o);
    o->prev_com_rate = o->com_rate;
    o->com_acc = r_get_com_acc_rate(o);
    o->length = o->init_length; o->width = o->init_width;
    o->g32 = 0;
    o->area = r_csa(o);
    o->volume = r_water_volume(o);
    o->water_mass = r_water_mass(o);
    o->mass = r_get_mass(o);
    o->prev_water_volume = o->volume;
    o->prev_water_mass = o->water_mass;
    o->pv32 = 0;
    o->mass_rate = r_get_mass_rate(o);
    o->prev_I = r_get_inertia(o);
    o->tcd = r_trans_cd(o);
    o->rcd = r_rot_cd(o);
    o->ou_force = vzero();             /* force_disturbance.reset() :454 */
    o->ou_torque = vzero();            /* torque_disturbance.reset() :455 */
}

/* src/robot.py:553-561 / 594-628 */
static void robot_coefficients(Obj* o) {
    SrCoef k;
    if (o->rand_dyn) {
        sr_draw_coefs(o->seed, o->env_id, (uint64_t)o->rng_ctl, &k);
        o->rng_ctl += 1.0;
    } else {
        sr_coef_means(&k);
    }
    o->discharge_coefficient = k.cd; o->drag_force_ratio = k.dfr; o->drag_torque_ratio = k.dtr;
    o->amf = mdiag(k.amf[0], k.amf[1], k.amf[2]);
    o->amrf = mdiag(k.amrf[0], k.amrf[1], k.amrf[2]);
    o->amt = mdiag(k.amt[0], k.amt[1], k.amt[2]);
    o->amrt = mdiag(k.amrt[0], k.amrt[1], k.amrt[2]);
}

/* src/robot.py:544-592 */
static void robot_set_control(Obj* o, double contraction, double coast_time, double a1, double a2,
                              int c32) {
    robot_coefficients(o);
    o->avg_v = vzero(); o->avg_w = vzero();
    o->contraction = contraction; o->coast_time = coast_time;
    o->c32 = c32;
    nozzle_set_angles(&o->nz, a1, a2);
    o->cycle += 1;
    o->cycle_time = 0.0;
    o->refill_time = poly_time(o->contraction, c32, REFILL_C);
    o->jet_time = poly_time(o->contraction, c32, PROPUL_C);
    o->contract_rate = o->refill_time > 0 ? o->contraction / o->refill_time : 0.0;
    o->release_rate = o->jet_time > 0 ? o->contraction / o->jet_time : 0.0;
}

/* src/robot.py:640-649 */
static void robot_update_state(Obj* o) {
    double m = pymax(o->refill_time, o->nz.turn_time);
    if (o->cycle_time <= m) o->phase = REFILL;
    else if (o->cycle_time <= m + o->jet_time) o->phase = JET;
    else if (o->cycle_time <= m + o->jet_time + o->coast_time) o->phase = COAST;
    else o->phase = REST;
}
/* src/robot.py:651-668 */
static void robot_update_properties(Obj* o) {
    o->prev_water_volume = o->volume;
    o->pv32 = o->g32;
    o->prev_water_mass = o->pv32 ? (double)((float)o->prev_water_volume * (float)o->density)
                                 : o->prev_water_volume * o->density;
    int l32, w32;
    o->length = r_current_length(o, &l32);
    o->width = r_current_width(o, &w32);
    o->g32 = l32;
    o->area = r_csa(o);
    o->volume = r_water_volume(o);
    o->mass = r_get_mass(o);
    o->mass_rate = r_get_mass_rate(o);
    o->com = r_get_com(o);
    o->com_rate = r_get_com_rate(o);
    o->com_acc = r_get_com_acc_rate(o);
    o->tcd = r_trans_cd(o);
    o->rcd = r_rot_cd(o);
}

/* src/robot.py:937-951 */
static V3 robot_jet_force(Obj* o) {
    o->jet_velocity = compute_jet_velocity(o->phase, o->volume, o->prev_water_volume, DT,
                                           o->nz.area, nozzle_direction(&o->nz), o->g32 && o->pv32);
    if (o->phase != JET) return vzero();
    M3 mr = r_get_mass_rate(o);
    return vmuls(mvec(mr, o->jet_velocity), -o->discharge_coefficient);
}
/* src/robot.py:789-823 */
static V3 robot_newton(Obj* o) {
    o->coriolis_force = vneg(cross(o->w, mvec(r_get_mass(o), o->v)));
    o->drag_force = compute_drag_force(o->density, o->area, o->tcd, o->v, o->drag_force_ratio, o->g32);
    o->jet_force = robot_jet_force(o);
    o->added_mass_force = compute_added_mass_force(o->mass, o->amf, o->mass_rate, o->amrf, o->acc,
                                                   o->w, o->v);
    V3 noise = vzero();
    if (o->rand_dist) {
        /* force_disturbance.sample(), then force_noise[-1] = 0 zeroes the
         * process's own z state (the array is shared); the torque process is
         * stepped with the same tick's draws (its x, y are zeroed likewise) */
        double z0, z1, z2;
        sr_normals3(o->seed, o->env_id, (uint64_t)o->rng_tick, &z0, &z1, &z2);
        o->rng_tick += 1.0;
        o->ou_force = v3(sr_ou_step(o->ou_force.v[0], SR_OU_FORCE_THETA, SR_OU_FORCE_SIGMA, z0),
                         sr_ou_step(o->ou_force.v[1], SR_OU_FORCE_THETA, SR_OU_FORCE_SIGMA, z1), 0.0);
        o->ou_torque = v3(0.0, 0.0, sr_ou_step(o->ou_torque.v[2], SR_OU_TORQUE_THETA, SR_OU_TORQUE_SIGMA, z2));
        noise = o->ou_force;
    }
    o->mass = r_get_mass(o);
    V3 a_tan = cross(o->alpha, o->com);
    V3 a_cen = cross(o->w, cross(o->w, o->com));
    V3 a_cor = vmuls(cross(o->w, o->com_rate), 2.0);
    V3 a_rec = o->com_acc;
    V3 a_sum = vadd(vadd(vadd(a_cen, a_cor), a_tan), a_rec);
    o->acceleration_force = vmuls(a_sum, o->mass.m[0][0]);
    /* + acceleration_force, the product fused with SALP_FMA */
    V3 total = vmad(a_sum, o->mass.m[0][0],
                    vadd(vadd(vadd(vadd(o->jet_force, o->drag_force), o->added_mass_force), o->coriolis_force),
                         noise));
    /* np.linalg.solve(diag(m), F) == F / m (probed); product mode: F times
     * the correctly rounded 1 / m (the device keeps 1 / m with the geometry) */
#if SALP_FMA
    return v3(total.v[0] * (1.0 / o->mass.m[0][0]), total.v[1] * (1.0 / o->mass.m[1][1]),
              total.v[2] * (1.0 / o->mass.m[2][2]));
#else
    return v3(total.v[0] / o->mass.m[0][0], total.v[1] / o->mass.m[1][1], total.v[2] / o->mass.m[2][2]);
#endif
}
/* src/robot.py:825-851 */
static V3 robot_euler(Obj* o) {
    o->asymmetry_torque = v3(0.0, 0.0, 0.00 * norm3(o->v));
    o->coriolis_torque = vneg(cross(o->w, mvec(r_get_inertia(o), o->w)));
    o->drag_torque = compute_drag_torque(o->density, o->rcd, o->area, o->w, o->width, o->length,
                                         o->drag_torque_ratio, o->g32);
    o->jet_torque = cross(r_jet_moment_arm(o), o->jet_force);
    const M3 Ir_w = r_get_inertia_rate(o);
    o->deform_torque = vneg(mvec(Ir_w, o->w));
    M3 I_a = r_get_inertia(o);
    M3 Ir_a = r_get_inertia_rate(o); /* prev_I was just updated: exactly zero */
    o->added_mass_torque = compute_added_mass_torque(I_a, o->amt, Ir_a, o->amrt, r_get_mass(o),
                                                     o->amf, o->alpha, o->w, o->v);
    V3 noise = o->rand_dist ? o->ou_torque : vzero();
    M3 I = r_get_inertia(o);
    V3 part = vadd(vadd(vadd(o->jet_torque, o->drag_torque), o->coriolis_torque), o->asymmetry_torque);
#if SALP_FMA
    /* + deform_torque = -(I_rate @ w), I_rate diagonal: fused into the sum */
    part = vmadv(v3(-Ir_w.m[0][0], -Ir_w.m[1][1], -Ir_w.m[2][2]), o->w, part);
#else
    part = vadd(part, o->deform_torque);
#endif
    V3 total = vadd(vadd(part, o->added_mass_torque), noise);
#if SALP_FMA
    /* product mode: times the correctly rounded 1 / I (as robot_newton) */
    return v3(total.v[0] * (1.0 / I.m[0][0]), total.v[1] * (1.0 / I.m[1][1]), total.v[2] * (1.0 / I.m[2][2]));
#else
    return v3(total.v[0] / I.m[0][0], total.v[1] / I.m[1][1], total.v[2] / I.m[2][2]);
#endif
}
/* src/robot.py:860-875 */
static void robot_update_motion_states(Obj* o) {
    /* x + rate * dt: fused with SALP_FMA */
    o->v = vmad(o->acc, DT, o->v);
    o->w = vmad(o->alpha, DT, o->w);
    o->eta_rate = to_euler_angle_rate(o->eta, o->w);
    o->eta = vmad(o->eta_rate, DT, o->eta);
    o->vw = to_world_frame(o->eta, o->v);
    o->pw = vmad(o->vw, DT, o->pw);
    o->pos = vmad(o->v, DT, o->pos);
    o->ang = vmad(o->w, DT, o->ang);
}
/* src/robot.py:670-678, 854-858 */
static void robot_step(Obj* o) {
    o->acc = robot_newton(o);
    o->alpha = robot_euler(o);
    robot_update_motion_states(o);
    o->cycle_time += DT;
    o->time += DT;
    nozzle_step(&o->nz, o->cycle_time);
    robot_update_state(o);
    robot_update_properties(o);
}
/* One history sample (src/robot.py:687-738) in the SalpTraceCol layout of
 * include/salp.h, column col at rec[col * rs].  first: sample 0 of a cycle
 * (force values, euler_angle_rate and nozzle yaw are NaN there). */
static void robot_record(Obj* o, double* rec, int64_t rs, int first) {
#define PUT(c, x) rec[(int64_t)(c) * rs] = (x)
#define PUT3(c, vec) do { V3 v_ = (vec); PUT(c, v_.v[0]); PUT((c) + 1, v_.v[1]); PUT((c) + 2, v_.v[2]); } while (0)
    PUT(SALP_T_STATE, o->phase);
    PUT3(SALP_T_PW0, o->pw); PUT3(SALP_T_V0, o->v); PUT3(SALP_T_ACC0, o->acc);
    PUT3(SALP_T_ETA0, o->eta); PUT3(SALP_T_W0, o->w); PUT3(SALP_T_ALPHA0, o->alpha);
    PUT(SALP_T_LENGTH, o->length); PUT(SALP_T_WIDTH, o->width);
    PUT3(SALP_T_AREA0, o->area);
    PUT(SALP_T_VOLUME, o->volume);
    PUT(SALP_T_MASS, o->mass.m[0][0]);
    PUT(SALP_T_MASS_RATE, o->mass_rate.m[0][0]);
    M3 I = r_get_inertia(o);
    PUT(SALP_T_I0, I.m[0][0]); PUT(SALP_T_I1, I.m[1][1]); PUT(SALP_T_I2, I.m[2][2]);
    PUT3(SALP_T_TCD0, o->tcd); PUT3(SALP_T_RCD0, o->rcd);
    PUT(SALP_T_COM, o->com.v[0]); PUT(SALP_T_COM_RATE, o->com_rate.v[0]);
    PUT(SALP_T_COM_ACC, o->com_acc.v[0]);
    /* get_front_position_world_frame (src/robot.py:924-928) */
    PUT3(SALP_T_FRONT_W0, to_world_frame(o->eta, v3(o->length / 2, 0.0, 0.0)));
    if (first) {
        for (int k = SALP_T_FIRST_FORCE; k < SALP_TRACE_DIM; ++k) PUT(k, NAN);
        PUT(SALP_T_ETAR0, NAN); PUT(SALP_T_ETAR1, NAN); PUT(SALP_T_ETAR2, NAN);
        PUT(SALP_T_NOZZLE_YAW, NAN);
        return;
    }
    PUT3(SALP_T_ETAR0, o->eta_rate);
    PUT(SALP_T_NOZZLE_YAW, o->nz.current_yaw);
    PUT3(SALP_T_JETV0, o->jet_velocity); PUT3(SALP_T_JETF0, o->jet_force);
    PUT3(SALP_T_JETT0, o->jet_torque); PUT3(SALP_T_DRAGF0, o->drag_force);
    PUT3(SALP_T_DRAGT0, o->drag_torque); PUT3(SALP_T_CORF0, o->coriolis_force);
    PUT3(SALP_T_CORT0, o->coriolis_torque); PUT3(SALP_T_AMF0, o->added_mass_force);
    PUT3(SALP_T_AMT0, o->added_mass_torque); PUT3(SALP_T_DEFT0, o->deform_torque);
    PUT3(SALP_T_ACCF0, o->acceleration_force);
#undef PUT3
#undef PUT
}

/* src/robot.py:740-777; returns the tick count.  rows != NULL: record
 * (record=True), sample t of this env at rows + t * SALP_TRACE_DIM * rs. */
/* The loop's prologue (src/robot.py:740-748): the previous cycle's
 * displacement over this cycle's total time.  Returns the total. */
static double robot_cycle_prologue(Obj* o) {
    double total = pymax(o->refill_time, o->nz.turn_time) + o->jet_time + o->coast_time;
    o->avg_v = vdivs(vsub(o->pos, o->ppos), total);
    o->avg_w = vdivs(vsub(o->ang, o->pang), total);
    o->ppos = o->pos;
    o->pang = o->ang;
    return total;
}
static int64_t robot_step_through_cycle(Obj* o, double* rows, int64_t rs, int64_t max_samples,
                                        int64_t* n_samples) {
    const double total = robot_cycle_prologue(o);
    if (rows && max_samples > 0) robot_record(o, rows, rs, 1);
    int64_t n = 0;
    while (o->cycle_time < total) {
        robot_step(o);
        ++n;
        if (rows && n < max_samples) robot_record(o, rows + n * SALP_TRACE_DIM * rs, rs, 0);
    }
    if (n_samples) *n_samples = n + 1;
    return n;
}

/* ------------------------------------------------------ Env methods */
static double dist_to_target(const Obj* o) {
    return np_norm2(o->pw.v[0] - (double)o->target[0], o->pw.v[1] - (double)o->target[1]);
}
/* src/salp_robot_env.py:651-670 */
static void env_observation(const Obj* o, float* obs) {
    V3 d = v3((double)o->target[0] - o->pw.v[0], (double)o->target[1] - o->pw.v[1], 0.0);
    V3 db = to_body_frame(o->eta, d);
    double heading = sm_atan2(db.v[1], db.v[0]);
    obs[0] = (float)db.v[0]; obs[1] = (float)db.v[1];
    obs[2] = (float)o->v.v[0]; obs[3] = (float)o->v.v[1];
    obs[4] = (float)o->w.v[2]; obs[5] = (float)heading;
    for (int k = 0; k < o->num_obstacles; ++k) {
        if (k < o->n_obst) {
            obs[6 + 2 * k] = (float)((double)o->obst[k][0] - o->pw.v[0]);
            obs[7 + 2 * k] = (float)((double)o->obst[k][1] - o->pw.v[1]);
        } else {
            obs[6 + 2 * k] = 0.0f; obs[7 + 2 * k] = 0.0f; /* reference would shorten obs */
        }
    }
}
/* src/salp_robot_env.py:114-155 with target/obstacles supplied */
static void env_reset_with(Obj* o, const float* target, const float* obst, int n_obst, float* obs) {
    o->target[0] = target[0]; o->target[1] = target[1];
    o->n_obst = n_obst;
    for (int k = 0; k < SALP_MAX_OBSTACLES; ++k) {
        o->obst[k][0] = k < n_obst ? obst[2 * k] : 0.0f;
        o->obst[k][1] = k < n_obst ? obst[2 * k + 1] : 0.0f;
    }
    robot_reset(o);
    o->prev_dist = dist_to_target(o);
    o->prev_a2 = 0.0;
    o->action[0] = o->action[1] = o->action[2] = 0.0f;
    o->ep_len = 0; o->ep_return = 0.0; o->path_len = 0.0;
    o->last_px = o->pw.v[0]; o->last_py = o->pw.v[1];
    o->sum_a0 = o->sum_a1 = o->sum_abs_a2 = 0.0;
    o->sum_vel = np_norm2(o->vw.v[0], o->vw.v[1]);
    o->init_dist = o->prev_dist;
    for (int i = 0; i < 7; ++i) o->sum_r[i] = 0.0;
    o->episode += 1.0;
    o->pending = 0;
    if (obs) env_observation(o, obs);
}
/* Batched reset draws: src/salp_robot_env.py:449-533 ("random") and 535-559,
 * with np.random replaced by Philox(seed; env id, episode, draw). */
static void env_draw_reset(const Obj* o, uint64_t seed, uint64_t env_id, float* target,
                           float* obst, int* n_obst) {
    const double scale = 200.0;
    double x_min = (-o->width_px / 2.0 + o->tank_margin) / scale;
    double x_max = (o->width_px / 2.0 - o->tank_margin) / scale;
    double y_min = (-o->height_px / 2.0 + o->tank_margin) / scale;
    double y_max = (o->height_px / 2.0 - o->tank_margin) / scale;
    uint64_t ep = (uint64_t)o->episode;
    double u0, u1;
    sp_reset_pair(seed, env_id, ep, 0u, &u0, &u1);
    double tx = x_min + (x_max - x_min) * u0, ty = y_min + (y_max - y_min) * u1;
    if (tx < x_min) tx = x_min;
    if (tx > x_max) tx = x_max;
    if (ty < y_min) ty = y_min;
    if (ty > y_max) ty = y_max;
    target[0] = (float)tx; target[1] = (float)ty;
    const double min_clear = 0.5;
    const double sep = 2 * o->obstacle_radius + 0.1;
    int n = 0;
    for (int k = 0; k < o->num_obstacles; ++k) {
        for (int att = 0; att < 200; ++att) {
            sp_reset_pair(seed, env_id, ep, (uint32_t)(1 + k * 200 + att), &u0, &u1);
            float px = (float)(x_min + (x_max - x_min) * u0);
            float py = (float)(y_min + (y_max - y_min) * u1);
            float ds = sqrtf(sm_fmaf(py, py, px * px));
            float dx = px - target[0], dy = py - target[1];
            float dt = sqrtf(sm_fmaf(dy, dy, dx * dx));
            int close = 0;
            for (int j = 0; j < n; ++j) {
                float ex = px - obst[2 * j], ey = py - obst[2 * j + 1];
                if ((double)sqrtf(sm_fmaf(ey, ey, ex * ex)) < sep) close = 1;
            }
            if ((double)ds > min_clear && (double)dt > min_clear && !close) {
                obst[2 * n] = px; obst[2 * n + 1] = py; ++n;
                break;
            }
        }
    }
    *n_obst = n;
}

/* src/salp_robot_env.py:166-174 (float32 arithmetic, NumPy 2 promotion) */
static void env_rescale_action(const float* a, float* r) {
    r[0] = a[0] * 0.06f;
    r[1] = a[1] * 10.0f;
    r[2] = a[2] * (float)(PI / 2);
}

/* src/salp_robot_env.py:196-209 (step up to step_through_cycle) */
static void env_begin(Obj* o, const float* action) {
    o->action[0] = action[0]; o->action[1] = action[1]; o->action[2] = action[2];
    float r[3];
    env_rescale_action(action, r);
    if (o->rand_act) {   /* _randomize_actions (:176-181): Python floats from here */
        double ra[3];
        sr_randomize_action(o->seed, o->env_id, (uint64_t)o->step_count, r, ra);
        nozzle_set_yaw_angle(&o->nz, ra[2]);
        nozzle_solve_angles(&o->nz, 0);
        robot_set_control(o, ra[0], ra[1], o->nz.angle1, o->nz.angle2, 0);
    } else {
        nozzle_set_yaw_angle(&o->nz, (double)r[2]);
        nozzle_solve_angles(&o->nz, 1);
        robot_set_control(o, (double)r[0], (double)r[1], o->nz.angle1, o->nz.angle2, 1);
    }
}
/* src/salp_robot_env.py:196-210 (first half of step: through the cycle) */
static int64_t env_begin_and_run_cycle(Obj* o, const float* action) {
    env_begin(o, action);
    return robot_step_through_cycle(o, NULL, 0, 0, NULL);
}

/* src/salp_robot_env.py:349-397 */
static double env_reward(Obj* o, double* comp) {
    double dx = o->pw.v[0] - (double)o->target[0], dy = o->pw.v[1] - (double)o->target[1];
    double cur = np_norm2(dx, dy);
    double r_track = (-cur + o->prev_dist) * 100;
    o->prev_dist = cur;
    V3 db = to_body_frame(o->eta, v3(dx, dy, 0.0));
    double r_heading = -0.5 * fabs(sm_atan2(-db.v[1], -db.v[0]));
    double r_smooth;
    if (o->ep_len == 0) { /* prev_action is the fp64 zeros of reset() */
        double ch = (double)o->action[2] - o->prev_a2;
        r_smooth = -1.0 * (ch * ch);
    } else {              /* float32 - float32, float32 ** 2 */
        float ch = o->action[2] - (float)o->prev_a2;
        r_smooth = (double)(-(ch * ch));
    }
    double r_yaw = -10.0 * fabs(o->avg_w.v[2]);
    double r_time = -0.1;
    double r_sideslip = -100.0 * fabs(o->avg_v.v[1]);
    double r_obstacle = 0.0;
    if (o->n_obst > 0) {
        double md = 0.0;
        for (int k = 0; k < o->n_obst; ++k) {
            double d = np_norm2(o->pw.v[0] - (double)o->obst[k][0], o->pw.v[1] - (double)o->obst[k][1]);
            if (k == 0 || d < md) md = d;
        }
        double danger = 2.0 * o->obstacle_radius;
        if (md < danger) r_obstacle = -1.0 * (1.0 - md / danger);
    }
    comp[0] = r_track; comp[1] = r_heading; comp[2] = r_smooth; comp[3] = r_yaw;
    comp[4] = r_time; comp[5] = r_sideslip; comp[6] = r_obstacle;
    return r_track + r_heading + r_smooth + r_yaw + r_time + r_sideslip + r_obstacle;
}
/* src/salp_robot_env.py:561-568 */
static int env_hit_obstacle(const Obj* o) {
    int l32;
    double L = r_current_length(o, &l32);
    double thr = l32 ? (double)((float)o->obstacle_radius + (float)L / 2.0f) : o->obstacle_radius + L / 2;
    for (int k = 0; k < o->n_obst; ++k) {
        double d = np_norm2(o->pw.v[0] - (double)o->obst[k][0], o->pw.v[1] - (double)o->obst[k][1]);
        if (d < thr) return 1;
    }
    return 0;
}
/* src/salp_robot_env.py:237-299 (second half of step) and 399-447 (metrics) */
static double env_finish_step(Obj* o, float* obs, uint8_t* term_out, uint8_t* trunc_out,
                              double* info) {
    /* episode_positions / velocities / distances */
    double px = o->pw.v[0], py = o->pw.v[1];
    o->path_len = o->path_len + np_norm2(px - o->last_px, py - o->last_py);
    o->last_px = px; o->last_py = py;
    o->sum_vel = o->sum_vel + np_norm2(o->vw.v[0], o->vw.v[1]);
    double dist = dist_to_target(o);
    double comp[7];
    double reward = env_reward(o, comp);
    env_observation(o, obs);
    if (o->rand_obs) sr_randomize_obs(o->seed, o->env_id, (uint64_t)o->step_count, obs);  /* :253-254 */
    int hit = env_hit_obstacle(o);
    int done = 0, truncated = 0;
    if (dist < o->target_radius) { done = 1; reward += 500.0; }
    else if (dist > 5.0) { truncated = 1; reward -= 200.0; }
    if (hit) { truncated = 1; reward -= 200.0; }
    if (o->cycle >= o->max_cycles) { truncated = 1; reward -= 50.0; }
    /* episode accumulators (episode_actions, episode_rewards, components) */
    o->ep_len += 1.0;
    o->ep_return = o->ep_return + reward;
    o->sum_a0 = o->sum_a0 + (double)o->action[0];
    o->sum_a1 = o->sum_a1 + (double)o->action[1];
    o->sum_abs_a2 = o->sum_abs_a2 + (double)fabsf(o->action[2]);
    for (int i = 0; i < 7; ++i) o->sum_r[i] = o->sum_r[i] + comp[i];
    if (info) {
        for (int i = 0; i < SALP_INFO_DIM; ++i) info[i] = 0.0;
        for (int i = 0; i < 7; ++i) info[SALP_INFO_R_TRACK + i] = comp[i];
        info[SALP_INFO_EP_RETURN] = o->ep_return;
        info[SALP_INFO_EP_LEN] = o->ep_len;
        info[SALP_INFO_HIT_OBSTACLE] = hit;
        if (done || truncated) {
            double dd = np_norm2(px - 0.0, py - 0.0);
            info[SALP_INFO_HAS_METRICS] = 1.0;
            info[SALP_INFO_PATH_LENGTH] = o->path_len;
            info[SALP_INFO_DIRECT_DISTANCE] = dd;
            info[SALP_INFO_PATH_EFFICIENCY] = o->path_len > 0 ? dd / o->path_len : 0.0;
            info[SALP_INFO_FINAL_DISTANCE] = dist;
            info[SALP_INFO_INITIAL_DISTANCE] = o->init_dist;
            info[SALP_INFO_AVG_COMPRESSION] = o->sum_a0 / o->ep_len;
            info[SALP_INFO_AVG_COAST_TIME] = o->sum_a1 / o->ep_len;
            info[SALP_INFO_AVG_NOZZLE_ANGLE] = o->sum_abs_a2 / o->ep_len;
            info[SALP_INFO_AVG_VELOCITY] = o->sum_vel / (o->ep_len + 1.0);
            for (int i = 0; i < 7; ++i) info[SALP_INFO_AVG_R_TRACK + i] = o->sum_r[i] / o->ep_len;
        }
    }
    o->prev_a2 = (double)o->action[2];
    o->pending = 0;
    if (o->latency) {    /* src/salp_robot_env.py:292-297 */
        double lat = sr_latency(o->seed, o->env_id, (uint64_t)o->step_count);
        robot_set_control(o, 0.0, lat, o->nz.angle1, o->nz.angle2, 0);
    }
    *term_out = (uint8_t)done;
    *trunc_out = (uint8_t)truncated;
    return reward;
}

/* ------------------------------------------------------ SoA pack/unpack */
#define F(s, f, n, i) (s)[(size_t)(f) * (size_t)(n) + (size_t)(i)]

static void obj_pack(const Obj* o, double* s, int64_t n, int64_t i) {
    for (int k = 0; k < 3; ++k) {
        F(s, SALP_F_V0 + k, n, i) = o->v.v[k];
        F(s, SALP_F_W0 + k, n, i) = o->w.v[k];
        F(s, SALP_F_ACC0 + k, n, i) = o->acc.v[k];
        F(s, SALP_F_ALPHA0 + k, n, i) = o->alpha.v[k];
        F(s, SALP_F_ETA0 + k, n, i) = o->eta.v[k];
        F(s, SALP_F_PW0 + k, n, i) = o->pw.v[k];
        F(s, SALP_F_POS0 + k, n, i) = o->pos.v[k];
        F(s, SALP_F_ANG0 + k, n, i) = o->ang.v[k];
        F(s, SALP_F_PPOS0 + k, n, i) = o->ppos.v[k];
        F(s, SALP_F_PANG0 + k, n, i) = o->pang.v[k];
        F(s, SALP_F_AVGV0 + k, n, i) = o->avg_v.v[k];
        F(s, SALP_F_AVGW0 + k, n, i) = o->avg_w.v[k];
        F(s, SALP_F_PREV_I0 + k, n, i) = o->prev_I.m[k][k];
    }
    F(s, SALP_F_LENGTH, n, i) = o->length;
    F(s, SALP_F_WIDTH, n, i) = o->width;
    F(s, SALP_F_VOLUME, n, i) = o->volume;
    F(s, SALP_F_PREV_VOLUME, n, i) = o->prev_water_volume;
    F(s, SALP_F_COM, n, i) = o->com.v[0];
    F(s, SALP_F_COM_RATE, n, i) = o->com_rate.v[0];
    F(s, SALP_F_COM_ACC, n, i) = o->com_acc.v[0];
    F(s, SALP_F_GEOM32, n, i) = o->g32;
    F(s, SALP_F_PVOL32, n, i) = o->pv32;
    F(s, SALP_F_CYCLE_TIME, n, i) = o->cycle_time;
    F(s, SALP_F_TIME, n, i) = o->time;
    F(s, SALP_F_REFILL_TIME, n, i) = o->refill_time;
    F(s, SALP_F_JET_TIME, n, i) = o->jet_time;
    F(s, SALP_F_COAST_TIME, n, i) = o->coast_time;
    F(s, SALP_F_CONTRACTION, n, i) = o->contraction;
    F(s, SALP_F_CONTRACT_RATE, n, i) = o->contract_rate;
    F(s, SALP_F_RELEASE_RATE, n, i) = o->release_rate;
    F(s, SALP_F_PHASE, n, i) = o->phase;
    F(s, SALP_F_CYCLE, n, i) = o->cycle;
    F(s, SALP_F_CONTR32, n, i) = o->c32;
    F(s, SALP_F_ANGLE1, n, i) = o->nz.angle1;
    F(s, SALP_F_ANGLE2, n, i) = o->nz.angle2;
    F(s, SALP_F_PREV_ANGLE1, n, i) = o->nz.prev_angle1;
    F(s, SALP_F_PREV_ANGLE2, n, i) = o->nz.prev_angle2;
    F(s, SALP_F_YAW, n, i) = o->nz.yaw;
    F(s, SALP_F_PREV_YAW, n, i) = o->nz.prev_yaw;
    F(s, SALP_F_TURN_TIME, n, i) = o->nz.turn_time;
    F(s, SALP_F_TARGET0, n, i) = o->target[0];
    F(s, SALP_F_TARGET1, n, i) = o->target[1];
    for (int k = 0; k < SALP_MAX_OBSTACLES; ++k) {
        F(s, SALP_F_OBST0 + 2 * k, n, i) = o->obst[k][0];
        F(s, SALP_F_OBST0 + 2 * k + 1, n, i) = o->obst[k][1];
    }
    F(s, SALP_F_N_OBST, n, i) = o->n_obst;
    F(s, SALP_F_PREV_DIST, n, i) = o->prev_dist;
    F(s, SALP_F_PREV_A2, n, i) = o->prev_a2;
    F(s, SALP_F_EP_LEN, n, i) = o->ep_len;
    F(s, SALP_F_EP_RETURN, n, i) = o->ep_return;
    F(s, SALP_F_PATH_LEN, n, i) = o->path_len;
    F(s, SALP_F_LAST_PX, n, i) = o->last_px;
    F(s, SALP_F_LAST_PY, n, i) = o->last_py;
    F(s, SALP_F_SUM_A0, n, i) = o->sum_a0;
    F(s, SALP_F_SUM_A1, n, i) = o->sum_a1;
    F(s, SALP_F_SUM_ABS_A2, n, i) = o->sum_abs_a2;
    F(s, SALP_F_SUM_VEL, n, i) = o->sum_vel;
    F(s, SALP_F_INIT_DIST, n, i) = o->init_dist;
    for (int k = 0; k < 7; ++k) F(s, SALP_F_SUM_R0 + k, n, i) = o->sum_r[k];
    F(s, SALP_F_ACT0, n, i) = o->action[0];
    F(s, SALP_F_ACT1, n, i) = o->action[1];
    F(s, SALP_F_ACT2, n, i) = o->action[2];
    F(s, SALP_F_PENDING, n, i) = o->pending;
    F(s, SALP_F_STEP_COUNT, n, i) = o->step_count;
    F(s, SALP_F_EPISODE, n, i) = o->episode;
    F(s, SALP_F_CD, n, i) = o->discharge_coefficient;
    F(s, SALP_F_DFR, n, i) = o->drag_force_ratio;
    F(s, SALP_F_DTR, n, i) = o->drag_torque_ratio;
    for (int k = 0; k < 3; ++k) {
        F(s, SALP_F_AMF0 + k, n, i) = o->amf.m[k][k];
        F(s, SALP_F_AMRF0 + k, n, i) = o->amrf.m[k][k];
        F(s, SALP_F_AMT0 + k, n, i) = o->amt.m[k][k];
        F(s, SALP_F_AMRT0 + k, n, i) = o->amrt.m[k][k];
        F(s, SALP_F_OUF0 + k, n, i) = o->ou_force.v[k];
        F(s, SALP_F_OUT0 + k, n, i) = o->ou_torque.v[k];
    }
    F(s, SALP_F_RNG_CTL, n, i) = o->rng_ctl;
    F(s, SALP_F_RNG_TICK, n, i) = o->rng_tick;
}

/* Rebuild the full reference object from the minimal state.  Every derived
 * attribute is a pure function of stored ones at an env-step boundary. */
static void obj_unpack(Obj* o, const SalpParams* p, const double* s, int64_t n, int64_t i, uint64_t seed,
                       int64_t env_offset) {
    robot_init(o, p);
    o->seed = seed;
    o->env_id = (uint64_t)(env_offset + i);
    for (int k = 0; k < 3; ++k) {
        o->v.v[k] = F(s, SALP_F_V0 + k, n, i);
        o->w.v[k] = F(s, SALP_F_W0 + k, n, i);
        o->acc.v[k] = F(s, SALP_F_ACC0 + k, n, i);
        o->alpha.v[k] = F(s, SALP_F_ALPHA0 + k, n, i);
        o->eta.v[k] = F(s, SALP_F_ETA0 + k, n, i);
        o->pw.v[k] = F(s, SALP_F_PW0 + k, n, i);
        o->pos.v[k] = F(s, SALP_F_POS0 + k, n, i);
        o->ang.v[k] = F(s, SALP_F_ANG0 + k, n, i);
        o->ppos.v[k] = F(s, SALP_F_PPOS0 + k, n, i);
        o->pang.v[k] = F(s, SALP_F_PANG0 + k, n, i);
        o->avg_v.v[k] = F(s, SALP_F_AVGV0 + k, n, i);
        o->avg_w.v[k] = F(s, SALP_F_AVGW0 + k, n, i);
    }
    o->prev_I = mdiag(F(s, SALP_F_PREV_I0, n, i), F(s, SALP_F_PREV_I1, n, i), F(s, SALP_F_PREV_I2, n, i));
    o->length = F(s, SALP_F_LENGTH, n, i);
    o->width = F(s, SALP_F_WIDTH, n, i);
    o->volume = F(s, SALP_F_VOLUME, n, i);
    o->prev_water_volume = F(s, SALP_F_PREV_VOLUME, n, i);
    o->com = v3(F(s, SALP_F_COM, n, i), 0.0, 0.0);
    o->prev_com = o->com;
    o->com_rate = v3(F(s, SALP_F_COM_RATE, n, i), 0.0, 0.0);
    o->prev_com_rate = o->com_rate;
    o->com_acc = v3(F(s, SALP_F_COM_ACC, n, i), 0.0, 0.0);
    o->g32 = (int)F(s, SALP_F_GEOM32, n, i);
    o->pv32 = (int)F(s, SALP_F_PVOL32, n, i);
    o->cycle_time = F(s, SALP_F_CYCLE_TIME, n, i);
    o->time = F(s, SALP_F_TIME, n, i);
    o->refill_time = F(s, SALP_F_REFILL_TIME, n, i);
    o->jet_time = F(s, SALP_F_JET_TIME, n, i);
    o->coast_time = F(s, SALP_F_COAST_TIME, n, i);
    o->contraction = F(s, SALP_F_CONTRACTION, n, i);
    o->contract_rate = F(s, SALP_F_CONTRACT_RATE, n, i);
    o->release_rate = F(s, SALP_F_RELEASE_RATE, n, i);
    o->phase = (int)F(s, SALP_F_PHASE, n, i);
    o->cycle = (int)F(s, SALP_F_CYCLE, n, i);
    o->c32 = (int)F(s, SALP_F_CONTR32, n, i);
    o->nz.angle1 = F(s, SALP_F_ANGLE1, n, i);
    o->nz.angle2 = F(s, SALP_F_ANGLE2, n, i);
    o->nz.prev_angle1 = F(s, SALP_F_PREV_ANGLE1, n, i);
    o->nz.prev_angle2 = F(s, SALP_F_PREV_ANGLE2, n, i);
    o->nz.yaw = F(s, SALP_F_YAW, n, i);
    o->nz.prev_yaw = F(s, SALP_F_PREV_YAW, n, i);
    o->nz.turn_time = F(s, SALP_F_TURN_TIME, n, i);
    nozzle_rotation_matrices(&o->nz);
    /* derived */
    o->area = r_csa(o);
    o->water_mass = r_water_mass(o);
    o->mass = r_get_mass(o);
    o->prev_water_mass = o->pv32 ? (double)((float)o->prev_water_volume * (float)o->density)
                                 : o->prev_water_volume * o->density;
    o->mass_rate = r_get_mass_rate(o);
    o->tcd = r_trans_cd(o);
    o->rcd = r_rot_cd(o);
    o->vw = to_world_frame(o->eta, o->v);
    /* env */
    o->target[0] = (float)F(s, SALP_F_TARGET0, n, i);
    o->target[1] = (float)F(s, SALP_F_TARGET1, n, i);
    for (int k = 0; k < SALP_MAX_OBSTACLES; ++k) {
        o->obst[k][0] = (float)F(s, SALP_F_OBST0 + 2 * k, n, i);
        o->obst[k][1] = (float)F(s, SALP_F_OBST0 + 2 * k + 1, n, i);
    }
    o->n_obst = (int)F(s, SALP_F_N_OBST, n, i);
    o->prev_dist = F(s, SALP_F_PREV_DIST, n, i);
    o->prev_a2 = F(s, SALP_F_PREV_A2, n, i);
    o->ep_len = F(s, SALP_F_EP_LEN, n, i);
    o->ep_return = F(s, SALP_F_EP_RETURN, n, i);
    o->path_len = F(s, SALP_F_PATH_LEN, n, i);
    o->last_px = F(s, SALP_F_LAST_PX, n, i);
    o->last_py = F(s, SALP_F_LAST_PY, n, i);
    o->sum_a0 = F(s, SALP_F_SUM_A0, n, i);
    o->sum_a1 = F(s, SALP_F_SUM_A1, n, i);
    o->sum_abs_a2 = F(s, SALP_F_SUM_ABS_A2, n, i);
    o->sum_vel = F(s, SALP_F_SUM_VEL, n, i);
    o->init_dist = F(s, SALP_F_INIT_DIST, n, i);
    for (int k = 0; k < 7; ++k) o->sum_r[k] = F(s, SALP_F_SUM_R0 + k, n, i);
    o->action[0] = (float)F(s, SALP_F_ACT0, n, i);
    o->action[1] = (float)F(s, SALP_F_ACT1, n, i);
    o->action[2] = (float)F(s, SALP_F_ACT2, n, i);
    o->pending = (int)F(s, SALP_F_PENDING, n, i);
    o->step_count = F(s, SALP_F_STEP_COUNT, n, i);
    o->episode = F(s, SALP_F_EPISODE, n, i);
    o->discharge_coefficient = F(s, SALP_F_CD, n, i);
    o->drag_force_ratio = F(s, SALP_F_DFR, n, i);
    o->drag_torque_ratio = F(s, SALP_F_DTR, n, i);
    o->amf = mdiag(F(s, SALP_F_AMF0, n, i), F(s, SALP_F_AMF1, n, i), F(s, SALP_F_AMF2, n, i));
    o->amrf = mdiag(F(s, SALP_F_AMRF0, n, i), F(s, SALP_F_AMRF1, n, i), F(s, SALP_F_AMRF2, n, i));
    o->amt = mdiag(F(s, SALP_F_AMT0, n, i), F(s, SALP_F_AMT1, n, i), F(s, SALP_F_AMT2, n, i));
    o->amrt = mdiag(F(s, SALP_F_AMRT0, n, i), F(s, SALP_F_AMRT1, n, i), F(s, SALP_F_AMRT2, n, i));
    o->ou_force = v3(F(s, SALP_F_OUF0, n, i), F(s, SALP_F_OUF1, n, i), F(s, SALP_F_OUF2, n, i));
    o->ou_torque = v3(F(s, SALP_F_OUT0, n, i), F(s, SALP_F_OUT1, n, i), F(s, SALP_F_OUT2, n, i));
    o->rng_ctl = F(s, SALP_F_RNG_CTL, n, i);
    o->rng_tick = F(s, SALP_F_RNG_TICK, n, i);
}

/* --------------------------------------------------------- exported API */
int oracle_abi_version(void) { return SALP_ABI_VERSION; }
int oracle_num_fields(void) { return SALP_NUM_FIELDS; }

/* Fresh envs: Robot/Nozzle/SalpRobotEnv constructors; the env constructor's
 * reset() is performed by a following oracle_reset*/
int oracle_init(const SalpParams* p, int64_t n, double* state) {
    for (int64_t i = 0; i < n; ++i) {
        Obj o;
        robot_init(&o, p);
        o.n_obst = 0;
        obj_pack(&o, state, n, i);
    }
    return 0;
}

int oracle_reset_to(const SalpParams* p, int64_t n, double* state, const uint8_t* mask,
                    const float* targets, const float* obstacles, const int32_t* n_obst,
                    float* obs_out, int obs_dim) {
    const uint64_t seed = 0;
    const int64_t env_offset = 0;
#pragma omp parallel for schedule(dynamic, 16)
    for (int64_t i = 0; i < n; ++i) {
        if (mask && !mask[i]) continue;
        Obj o;
        obj_unpack(&o, p, state, n, i, seed, env_offset);
        env_reset_with(&o, targets + 2 * i, obstacles + 2 * SALP_MAX_OBSTACLES * i, n_obst[i],
                       obs_out ? obs_out + (size_t)obs_dim * i : NULL);
        obj_pack(&o, state, n, i);
    }
    return 0;
}

int oracle_reset(const SalpParams* p, int64_t n, double* state, const uint8_t* mask,
                 uint64_t seed, int64_t env_offset, float* obs_out, int obs_dim) {
#pragma omp parallel for schedule(dynamic, 16)
    for (int64_t i = 0; i < n; ++i) {
        if (mask && !mask[i]) continue;
        Obj o;
        obj_unpack(&o, p, state, n, i, seed, env_offset);
        float tgt[2], obst[2 * SALP_MAX_OBSTACLES];
        int nob;
        env_draw_reset(&o, seed, (uint64_t)(env_offset + i), tgt, obst, &nob);
        env_reset_with(&o, tgt, obst, nob, obs_out ? obs_out + (size_t)obs_dim * i : NULL);
        obj_pack(&o, state, n, i);
    }
    return 0;
}

/* One env.step per env (+ optional SB3-style auto-reset with Philox draws). */
int oracle_step(const SalpParams* p, int64_t n, double* state, const float* actions,
                float* obs_out, double* reward_out, uint8_t* term_out, uint8_t* trunc_out,
                int auto_reset, float* term_obs_out, double* info_out, int64_t* ticks_out,
                uint64_t seed, int64_t env_offset, int obs_dim) {
#pragma omp parallel for schedule(dynamic, 4)
    for (int64_t i = 0; i < n; ++i) {
        Obj o;
        obj_unpack(&o, p, state, n, i, seed, env_offset);
        float obs[SALP_OBS_DIM_MAX];
        uint8_t te, tr;
        int64_t ticks = env_begin_and_run_cycle(&o, actions + 3 * i);
        o.step_count += 1.0;
        double rw = env_finish_step(&o, obs, &te, &tr, info_out ? info_out + (size_t)SALP_INFO_DIM * i : NULL);
        if (reward_out) reward_out[i] = rw;
        if (term_out) term_out[i] = te;
        if (trunc_out) trunc_out[i] = tr;
        if (ticks_out) ticks_out[i] = ticks;
        if (term_obs_out) memcpy(term_obs_out + (size_t)obs_dim * i, obs, sizeof(float) * obs_dim);
        if (auto_reset && (te || tr)) {
            float tgt[2], obst[2 * SALP_MAX_OBSTACLES];
            int nob;
            env_draw_reset(&o, seed, (uint64_t)(env_offset + i), tgt, obst, &nob);
            env_reset_with(&o, tgt, obst, nob, obs);
        }
        if (obs_out) memcpy(obs_out + (size_t)obs_dim * i, obs, sizeof(float) * obs_dim);
        obj_pack(&o, state, n, i);
    }
    return 0;
}

/* Random-action rollout (the bench workload, CPU baseline): each env runs
 * n_steps env-steps with Philox actions and auto-reset.  Returns total ticks. */
int64_t oracle_step_random(const SalpParams* p, int64_t n, double* state, int32_t n_steps,
                           uint64_t seed, int64_t env_offset, double* reward_sum, int nthreads) {
    int64_t total_ticks = 0;
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#else
    (void)nthreads;
#endif
#pragma omp parallel for schedule(dynamic, 1) reduction(+ : total_ticks)
    for (int64_t i = 0; i < n; ++i) {
        Obj o;
        obj_unpack(&o, p, state, n, i, seed, env_offset);
        double rs = 0.0;
        for (int32_t k = 0; k < n_steps; ++k) {
            float a[3], obs[SALP_OBS_DIM_MAX];
            uint8_t te, tr;
            sp_action(seed, (uint64_t)(env_offset + i), (uint64_t)o.step_count, a);
            total_ticks += env_begin_and_run_cycle(&o, a);
            o.step_count += 1.0;
            rs += env_finish_step(&o, obs, &te, &tr, NULL);
            if (te || tr) {
                float tgt[2], obst[2 * SALP_MAX_OBSTACLES];
                int nob;
                env_draw_reset(&o, seed, (uint64_t)(env_offset + i), tgt, obst, &nob);
                env_reset_with(&o, tgt, obst, nob, obs);
            }
        }
        if (reward_sum) reward_sum[i] = rs;
        obj_pack(&o, state, n, i);
    }
    return total_ticks;
}

/* Replay of sampled envs of a chained random-action rollout (the bench
 * workload, salp_rollout): env j, global id env_ids[j], is constructed and
 * reset as salp_create does, then runs n_steps[j] env-steps with Philox
 * actions and auto-reset; if ct_stop[j] >= 0 it then begins its next env-step
 * and ticks that cycle while cycle_time < ct_stop[j] (the in-flight cycle a
 * launch leaves pending: the device state's cycle_time).  The rollout-buffer
 * rows of the last `cap` env-steps go to slot (k % cap) of obs / obs_before
 * [cap][n][obs_dim], actions [cap][n][3], rewards [cap][n] (float32) and
 * dones [cap][n] (terminated | truncated << 1), as k_rollout writes them;
 * the in-flight env-step's obs_before goes to its slot too.
 * state: [NUM_FIELDS][n].  Returns the total ticks. */
int64_t oracle_replay(const SalpParams* p, int64_t n, const int64_t* env_ids, const int64_t* n_steps,
                      const double* ct_stop, uint64_t seed, double* state, int64_t cap, float* obs,
                      float* obs_before, float* actions, float* rewards, uint8_t* dones, int obs_dim,
                      int nthreads, int64_t* ticks_out) {
    int64_t total_ticks = 0;
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#else
    (void)nthreads;
#endif
#pragma omp parallel for schedule(dynamic, 1) reduction(+ : total_ticks)
    for (int64_t j = 0; j < n; ++j) {
        /* constructor, then reset (salp_create: k_construct + k_reset) */
        double s1[SALP_NUM_FIELDS];
        Obj o;
        robot_init(&o, p);
        o.n_obst = 0;
        obj_pack(&o, s1, 1, 0);
        obj_unpack(&o, p, s1, 1, 0, seed, env_ids[j]);
        const uint64_t id = (uint64_t)env_ids[j];
        float cur[SALP_OBS_DIM_MAX], tgt[2], obst[2 * SALP_MAX_OBSTACLES];
        int nob;
        env_draw_reset(&o, seed, id, tgt, obst, &nob);
        env_reset_with(&o, tgt, obst, nob, cur);
        int64_t done_ticks = 0;   /* ticks of the completed env-steps (in-flight cycle excluded) */
        for (int64_t k = 0; k < n_steps[j]; ++k) {
            float a[3], ob[SALP_OBS_DIM_MAX];
            uint8_t te, tr;
            sp_action(seed, id, (uint64_t)o.step_count, a);
            const int rec = cap > 0 && k >= n_steps[j] - cap;
            const size_t row = (size_t)(k % (cap > 0 ? cap : 1)) * (size_t)n + (size_t)j;
            if (rec && obs_before) memcpy(obs_before + row * obs_dim, cur, sizeof(float) * obs_dim);
            done_ticks += env_begin_and_run_cycle(&o, a);
            o.step_count += 1.0;
            double rw = env_finish_step(&o, ob, &te, &tr, NULL);
            if (rec) {
                if (obs) memcpy(obs + row * obs_dim, ob, sizeof(float) * obs_dim);
                if (actions) memcpy(actions + row * 3, a, sizeof(float) * 3);
                if (rewards) rewards[row] = (float)rw;
                if (dones) dones[row] = (uint8_t)(te | (tr << 1));
            }
            if (te || tr) {
                env_draw_reset(&o, seed, id, tgt, obst, &nob);
                env_reset_with(&o, tgt, obst, nob, ob);
            }
            memcpy(cur, ob, sizeof(float) * obs_dim);
        }
        total_ticks += done_ticks;
        if (ticks_out) ticks_out[j] = done_ticks;
        if (ct_stop && ct_stop[j] >= 0.0) {
            float a[3];
            sp_action(seed, id, (uint64_t)o.step_count, a);
            if (cap > 0 && obs_before)   /* the in-flight step's row: only its obs_before is written */
                memcpy(obs_before + ((size_t)(n_steps[j] % cap) * (size_t)n + (size_t)j) * obs_dim, cur,
                       sizeof(float) * obs_dim);
            env_begin(&o, a);
            const double total = robot_cycle_prologue(&o);
            while (o.cycle_time < total && o.cycle_time < ct_stop[j]) {
                robot_step(&o);
                ++total_ticks;
            }
            o.pending = 1;
        }
        obj_pack(&o, state, n, j);
    }
    return total_ticks;
}

/* Robot-only per-tick trace (src/robot.py:740-777 with record=True) for the
 * tick_trace fixture.  Row layout per recorded sample (29 doubles):
 * pw3 v3 acc3 eta3 eta_rate3 w3 alpha3 L W V m Ixx Iyy Izz com_x phase.
 * Sample 0 of each cycle is the pre-loop state, like the reference lists. */
int64_t oracle_robot_trace(const SalpParams* p, const float* actions, int n_actions, double* out,
                           int64_t max_rows) {
    Obj o;
    robot_init(&o, p);
    robot_reset(&o);
    int64_t row = 0;
    for (int c = 0; c < n_actions; ++c) {
        float r[3];
        env_rescale_action(actions + 3 * c, r);
        nozzle_set_yaw_angle(&o.nz, (double)r[2]);
        nozzle_solve_angles(&o.nz, 1);
        robot_set_control(&o, (double)r[0], (double)r[1], o.nz.angle1, o.nz.angle2, 1);
        double total = pymax(o.refill_time, o.nz.turn_time) + o.jet_time + o.coast_time;
        o.avg_v = vdivs(vsub(o.pos, o.ppos), total);
        o.avg_w = vdivs(vsub(o.ang, o.pang), total);
        o.ppos = o.pos; o.pang = o.ang;
        int first = 1;
        while (first || o.cycle_time < total) {
            if (!first) robot_step(&o);
            first = 0;
            if (row >= max_rows) return -1;
            double* q = out + 29 * row;
            M3 I = r_get_inertia(&o);
            for (int k = 0; k < 3; ++k) {
                q[0 + k] = o.pw.v[k]; q[3 + k] = o.v.v[k]; q[6 + k] = o.acc.v[k];
                q[9 + k] = o.eta.v[k]; q[12 + k] = o.eta_rate.v[k]; q[15 + k] = o.w.v[k];
                q[18 + k] = o.alpha.v[k]; q[25 + k] = I.m[k][k];
            }
            q[21] = o.length; q[22] = o.width; q[23] = o.volume; q[24] = o.mass.m[0][0];
            q[28] = o.com.v[0];
            ++row;
            if (!(o.cycle_time < total)) break;
        }
    }
    return row;
}

/* Robot / Nozzle level (include/salp.h salp_robot_*, salp_nozzle_*). */
int oracle_robot_reset(const SalpParams* p, int64_t n, double* state, const uint8_t* mask) {
    const uint64_t seed = 0;
    const int64_t env_offset = 0;
    for (int64_t i = 0; i < n; ++i) {
        if (mask && !mask[i]) continue;
        Obj o;
        obj_unpack(&o, p, state, n, i, seed, env_offset);
        robot_reset(&o);
        o.pending = 0;
        obj_pack(&o, state, n, i);
    }
    return 0;
}
int oracle_nozzle_set_angles(const SalpParams* p, int64_t n, double* state, const double* ang) {
    const uint64_t seed = 0;
    const int64_t env_offset = 0;
    for (int64_t i = 0; i < n; ++i) {
        Obj o;
        obj_unpack(&o, p, state, n, i, seed, env_offset);
        nozzle_set_angles(&o.nz, ang[2 * i], ang[2 * i + 1]);
        obj_pack(&o, state, n, i);
    }
    return 0;
}
int oracle_nozzle_solve(const SalpParams* p, int64_t n, double* state, const double* yaw, int yaw32) {
    const uint64_t seed = 0;
    const int64_t env_offset = 0;
    for (int64_t i = 0; i < n; ++i) {
        Obj o;
        obj_unpack(&o, p, state, n, i, seed, env_offset);
        nozzle_set_yaw_angle(&o.nz, yaw[i]);
        nozzle_solve_angles(&o.nz, yaw32);
        obj_pack(&o, state, n, i);
    }
    return 0;
}
int oracle_robot_set_control(const SalpParams* p, int64_t n, double* state, const double* ctl, int c32,
                             uint64_t seed, int64_t env_offset) {
    for (int64_t i = 0; i < n; ++i) {
        Obj o;
        obj_unpack(&o, p, state, n, i, seed, env_offset);
        robot_set_control(&o, ctl[4 * i], ctl[4 * i + 1], ctl[4 * i + 2], ctl[4 * i + 3], c32);
        obj_pack(&o, state, n, i);
    }
    return 0;
}
/* step_through_cycle for every env; rows/n_samples may be NULL (no record).
 * ticks_out [n] may be NULL. */
int oracle_robot_cycle(const SalpParams* p, int64_t n, double* state, double* rows,
                       int64_t max_samples, int64_t* n_samples, int64_t* ticks_out, uint64_t seed,
                       int64_t env_offset) {
#pragma omp parallel for schedule(dynamic, 4)
    for (int64_t i = 0; i < n; ++i) {
        Obj o;
        obj_unpack(&o, p, state, n, i, seed, env_offset);
        int64_t t = robot_step_through_cycle(&o, rows ? rows + i : NULL, n, max_samples,
                                             n_samples ? n_samples + i : NULL);
        o.pending = 0;
        if (ticks_out) ticks_out[i] = t;
        obj_pack(&o, state, n, i);
    }
    return 0;
}

/* Math self-test rows, same layout as salp_math_selftest (host side). */
void oracle_math_selftest(const double* x, const double* y, int64_t n, double* out) {
    for (int64_t i = 0; i < n; ++i) {
        out[0 * n + i] = sm_sin(x[i]);
        out[1 * n + i] = sm_cos(x[i]);
        out[2 * n + i] = sm_tan(x[i]);
        out[3 * n + i] = sm_atan2(x[i], y[i]);
        out[4 * n + i] = sm_asin(x[i]);
        out[5 * n + i] = sm_acos(x[i]);
        out[6 * n + i] = sm_cube(x[i]);
        float s, c;
        sm_np_sincosf((float)x[i], &s, &c);
        out[7 * n + i] = c;
        out[8 * n + i] = s;
        double snb, cnb;
        sm_sincos_nb_p(x[i], &snb, &cnb, sm_poly());
        out[9 * n + i] = snb;
        out[10 * n + i] = cnb;
        out[11 * n + i] = x[i] / y[i];   /* device: qdiv(x, rcp_of(y)) */
        double sy, cy, s0, c0, s1, c1, sz, cz, wf[3];
        sm_sincos_yaw_p(x[i], &sy, &cy, sm_poly());
        out[12 * n + i] = sy;
        out[13 * n + i] = cy;
        sm_sincos_rp2(x[i], y[i], &s0, &c0, &s1, &c1, sm_poly());
        out[14 * n + i] = s0;
        out[15 * n + i] = c0;
        out[16 * n + i] = s1;
        out[17 * n + i] = c1;
        sm_sincos_yaw_p(x[i] + y[i], &sz, &cz, sm_poly());
        sm_world_frame(s0, c0, s1, c1, sz, cz, y[i], x[i], 1.0, wf);
        out[18 * n + i] = wf[0];
        out[19 * n + i] = wf[1];
        out[20 * n + i] = wf[2];
        out[21 * n + i] = sm_atan(x[i]);
        out[22 * n + i] = sm_atan_ref(x[i]);
    }
}

void oracle_philox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0, uint32_t k1,
                   uint32_t* out) {
    sp_u32x4 r = sp_philox4x32_10(c0, c1, c2, c3, k0, k1);
    for (int i = 0; i < 4; ++i) out[i] = r.v[i];
}
