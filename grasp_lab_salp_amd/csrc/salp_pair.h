/*
 * salp_pair.h — one env's physics tick split over TWO waves (k_rollout_pair).
 *
 * k_rollout runs one env per lane: 32 768 envs (BASELINE configs[4]'s PPO
 * collection) are 512 waves, one per SIMD on half of the chip's 1 024 SIMDs,
 * whatever the workgroup shape (profiles/r3_experiments.md r3ag-r3ah).  Here
 * an env is held by the same lane of two waves of one workgroup that run
 * DIFFERENT code on different SIMDs and swap a few values through LDS once per
 * tick:
 *
 *   wave A (translation + mass side): Newton's equations (src/robot.py:
 *     789-823), v and position integration, the world-frame position update
 *     (yaw sin/cos, R v: src/dynamics.py:34-58), and in full ticks the volume /
 *     water mass / centre of mass / mass / jet rates of update_properties;
 *   wave B (rotation + shape side): Euler's equations (src/robot.py:825-851),
 *     angular velocity and Euler-angle integration (to_euler_angle_rate_jit,
 *     src/dynamics.py:20-31), roll / pitch sin/cos, and in full ticks the drag
 *     coefficients, body cubes and inertia (src/geometry.py:104-183).
 *
 * Both waves run the clock and the phase machine (cheap).  Per tick A sends
 * B the two terms of Euler's equations that need the translational state
 * (v x (M_a v) of the added-mass torque, src/dynamics.py:144-156, and the jet
 * torque r x F_jet, src/robot.py:931-935) and the next tick's mode; B sends A
 * the new angular velocity, the angular acceleration terms of the fictitious
 * forces, roll / pitch sin/cos, the yaw and the drag-force coefficients.
 *
 * Every value is computed by exactly the expression salp_device.h tick() uses
 * (same helpers, same operand order), so a pair-kernel env equals a k_rollout
 * env, and the oracle, bit for bit: tests/test_gpu_pair.py.  Only the plain
 * kernels (no randomisation, no recording) have a pair form.
 */
#ifndef SALP_PAIR_H
#define SALP_PAIR_H

#include "salp_device.h"

namespace salp {

enum PairMode { PM_FULL = 0, PM_STEADY = 1, PM_SETTLED = 2, PM_END = 3 };

/* wave A's state of one env */
struct HotA {
    double v0, v1, v2, a0, a1, a2, q0, q1, q2, p0, p1, p2;
    double L, W, V, pV, com, comr, coma;
    double ct, time, refill, jet, coast, c, cr, rr, turn, mx, b1, b2;
    double d0, d1, d2;
    double m, rm, mr, speed;                 /* mass-side geometry (+ 1/m) */
    double amv0, amv1, amv2, jf0, jf1, jf2;  /* this tick's (M_a v) and jet force, prepared */
    /* from wave B: state after the previous tick */
    double w0, w1, w2, al1, al2, sp, cp, st, cth, ss, cs, kc0, kc1;
    int phase;
    bool g32, pv32, c32;
};
/* wave B's state of one env */
struct HotB {
    double w0, w1, w2, al0, al1, al2, e0, e1, e2, g0, g1, g2, pI0, pI1, pI2;
    double sp, cp, st, cth, ss, cs;   /* sin/cos of roll, pitch (and yaw, for wave A) */
    double L, W, ct, refill, c, cr, rr, mx, b1, b2;
    double I0, I1, rI0, rI1, ra0, ra1, dimx, dimy, kc0, kc1;
    /* from wave A: this tick's v x (M_a v) and jet torque y, z */
    double X0, X1, X2, jt1, jt2;
    int phase;
    bool g32, c32;
};

/* This tick's added-mass momentum M_a v (am = m C_a, src/dynamics.py:131-141)
 * and jet force (src/robot.py:937-951), as tick() forms them from the state at
 * the start of the tick; and from them the two Euler terms wave B needs:
 * v x (M_a v) (src/dynamics.py:152) and r x F_jet, r = (mid_x - L/2, 0, 0). */
SD void pair_terms(const Params& P, double v0, double v1, double v2, double m, double mr, double speed, double d0,
                   double d1, double d2, int phase, double L, double* amv, double* jf, double* X, double* jt) {
    const double am0 = m * AMF0, am1 = m * AMF1, am2 = m * AMF2;
    amv[0] = am0 * v0; amv[1] = am1 * v1; amv[2] = am2 * v2;
    /* a settled tick never starts in JET (its previous steady tick set COAST / REST) */
    const bool jet = phase == JET;
    jf[0] = jet ? mr * (d0 * speed) * -CD : 0.0;
    jf[1] = jet ? mr * (d1 * speed) * -CD : 0.0;
    jf[2] = jet ? mr * (d2 * speed) * -CD : 0.0;
    X[0] = cross_c(v1, amv[2], v2, amv[1]);
    X[1] = cross_c(v2, amv[0], v0, amv[2]);
    X[2] = cross_c(v0, amv[1], v1, amv[0]);
    const double rx = jet_arm(P, L);
    jt[0] = -(rx * jf[2]);
    jt[1] = rx * jf[1];
}
SD void a_prepare(HotA& h, const Params& P, double* X, double* jt) {
    double amv[3], jf[3];
    pair_terms(P, h.v0, h.v1, h.v2, h.m, h.mr, h.speed, h.d0, h.d1, h.d2, h.phase, h.L, amv, jf, X, jt);
    h.amv0 = amv[0]; h.amv1 = amv[1]; h.amv2 = amv[2];
    h.jf0 = jf[0]; h.jf1 = jf[1]; h.jf2 = jf[2];
}

/* The clock and update_state's phase chain (tick(), both waves). */
template <bool STEADY>
SD void pair_clock(double& ct, int& phase, double b1, double b2, double mx) {
    ct += DT;
    if (STEADY) {
        phase = ct <= b2 ? COAST : REST;
    } else {
        int ph = ct <= b2 ? COAST : REST;
        ph = ct <= b1 ? JET : ph;
        phase = ct <= mx ? REFILL : ph;
    }
}

/* The world-frame position update of the tick just done (tick()'s
 * to_world_frame_jit block): yaw sin/cos, R at the new angles (roll / pitch
 * sin/cos from wave B), p += (R v) dt. */
SD void a_world(HotA& h, const Params&) {
    double vw[3];
    sm_world_frame(h.sp, h.cp, h.st, h.cth, h.ss, h.cs, h.v0, h.v1, h.v2, vw);
    h.p0 = sm_mad(vw[0], DT, h.p0); h.p1 = sm_mad(vw[1], DT, h.p1); h.p2 = sm_mad(vw[2], DT, h.p2);
}

/* ---------------------------------------------- the scheduled ticks */
/* Each wave's part of a tick is scheduled for instruction-level parallelism: with one wave per SIMD a wave is issue-bound only while it has
 * independent work between dependent instructions, and half a tick is a few
 * long dependence chains.  step_a / step_b compute the same values in one
 * basic block per tick kind: wave A interleaves the previous tick's
 * world-frame update (yaw sin/cos, R v), this tick's clock / phase / mass-side
 * geometry and Newton's equations (the geometry into temporaries, committed
 * after Newton, which reads the tick-start values); wave B its shape-side
 * geometry with Euler's equations, roll / pitch sin/cos (salp_math.h
 * sm_sincos_rp2), then the yaw's for wave A.  Every value is the expression tick() computes. */

/* A tick's clock, phase and (full ticks) mass-side geometry: a function of
 * wave A's own state alone.  (Computing it between publishing and waiting,
 * to fill the wait, measured slower: profiles/r4_experiments.md r4s.) */
struct PreA {
    double ct, L, W, V, com, comr, coma, m, mr, speed, rm;
    int phase;
    bool f;
};
template <int MODE>
SD PreA pre_a(const HotA& h, const Params& P, Cache32 c32) {
    constexpr bool STEADY = MODE != PM_FULL;
    double ct = h.ct;
    int phase = h.phase;
    pair_clock<STEADY>(ct, phase, h.b1, h.b2, h.mx);
    double L = h.L, W = h.W, V = h.V, com = h.com, comr = h.comr, coma = h.coma, mn = h.m, mr = h.mr, sp = h.speed,
           rmn = h.rm;
    bool f = h.g32;
    if (!STEADY) {
        body_lw(P, phase, ct, h.refill, h.mx, h.c, h.cr, h.rr, h.c32, &L, &W, &f);
        const Core c = core(L, W, false);
        V = water_volume(P, c, false);
        double wm = water_mass(P, V, false);
        com = center_of_mass(P, c, wm, false);
        mn = geo_mass(P, wm, false);
        if (f) {
            V = c32[C32_V]; wm = c32[C32_WM]; com = c32[C32_COM]; mn = c32[C32_M];
        }
        comr = div_dt(com - h.com);
        coma = div_dt(comr - h.comr);
        Geo ng;
        ng.m = mn;
        jet_rates(P, V, h.V, wm, f, h.g32, ng);   /* pV <- V, pv32 <- g32 first (tick()) */
        mr = ng.mr;
        sp = ng.speed;
        rmn = rcr(mn);
    }
    return PreA{ct, L, W, V, com, comr, coma, mn, mr, sp, rmn, phase, f};
}

/* The world-frame update owed for the previous tick (pend: it ticked), then
 * this tick with its clock / geometry g (pre_a).  Returns, for a steady tick,
 * whether the lane is settled. */
template <int MODE>
SD bool step_a_newton(HotA& h, const Params& P, const PreA& g);
template <int MODE>
SD bool step_a(HotA& h, const Params& P, const PreA& g, bool pend) {
    {   /* a_world of the previous tick, with v before this tick's Newton */
        double vw[3];
        sm_world_frame(h.sp, h.cp, h.st, h.cth, h.ss, h.cs, h.v0, h.v1, h.v2, vw);
        const double p0 = sm_mad(vw[0], DT, h.p0), p1 = sm_mad(vw[1], DT, h.p1), p2 = sm_mad(vw[2], DT, h.p2);
        h.p0 = pend ? p0 : h.p0;
        h.p1 = pend ? p1 : h.p1;
        h.p2 = pend ? p2 : h.p2;
    }
    return step_a_newton<MODE>(h, P, g);
}
/* Newton's equations with the tick-start values, then the tick's clock and
 * mass-side properties committed. */
template <int MODE>
SD bool step_a_newton(HotA& h, const Params& P, const PreA& g) {
    constexpr bool STEADY = MODE != PM_FULL, SETTLED = MODE == PM_SETTLED;
    const double m = h.m;
    double mv0 = m * h.v0, mv1 = m * h.v1, mv2 = m * h.v2;
    double cf0 = -cross_c(h.w1, mv2, h.w2, mv1), cf1 = -cross_c(h.w2, mv0, h.w0, mv2),
           cf2 = -cross_c(h.w0, mv1, h.w1, mv0);
    const double vnr = np_norm3(h.v0, h.v1, h.v2) + DRAG_FORCE_RATIO;
    double df0 = (h.kc0 * h.v0) * vnr;
    double df1 = (h.kc1 * h.v1) * vnr;
    double df2 = (h.kc1 * h.v2) * vnr;
    const double mrt = SETTLED ? 0.0 : h.mr;
    double am0 = m * AMF0, am1 = m * AMF1, am2 = m * AMF2;
    double amr0 = mrt * AMRF, amr1 = mrt * AMRF, amr2 = mrt * AMRF;
    double af0 = -sm_mad(amr0, h.v0, sm_mad(am0, h.a0, cross_c(h.w1, h.amv2, h.w2, h.amv1)));
    double af1 = -sm_mad(amr1, h.v1, sm_mad(am1, h.a1, cross_c(h.w2, h.amv0, h.w0, h.amv2)));
    double af2 = -sm_mad(amr2, h.v2, sm_mad(am2, h.a2, cross_c(h.w0, h.amv1, h.w1, h.amv0)));
    const double cx = h.com, crx = SETTLED ? 0.0 : h.comr;
    double acc_y = (h.w0 * (h.w1 * cx) + (h.w2 * crx) * 2.0) + h.al2 * cx;
    double acc_z = (h.w0 * (h.w2 * cx) + -(h.w1 * crx) * 2.0) + -(h.al1 * cx);
    double acc_x = cross_c(h.w1, -(h.w1 * cx), h.w2, h.w2 * cx) + (SETTLED ? 0.0 : h.coma);
    const double rm = h.rm;
    const double na0 = sm_mad(acc_x, m, ((h.jf0 + df0) + af0) + cf0) * rm;
    const double na1 = sm_mad(acc_y, m, ((h.jf1 + df1) + af1) + cf1) * rm;
    const double na2 = sm_mad(acc_z, m, ((h.jf2 + df2) + af2) + cf2) * rm;
    h.a0 = na0; h.a1 = na1; h.a2 = na2;
    h.v0 = sm_mad(na0, DT, h.v0); h.v1 = sm_mad(na1, DT, h.v1); h.v2 = sm_mad(na2, DT, h.v2);
    h.q0 = sm_mad(h.v0, DT, h.q0); h.q1 = sm_mad(h.v1, DT, h.q1); h.q2 = sm_mad(h.v2, DT, h.q2);
    /* commit the tick's clock and properties */
    h.ct = g.ct;
    h.phase = g.phase;
    h.time += DT;
    h.pV = h.V;
    if (STEADY) {
        h.pv32 = false;
        if (SETTLED) return true;
        const auto zero = [&] {
            return (__double_as_longlong(h.comr) | __double_as_longlong(h.coma) | __double_as_longlong(h.mr) |
                    __double_as_longlong(h.speed)) == 0;
        };
        if (!__all(zero())) {
            const double cr = div_dt(h.com - h.com);
            h.coma = div_dt(cr - h.comr);
            h.comr = cr;
            const double pwm = r32(sel(h.pv32, P.density) * h.pV, h.pv32);
            h.mr = div_dt(water_mass(P, h.V, false) - pwm);
            h.speed = qdiv(div_dt(h.V - h.pV), rcp_of(P.nozzle_area));
        }
        return zero();
    }
    h.pv32 = h.g32;
    h.L = g.L; h.W = g.W; h.g32 = g.f;
    h.V = g.V; h.com = g.com; h.comr = g.comr; h.coma = g.coma;
    h.m = g.m; h.mr = g.mr; h.speed = g.speed; h.rm = g.rm;
    return false;
}
template <int MODE>
SD bool step_a(HotA& h, const Params& P, Cache32 c32, bool pend) {
    return step_a<MODE>(h, P, pre_a<MODE>(h, P, c32), pend);
}

/* Wave B's clock, phase and (full ticks) shape-side geometry of a tick. */
struct PreB {
    double ct, L, W;
    Geo ng;
    int phase;
    bool f;
};
template <int MODE>
SD PreB pre_b(const HotB& h, const Params& P, Cache32 c32) {
    constexpr bool STEADY = MODE != PM_FULL;
    double ct = h.ct;
    int phase = h.phase;
    pair_clock<STEADY>(ct, phase, h.b1, h.b2, h.mx);
    double L = h.L, W = h.W;
    bool f = h.g32;
    Geo ng;
    if (!STEADY) {
        body_lw(P, phase, ct, h.refill, h.mx, h.c, h.cr, h.rr, h.c32, &L, &W, &f);
        const Core c = core(L, W, false);
        geo_shape(P, c, L, W, false, ng);
        if (f) {
            ng.I0 = c32[C32_I0]; ng.I1 = c32[C32_I1];
            ng.kc0 = c32[C32_KC0]; ng.kc1 = c32[C32_KC1]; ng.ra0 = c32[C32_RA0]; ng.ra1 = c32[C32_RA1];
            ng.dimx = c32[C32_DIMX]; ng.dimy = c32[C32_DIMY];
        }
        ng.rI0 = rcr(ng.I0);
        ng.rI1 = rcr(ng.I1);
    }
    return PreB{ct, L, W, ng, phase, f};
}

/* Euler's equations with the tick-start values: the new angular velocity and
 * acceleration (all wave A needs before its next Newton step). */
template <int MODE>
SD void step_b1(HotB& h, const Params& P) {
    constexpr bool SETTLED = MODE == PM_SETTLED;
    const double I0 = h.I0, I1 = h.I1;
    double iw0 = I0 * h.w0, iw1 = I1 * h.w1, iw2 = I1 * h.w2;
    double ct0 = -cross_c(h.w1, iw2, h.w2, iw1), ct1 = -cross_c(h.w2, iw0, h.w0, iw2),
           ct2 = -cross_c(h.w0, iw1, h.w1, iw0);
    const double wn = np_norm3(h.w0, h.w1, h.w2), wr = h.W * DRAG_TORQUE_RATIO;
    const double sx = sm_fma(wn, h.dimx, wr), sy = sm_fma(wn, h.dimy, wr);
    double dt0 = (h.ra0 * h.w0) * sx;
    double dt1 = (h.ra1 * h.w1) * sy;
    double dt2 = (h.ra1 * h.w2) * sy;
    double ir0 = 0.0, ir1 = 0.0, ir2 = 0.0;
    if (!SETTLED) {
        ir0 = div_dt(I0 - h.pI0);
        ir1 = div_dt(I1 - h.pI1);
        const double ir2b = div_dt(I1 - h.pI2);
        ir2 = h.pI2 != h.pI1 ? ir2b : ir1;
        h.pI0 = I0; h.pI1 = I1; h.pI2 = I1;
    }
    double at0 = I0 * AMT0, at1 = I1 * AMT1, at2 = I1 * AMT2;
    double atw0 = at0 * h.w0, atw1 = at1 * h.w1, atw2 = at2 * h.w2;
    double amt0 = -(sm_mad(at0, h.al0, cross_c(h.w1, atw2, h.w2, atw1)) + h.X0);
    double amt1 = -(sm_mad(at1, h.al1, cross_c(h.w2, atw0, h.w0, atw2)) + h.X1);
    double amt2 = -(sm_mad(at2, h.al2, cross_c(h.w0, atw1, h.w1, atw0)) + h.X2);
    const double rI0 = h.rI0, rI1 = h.rI1;
    const double nal0 = (sm_mad(-ir0, h.w0, dt0 + ct0) + amt0) * rI0;
    const double nal1 = (sm_mad(-ir1, h.w1, (h.jt1 + dt1) + ct1) + amt1) * rI1;
    const double nal2 = (sm_mad(-ir2, h.w2, (h.jt2 + dt2) + ct2) + amt2) * rI1;
    h.al0 = nal0; h.al1 = nal1; h.al2 = nal2;
    h.w0 = sm_mad(nal0, DT, h.w0); h.w1 = sm_mad(nal1, DT, h.w1); h.w2 = sm_mad(nal2, DT, h.w2);
}
/* The rest of wave B's tick: Euler-angle and angle integration, the clock and
 * shape-side properties committed, roll / pitch / yaw sin/cos at the new
 * angles (the yaw's for wave A). */
template <int MODE>
SD void step_b2(HotB& h, const Params& P, const PreB& g) {
    constexpr bool STEADY = MODE != PM_FULL;
    {   /* tick()'s Euler-rate map */
        const double u = sm_fma(h.cp, h.w2, h.sp * h.w1);
        const double g2 = qdiv(u, rcp_of(h.cth));
        double r0 = sm_fma(h.st, g2, h.w0);
        double r1 = sm_fma(-h.sp, h.w2, h.cp * h.w1);
        double r2 = g2;
        h.e0 = sm_mad(r0, DT, h.e0); h.e1 = sm_mad(r1, DT, h.e1); h.e2 = sm_mad(r2, DT, h.e2);
    }
    h.g0 = sm_mad(h.w0, DT, h.g0); h.g1 = sm_mad(h.w1, DT, h.g1); h.g2 = sm_mad(h.w2, DT, h.g2);
    h.ct = g.ct;
    h.phase = g.phase;
    if (!STEADY) {
        h.L = g.L; h.W = g.W; h.g32 = g.f;
        h.I0 = g.ng.I0; h.I1 = g.ng.I1; h.rI0 = g.ng.rI0; h.rI1 = g.ng.rI1;
        h.kc0 = g.ng.kc0; h.kc1 = g.ng.kc1; h.ra0 = g.ng.ra0; h.ra1 = g.ng.ra1;
        h.dimx = g.ng.dimx; h.dimy = g.ng.dimy;
    }
    sm_sincos_rp2(h.e0, h.e1, &h.sp, &h.cp, &h.st, &h.cth, P.sk);
    sm_sincos_yaw_p(h.e2, &h.ss, &h.cs, P.sk);   /* yaw: wave A's world-frame update */
}
template <int MODE>
SD void step_b(HotB& h, const Params& P, const PreB& g) {
    step_b1<MODE>(h, P);
    step_b2<MODE>(h, P, g);
}
template <int MODE>
SD void step_b(HotB& h, const Params& P, Cache32 c32) {
    step_b<MODE>(h, P, pre_b<MODE>(h, P, c32));
}


/* ---------------------------------------- LDS slot <-> the two waves */
/* The spill slot (salp_device.h spill / unspill, non-RAND layout) is the
 * meeting point at env-step boundaries: each wave writes the fields it owns,
 * wave A runs the boundary on the whole Hot, each wave reads its fields back. */
enum {
    SP_V = 0, SP_W = 3, SP_A = 6, SP_AL = 9, SP_E = 12, SP_P = 15, SP_Q = 18, SP_G = 21, SP_L = 24, SP_WID = 25,
    SP_VOL = 26, SP_PV = 27, SP_COM = 28, SP_COMR = 29, SP_COMA = 30, SP_PI = 31, SP_CT = 34, SP_TIME = 35,
    SP_REFILL = 36, SP_JET = 37, SP_COAST = 38, SP_C = 39, SP_CR = 40, SP_RR = 41, SP_TURN = 42, SP_D = 43,
    SP_FLAGS = 46, SP_SP = 47, SP_CP = 48, SP_ST = 49, SP_CTH = 50, SP_M = 51, SP_MR = 52, SP_I0 = 53, SP_I1 = 54,
    SP_KC0 = 55, SP_KC1 = 56, SP_RA0 = 57, SP_RA1 = 58, SP_DIMX = 59, SP_DIMY = 60, SP_SPEED = 61, SP_RX = 62
};
static_assert(SPILL_N == 63, "pair slot layout follows spill<false>");

SD void spill_a(const HotA& h, SpillSlot s, const Params& P) {
    s[SP_V] = h.v0; s[SP_V + 1] = h.v1; s[SP_V + 2] = h.v2;
    s[SP_A] = h.a0; s[SP_A + 1] = h.a1; s[SP_A + 2] = h.a2;
    s[SP_P] = h.p0; s[SP_P + 1] = h.p1; s[SP_P + 2] = h.p2;
    s[SP_Q] = h.q0; s[SP_Q + 1] = h.q1; s[SP_Q + 2] = h.q2;
    s[SP_L] = h.L; s[SP_WID] = h.W; s[SP_VOL] = h.V; s[SP_PV] = h.pV;
    s[SP_COM] = h.com; s[SP_COMR] = h.comr; s[SP_COMA] = h.coma;
    s[SP_CT] = h.ct; s[SP_TIME] = h.time;
    s[SP_REFILL] = h.refill; s[SP_JET] = h.jet; s[SP_COAST] = h.coast; s[SP_C] = h.c; s[SP_CR] = h.cr;
    s[SP_RR] = h.rr; s[SP_TURN] = h.turn;
    s[SP_D] = h.d0; s[SP_D + 1] = h.d1; s[SP_D + 2] = h.d2;
    s[SP_FLAGS] = (double)(h.phase | (h.g32 ? 4 : 0) | (h.pv32 ? 8 : 0) | (h.c32 ? 16 : 0));
    s[SP_M] = h.m; s[SP_MR] = h.mr; s[SP_SPEED] = h.speed; s[SP_RX] = jet_arm(P, h.L);
}
SD void spill_b(const HotB& h, SpillSlot s) {
    s[SP_W] = h.w0; s[SP_W + 1] = h.w1; s[SP_W + 2] = h.w2;
    s[SP_AL] = h.al0; s[SP_AL + 1] = h.al1; s[SP_AL + 2] = h.al2;
    s[SP_E] = h.e0; s[SP_E + 1] = h.e1; s[SP_E + 2] = h.e2;
    s[SP_G] = h.g0; s[SP_G + 1] = h.g1; s[SP_G + 2] = h.g2;
    s[SP_PI] = h.pI0; s[SP_PI + 1] = h.pI1; s[SP_PI + 2] = h.pI2;
    s[SP_SP] = h.sp; s[SP_CP] = h.cp; s[SP_ST] = h.st; s[SP_CTH] = h.cth;
    s[SP_I0] = h.I0; s[SP_I1] = h.I1; s[SP_KC0] = h.kc0; s[SP_KC1] = h.kc1;
    s[SP_RA0] = h.ra0; s[SP_RA1] = h.ra1; s[SP_DIMX] = h.dimx; s[SP_DIMY] = h.dimy;
}
SD void cycle_bounds_of(double refill, double turn, double jet, double coast, double* mx, double* b1, double* b2) {
    *mx = pymax(refill, turn);
    *b1 = *mx + jet;
    *b2 = *b1 + coast;
}
SD void unspill_a(HotA& h, SpillSlot s) {
    h.v0 = s[SP_V]; h.v1 = s[SP_V + 1]; h.v2 = s[SP_V + 2];
    h.a0 = s[SP_A]; h.a1 = s[SP_A + 1]; h.a2 = s[SP_A + 2];
    h.p0 = s[SP_P]; h.p1 = s[SP_P + 1]; h.p2 = s[SP_P + 2];
    h.q0 = s[SP_Q]; h.q1 = s[SP_Q + 1]; h.q2 = s[SP_Q + 2];
    h.L = s[SP_L]; h.W = s[SP_WID]; h.V = s[SP_VOL]; h.pV = s[SP_PV];
    h.com = s[SP_COM]; h.comr = s[SP_COMR]; h.coma = s[SP_COMA];
    h.ct = s[SP_CT]; h.time = s[SP_TIME];
    h.refill = s[SP_REFILL]; h.jet = s[SP_JET]; h.coast = s[SP_COAST]; h.c = s[SP_C]; h.cr = s[SP_CR];
    h.rr = s[SP_RR]; h.turn = s[SP_TURN];
    h.d0 = s[SP_D]; h.d1 = s[SP_D + 1]; h.d2 = s[SP_D + 2];
    const int fl = (int)s[SP_FLAGS];
    h.phase = fl & 3; h.g32 = (fl & 4) != 0; h.pv32 = (fl & 8) != 0; h.c32 = (fl & 16) != 0;
    h.m = s[SP_M]; h.mr = s[SP_MR]; h.speed = s[SP_SPEED];
    h.rm = rcr(h.m);
    /* wave B's state, as its packet would carry it */
    h.w0 = s[SP_W]; h.w1 = s[SP_W + 1]; h.w2 = s[SP_W + 2];
    h.al1 = s[SP_AL + 1]; h.al2 = s[SP_AL + 2];
    h.sp = s[SP_SP]; h.cp = s[SP_CP]; h.st = s[SP_ST]; h.cth = s[SP_CTH];
    h.ss = 0.0; h.cs = 1.0;   /* the first packet brings the yaw's (no world update is owed yet) */
    h.kc0 = s[SP_KC0]; h.kc1 = s[SP_KC1];
    cycle_bounds_of(h.refill, h.turn, h.jet, h.coast, &h.mx, &h.b1, &h.b2);
}
/* Wave B's fields; X / jt of the first tick from wave A's fields of the slot,
 * by the same expressions as a_prepare. */
SD void unspill_b(HotB& h, SpillSlot s, const Params& P) {
    h.w0 = s[SP_W]; h.w1 = s[SP_W + 1]; h.w2 = s[SP_W + 2];
    h.al0 = s[SP_AL]; h.al1 = s[SP_AL + 1]; h.al2 = s[SP_AL + 2];
    h.e0 = s[SP_E]; h.e1 = s[SP_E + 1]; h.e2 = s[SP_E + 2];
    h.g0 = s[SP_G]; h.g1 = s[SP_G + 1]; h.g2 = s[SP_G + 2];
    h.pI0 = s[SP_PI]; h.pI1 = s[SP_PI + 1]; h.pI2 = s[SP_PI + 2];
    h.sp = s[SP_SP]; h.cp = s[SP_CP]; h.st = s[SP_ST]; h.cth = s[SP_CTH];
    sm_sincos_yaw_p(h.e2, &h.ss, &h.cs, P.sk);
    h.I0 = s[SP_I0]; h.I1 = s[SP_I1]; h.kc0 = s[SP_KC0]; h.kc1 = s[SP_KC1];
    h.ra0 = s[SP_RA0]; h.ra1 = s[SP_RA1]; h.dimx = s[SP_DIMX]; h.dimy = s[SP_DIMY];
    h.rI0 = rcr(h.I0);
    h.rI1 = rcr(h.I1);
    h.L = s[SP_L]; h.W = s[SP_WID]; h.ct = s[SP_CT];
    h.refill = s[SP_REFILL]; h.c = s[SP_C]; h.cr = s[SP_CR]; h.rr = s[SP_RR];
    const double jet = s[SP_JET], coast = s[SP_COAST], turn = s[SP_TURN];
    const int fl = (int)s[SP_FLAGS];
    h.phase = fl & 3; h.g32 = (fl & 4) != 0; h.c32 = (fl & 16) != 0;
    cycle_bounds_of(h.refill, turn, jet, coast, &h.mx, &h.b1, &h.b2);
    double amv[3], jf[3], X[3], jt[2];
    pair_terms(P, s[SP_V], s[SP_V + 1], s[SP_V + 2], s[SP_M], s[SP_MR], s[SP_SPEED], s[SP_D], s[SP_D + 1],
               s[SP_D + 2], h.phase, h.L, amv, jf, X, jt);
    h.X0 = X[0]; h.X1 = X[1]; h.X2 = X[2]; h.jt1 = jt[0]; h.jt2 = jt[1];
}

/* next_tick_steady (salp_device.h) of either wave's copy of the clock / body */
SD bool pair_next_steady(double ct, double L, double W, bool g32, double b1, double mx, const Params& P) {
    const double n = ct + DT;
    return ct > 0.0 && L == P.L0 && W == P.W0 && !g32 && n > b1 && n > mx;
}

}  // namespace salp

#endif /* SALP_PAIR_H */
