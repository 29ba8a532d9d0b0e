// salp_kernels.hip — HIP kernels for gfx950 + the C ABI of include/salp.h.
//
// One env per lane, struct-of-arrays fp64 state in HBM.  Every kernel loads a
// lane's hot state once, runs whole breathing cycles (hundreds of physics
// ticks) in registers, and stores once; the only HBM traffic inside a cycle
// is nothing at all.  See DESIGN.md for the data layout and roofline.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#include "salp_device.h"
#include "salp_pair.h"
#include "salp_tanh.h"

using salp::Hot;
using salp::Params;

#define SF(f) salp::sref(S, P, i, (f))

namespace {

constexpr int kBlock = 256;
// Longest legitimate cycle: max(refill 3.3 s, turn 3.9 s) + jet 0.5 s + coast
// 10 s < 1500 ticks.  The guard only bounds a lane fed a corrupted state.
constexpr int kMaxTicksPerCycle = 1 << 16;
// Lock-step launches of at least this many envs run in sorted order by default.
constexpr int64_t kSortMinEnvs = 1024;

static_assert(kBlock == salp::LANES, "LDS cache stride is the workgroup size");

// This lane's column of the workgroup's per-cycle float32 geometry cache.
#define LANE_CACHE32()                                              \
    __shared__ double s_cache32[salp::C32_N * salp::LANES];         \
    const salp::Cache32 c32{s_cache32 + threadIdx.x}

template <bool RAND>
__device__ __forceinline__ void run_cycle(Hot& h, const Params& P, salp::Cache32 c32) {
    const Params PV = salp::pin_params(P);
    // Full ticks until every lane still ticking has reached the steady body
    // (COAST / REST after one tick of it), then the rest of the cycle without
    // the geometry (salp_device.h next_tick_steady).  All lanes of a lock-step
    // wave start the cycle together, so they usually get there together: about
    // half of a sorted wave's ticks run the short body.  Lanes that finish
    // drop out of the vote.
    int g = 0;
    for (; h.ct < h.b2 && g < kMaxTicksPerCycle; ++g) {
        if (__all(salp::next_tick_steady(h, PV))) break;
        salp::tick<false, RAND>(h, PV, c32);
    }
    // steady ticks until the wave's lanes are settled (salp_device.h tick), then settled ones
    for (; h.ct < h.b2 && g < kMaxTicksPerCycle; ++g) {
        if (__all(salp::tick<false, RAND, false, true>(h, PV, c32))) {
            ++g;
            break;
        }
    }
    for (; h.ct < h.b2 && g < kMaxTicksPerCycle; ++g) salp::tick<false, RAND, false, true, true>(h, PV, c32);
}

// ---------------------------------------------------------------- one env per workgroup
// The per-env step path (SalpRobotEnv.step: one env, one launch per env-step)
// is a latency: one lane runs the ~700 ticks of a cycle back to back while the
// rest of the chip idles.  k_step_wave gives every env a workgroup of two waves
// and splits each tick along two one-way dependences of Robot.step:
// * the geometry (update_properties: body length / width, volume, centre of
//   mass, mass, inertia, drag coefficients, jet rates; src/robot.py:640-668,
//   1055-1066) depends on the cycle's constants and the clock only, never on
//   the motion: wave 0's 64 lanes compute the geometry after each of the next
//   64 ticks at once (lane j: tick j; the values that chain from one tick to
//   the next - previous volume, float32 flag, centre of mass and its rate -
//   come from lane j - 1 by a shuffle) into an LDS table;
// * the forces and the velocity integration (tick_dynamics' TD_FORCES) never read the Euler
//   angles or the world position: wave 0 runs them on the table's geometry and
//   hands each tick's new velocities to wave 1 through an LDS ring; wave 1 runs
//   the angle / world-frame chain (TD_KINEMATICS) behind it.
// Every value is the expression tick() computes, evaluated on the same operands:
// results are those of k_step bit for bit (tests/test_gpu_step_wave.py).  A tick
// then costs wave 0 its forces plus a 1/64 share of the geometry.
enum {
    WG_CT, WG_TIME, WG_PHASE, WG_W, WG_COM, WG_COMR, WG_COMA,
    WG_M, WG_MR, WG_I0, WG_I1, WG_KC0, WG_KC1, WG_RA0, WG_RA1, WG_DIMX, WG_DIMY, WG_SPEED, WG_RX,
    WG_RM, WG_RI0, WG_RI1,                       /* read by every tick (22) */
    WG_L, WG_V, WG_PV, WG_G32, WG_PV32,          /* read after the block's last tick */
    WG_STRIDE = 28                               /* doubles per row (16-B aligned rows) */
};
constexpr int kWave = 64;

// Row j of the table: the geometry state after tick j of the block that starts
// at the lane's (uniform) state h; tick()'s clocks / update_state /
// update_properties / rates, in the same order on the same operands.
__device__ __forceinline__ void wave_geometry_rows(const Hot& h, const Params& P, salp::Cache32 c32, double* rows) {
    using namespace salp;
    const int j = (int)(threadIdx.x & (kWave - 1));
    double ct = h.ct, tm = h.time, my_ct = 0.0, my_tm = 0.0;
    for (int k = 0; k < kWave; ++k) {   /* cycle_time / time after k + 1 ticks: the same sums */
        ct += DT;
        tm += DT;
        my_ct = k == j ? ct : my_ct;
        my_tm = k == j ? tm : my_tm;
    }
    int ph = my_ct <= h.b2 ? COAST : REST;
    ph = my_ct <= h.b1 ? JET : ph;
    ph = my_ct <= h.mx ? REFILL : ph;
    double L, W;
    bool f;
    body_lw(P, ph, my_ct, h.refill, h.mx, h.c, h.cr, h.rr, h.c32, &L, &W, &f);
    const Core c = core(L, W, false);
    double V = water_volume(P, c, false);
    double wm = water_mass(P, V, false);
    double com = center_of_mass(P, c, wm, false);
    Geo ng = make_geo_shape(P, c, L, W, wm, false);
    if (f) {
        V = c32[C32_V]; wm = c32[C32_WM]; com = c32[C32_COM];
        ng.m = c32[C32_M]; ng.I0 = c32[C32_I0]; ng.I1 = c32[C32_I1];
        ng.kc0 = c32[C32_KC0]; ng.kc1 = c32[C32_KC1]; ng.ra0 = c32[C32_RA0]; ng.ra1 = c32[C32_RA1];
        ng.dimx = c32[C32_DIMX]; ng.dimy = c32[C32_DIMY];
    }
    /* the previous tick's volume, float32 flag and centre of mass: lane j - 1 (lane 0: the block's start) */
    double pV = __shfl_up(V, 1), pcom = __shfl_up(com, 1);
    int pv32 = __shfl_up((int)f, 1);
    if (j == 0) {
        pV = h.V;
        pcom = h.com;
        pv32 = h.g32;
    }
    const double comr = div_dt(com - pcom);
    double pcomr = __shfl_up(comr, 1);
    if (j == 0) pcomr = h.comr;
    const double coma = div_dt(comr - pcomr);
    jet_rates(P, V, pV, wm, f, pv32 != 0, ng);
    geo_recips(ng);
    double* r = rows + j * WG_STRIDE;
    r[WG_CT] = my_ct; r[WG_TIME] = my_tm; r[WG_PHASE] = (double)ph; r[WG_W] = W;
    r[WG_COM] = com; r[WG_COMR] = comr; r[WG_COMA] = coma;
    r[WG_M] = ng.m; r[WG_MR] = ng.mr; r[WG_I0] = ng.I0; r[WG_I1] = ng.I1;
    r[WG_KC0] = ng.kc0; r[WG_KC1] = ng.kc1; r[WG_RA0] = ng.ra0; r[WG_RA1] = ng.ra1;
    r[WG_DIMX] = ng.dimx; r[WG_DIMY] = ng.dimy; r[WG_SPEED] = ng.speed; r[WG_RX] = ng.rx;
    r[WG_RM] = ng.rm; r[WG_RI0] = ng.rI0; r[WG_RI1] = ng.rI1;
    r[WG_L] = L; r[WG_V] = V; r[WG_PV] = pV; r[WG_G32] = f ? 1.0 : 0.0; r[WG_PV32] = pv32 ? 1.0 : 0.0;
}

// The loop of Robot.step_through_cycle with record=True (src/robot.py:
// 750-765): sample 0 before the first tick, one sample per tick after it.
template <bool RAND>
__device__ void run_cycle_recorded(Hot& h, const double* S, const Params& P, salp::Cache32 c32,
                                   const SalpTraceBuffer& T, int64_t i) {
    const int64_t n = P.n;
    if (T.max_samples > 0) salp::record_state(h, P, S, i, T.rows + i, n, true);
    int64_t t = 0;
    for (int g = 0; h.ct < h.b2 && g < kMaxTicksPerCycle; ++g) {
        ++t;
        if (t < T.max_samples) {
            double* rec = T.rows + (size_t)t * SALP_TRACE_DIM * (size_t)n + (size_t)i;
            salp::tick<true, RAND>(h, P, c32, rec, n);
            salp::record_state(h, P, S, i, rec, n, false);
        } else {
            salp::tick<false, RAND>(h, P, c32);
        }
    }
    T.n_samples[i] = t + 1;
}

__global__ __launch_bounds__(kBlock) void k_construct(double* S, Params P) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P.n) return;
    salp::construct_env(S, P, i);
}

__global__ __launch_bounds__(kBlock) void k_reset(double* S, Params P, const uint8_t* mask,
                                                  float* obs) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P.n || (mask && !mask[i])) return;
    Hot h;
    salp::load_hot(h, S, P, i);
    float o[SALP_OBS_DIM_MAX];
    salp::reset_env_philox(h, S, P, i, o);
    salp::store_hot(h, S, P, i);
    if (obs)
        for (int k = 0; k < P.obs_dim; ++k) obs[(size_t)i * P.obs_dim + k] = o[k];
}

__global__ __launch_bounds__(kBlock) void k_reset_to(double* S, Params P, const uint8_t* mask,
                                                     const float* tgt, const float* obst,
                                                     const int32_t* nob, float* obs) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P.n || (mask && !mask[i])) return;
    Hot h;
    salp::load_hot(h, S, P, i);
    float o[SALP_OBS_DIM_MAX];
    int n = nob[i];
    n = n < 0 ? 0 : (n > P.num_obstacles ? P.num_obstacles : n);
    salp::reset_env(h, S, P, i, tgt + 2 * i, obst + 2 * SALP_MAX_OBSTACLES * i, n, o);
    salp::store_hot(h, S, P, i);
    if (obs)
        for (int k = 0; k < P.obs_dim; ++k) obs[(size_t)i * P.obs_dim + k] = o[k];
}

// The lock-step kernels run an env-step's prologue and epilogue on a register
// copy of the env's cold fields (salp::ColdRegs: one round of 16-B loads from
// its cold block, one of stores), as the rollout's boundary does, instead of
// one scattered 8-B access per field use.  SALP_LOCKSTEP_COLDREGS=0 keeps the
// direct accesses (A/B builds).
#ifndef SALP_LOCKSTEP_COLDREGS
#define SALP_LOCKSTEP_COLDREGS 1
#endif

// SalpRobotEnv.step for every env (one breathing cycle each).
template <bool REC, bool RAND>
__global__ __launch_bounds__(kBlock) void k_step(double* S, Params P, const float* actions,
                                                 float* obs_out, double* reward_out,
                                                 uint8_t* term_out, uint8_t* trunc_out,
                                                 int auto_reset, float* term_obs_out,
                                                 double* info_out, SalpTraceBuffer T, const int32_t* order) {
    const int64_t lane = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (lane >= P.n) return;
    const int64_t i = order ? (int64_t)order[lane] : lane;   // launch order (salp_sort.hip)
    LANE_CACHE32();
    Hot h;
    salp::load_hot<RAND>(h, S, P, i);
    float o[SALP_OBS_DIM_MAX];
    salp::StepOut r;
    double* info = info_out ? info_out + (size_t)SALP_INFO_DIM * i : nullptr;
    if (SALP_LOCKSTEP_COLDREGS) {
        salp::ColdRegs<RAND> C;
        salp::load_cold<RAND>(C, S, P, i);
        salp::begin_step<RAND>(h, &C, P, i, actions[3 * i], actions[3 * i + 1], actions[3 * i + 2], c32);
        salp::store_cold<RAND>(C, S, P, i);
    } else {
        salp::begin_step<RAND>(h, S, P, i, actions[3 * i], actions[3 * i + 1], actions[3 * i + 2], c32);
    }
    if (REC) run_cycle_recorded<RAND>(h, S, P, c32, T, i);
    else run_cycle<RAND>(h, P, c32);
    if (SALP_LOCKSTEP_COLDREGS) {
        salp::ColdRegs<RAND> C;
        salp::load_cold<RAND>(C, S, P, i);
        double& sc = salp::sref(&C, P, i, SALP_F_STEP_COUNT);
        sc = sc + 1.0;
        r = salp::finish_step<RAND>(h, &C, P, i, o, info);
        if (term_obs_out)
            for (int k = 0; k < P.obs_dim; ++k) term_obs_out[(size_t)i * P.obs_dim + k] = o[k];
        if (auto_reset && (r.terminated || r.truncated)) salp::reset_env_philox(h, &C, P, i, o);
        salp::store_cold<RAND>(C, S, P, i);
    } else {
        SF(SALP_F_STEP_COUNT) = SF(SALP_F_STEP_COUNT) + 1.0;
        r = salp::finish_step<RAND>(h, S, P, i, o, info);
        if (term_obs_out)
            for (int k = 0; k < P.obs_dim; ++k) term_obs_out[(size_t)i * P.obs_dim + k] = o[k];
        if (auto_reset && (r.terminated || r.truncated)) salp::reset_env_philox(h, S, P, i, o);
    }
    if (reward_out) reward_out[i] = r.reward;
    if (term_out) term_out[i] = r.terminated;
    if (trunc_out) trunc_out[i] = r.truncated;
    if (obs_out)
        for (int k = 0; k < P.obs_dim; ++k) obs_out[(size_t)i * P.obs_dim + k] = o[k];
    salp::store_hot<RAND>(h, S, P, i);
}

// Lock-step random-action env steps (every env does exactly n_steps).
template <bool RAND>
__global__ __launch_bounds__(kBlock) void k_step_random(double* S, Params P, int32_t n_steps,
                                                        double* reward_sum, const int32_t* order) {
    const int64_t lane = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (lane >= P.n) return;
    const int64_t i = order ? (int64_t)order[lane] : lane;   // launch order (salp_sort.hip)
    LANE_CACHE32();
    Hot h;
    salp::load_hot<RAND>(h, S, P, i);
    const uint64_t env_id = (uint64_t)(P.env_offset + i);
    double rs = 0.0;
    if (SALP_LOCKSTEP_COLDREGS) {
        // prologue of step k and epilogue of step k - 1 share one cold round
        salp::ColdRegs<RAND> C;
        if (n_steps > 0) {
            salp::load_cold<RAND>(C, S, P, i);
            float a[3];
            sp_action(P.seed, env_id, (uint64_t)salp::sref(&C, P, i, SALP_F_STEP_COUNT), a);
            salp::begin_step<RAND>(h, &C, P, i, a[0], a[1], a[2], c32);
            salp::store_cold<RAND>(C, S, P, i);
        }
        for (int32_t k = 0; k < n_steps; ++k) {
            run_cycle<RAND>(h, P, c32);
            salp::load_cold<RAND>(C, S, P, i);
            double& sc = salp::sref(&C, P, i, SALP_F_STEP_COUNT);
            sc = sc + 1.0;
            float o[SALP_OBS_DIM_MAX];
            salp::StepOut r = salp::finish_step<RAND>(h, &C, P, i, o, nullptr);
            rs += r.reward;
            if (r.terminated || r.truncated) salp::reset_env_philox(h, &C, P, i, o);
            if (k + 1 < n_steps) {
                float a[3];
                sp_action(P.seed, env_id, (uint64_t)sc, a);
                salp::begin_step<RAND>(h, &C, P, i, a[0], a[1], a[2], c32);
            }
            salp::store_cold<RAND>(C, S, P, i);
        }
    } else {
        for (int32_t k = 0; k < n_steps; ++k) {
            float a[3];
            sp_action(P.seed, env_id, (uint64_t)SF(SALP_F_STEP_COUNT), a);
            salp::begin_step<RAND>(h, S, P, i, a[0], a[1], a[2], c32);
            run_cycle<RAND>(h, P, c32);
            SF(SALP_F_STEP_COUNT) = SF(SALP_F_STEP_COUNT) + 1.0;
            float o[SALP_OBS_DIM_MAX];
            salp::StepOut r = salp::finish_step<RAND>(h, S, P, i, o, nullptr);
            rs += r.reward;
            if (r.terminated || r.truncated) salp::reset_env_philox(h, S, P, i, o);
        }
    }
    if (reward_sum) reward_sum[i] = rs;
    salp::store_hot<RAND>(h, S, P, i);
}

// Sort keys of the lock-step launch order: the predicted ticks of the env's
// next env-step (the given actions) or next n_steps random env-steps.
__global__ __launch_bounds__(kBlock) void k_predict_ticks(const double* S, Params P, const float* actions,
                                                          int32_t n_steps, uint32_t* keys, int32_t* ids) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P.n) return;
    double a1 = SF(SALP_F_ANGLE1), a2 = SF(SALP_F_ANGLE2);
    int64_t t = 0;
    if (actions) {
        t = salp::predict_cycle_ticks(P, actions[3 * i], actions[3 * i + 1], actions[3 * i + 2], &a1, &a2);
    } else {
        const uint64_t env_id = (uint64_t)(P.env_offset + i), sc = (uint64_t)SF(SALP_F_STEP_COUNT);
        for (int32_t k = 0; k < n_steps; ++k) {
            float a[3];
            sp_action(P.seed, env_id, sc + (uint64_t)k, a);
            t += salp::predict_cycle_ticks(P, a[0], a[1], a[2], &a1, &a2);
        }
    }
    keys[i] = (uint32_t)(t > 65535 ? 65535 : t);
    ids[i] = (int32_t)i;
}

// Chained random-action rollout, filling the rollout buffer.  Work proceeds in
// chunks of `chunk` physics ticks: inside a chunk every lane whose cycle is
// still running ticks (a tight loop over salp::tick only); between chunks the
// lanes whose cycle ended finish that env-step and start the next one
// together, so the heavy env-step epilogue runs once per chunk for all lanes
// that need it instead of once per lane.  A lane idles at most `chunk` ticks
// per env-step.  Per-env results depend only on (seed, env id): how the work
// is cut into launches and chunks changes nothing but the count of env-steps
// a launch completes.
// Policy-in-the-loop collection (salp_collect, include/salp.h): the SB3
// MlpPolicy evaluated per lane at env-step boundaries.  Weights are uniform
// over the launch, so their loads are scalar loads; the first hidden layer
// stays in registers and the second is folded into the heads as it is
// produced (no second activation array).  float32 like the torch policy.
constexpr int kPH = SALP_POLICY_HIDDEN, kPIN = SALP_OBS_DIM_MAX;
// The weights are read through the constant address space: the kernel writes
// global memory through other pointers, so a generic pointer's uniform loads
// would be vector loads (one latency-bound load round per hidden unit); from
// address space 4 they are scalar loads into SGPR operands (collect 18.8 ->
// 26.7 M env-steps/s at 65 536 envs, profiles/r2_experiments.md r2u).
typedef const __attribute__((address_space(4))) float* PolicyW;

// Packed fp32 (v_pk_fma_f32: two IEEE fmas per instruction, the weight pair
// an SGPR pair).  First layer: two hidden units per instruction, the input
// broadcast by op_sel.  Second layer: one row at a time, its even and odd
// inputs summed in the two halves, so that the row's 64 weights arrive as 32
// aligned SGPR pairs of one scalar-load burst (profiles/r4_experiments.md r4kp;
// float32 sums in another order than torch's, held to the torch policy by the
// collection tests).
typedef float PolicyF2 __attribute__((ext_vector_type(2)));
static_assert(kPH % 2 == 0, "hidden units go in pairs");

// tanh of the policy's hidden units: salp_tanh.h (shared with the PPO update).
__device__ __forceinline__ float policy_tanh(float x) { return salp_tanhf(x); }

__device__ __forceinline__ void policy_layer1(PolicyW w, int w1, int b1, const float* x, float* h1) {
#pragma unroll
    for (int j = 0; j < kPH; j += 2) {
        PolicyF2 acc = {w[b1 + j], w[b1 + j + 1]};
#pragma unroll
        for (int k = 0; k < kPIN; ++k) {
            const PolicyF2 wk = {w[w1 + j * kPIN + k], w[w1 + (j + 1) * kPIN + k]};
            const PolicyF2 xk = {x[k], x[k]};
            acc = __builtin_elementwise_fma(wk, xk, acc);
        }
        h1[j] = policy_tanh(acc.x);
        h1[j + 1] = policy_tanh(acc.y);
    }
}

template <int NOUT>
__device__ __forceinline__ void policy_mlp(PolicyW w, int w1, int b1, int w2, int b2, int hw,
                                           int hb, const float* x, float* out) {
    float h1[kPH];
    policy_layer1(w, w1, b1, x, h1);
#pragma unroll
    for (int c = 0; c < NOUT; ++c) out[c] = 0.0f;
#pragma unroll 1
    for (int j = 0; j < kPH; ++j) {
        // one row: even and odd inputs in the two halves of a packed sum
        PolicyF2 acc = {w[b2 + j], 0.0f};
#pragma unroll
        for (int k = 0; k < kPH; k += 2) {
            const PolicyF2 wk = {w[w2 + j * kPH + k], w[w2 + j * kPH + k + 1]};
            const PolicyF2 hk = {h1[k], h1[k + 1]};
            acc = __builtin_elementwise_fma(wk, hk, acc);
        }
        const float t = policy_tanh(acc.x + acc.y);
#pragma unroll
        for (int c = 0; c < NOUT; ++c) out[c] = fmaf(w[hw + c * kPH + j], t, out[c]);
    }
#pragma unroll
    for (int c = 0; c < NOUT; ++c) out[c] += w[hb + c];
}

// The actor's second layer and heads read from a copy in LDS (k_rollout_pair
// stages it once per workgroup): a row's 64 weights arrive as 16 broadcast
// 16-B LDS reads, in order, instead of scalar loads whose out-of-order return
// makes every row wait for its whole burst from L2.  The same operations in the
// same order as policy_mlp: bit-identical.
constexpr int kPolL2 = kPH * kPH + kPH + 3 * kPH;   // W2 [64][64], B2 [64], action head [3][64]
static_assert(SALP_POLICY_PI_B2 == SALP_POLICY_PI_W2 + kPH * kPH && SALP_POLICY_ACT_W == SALP_POLICY_PI_B2 + kPH,
              "the staged actor tensors are contiguous in the packed policy");
__device__ __forceinline__ void policy_actor_l2(PolicyW w, const float* l2, const float* x, float* out) {
    float h1[kPH];
    policy_layer1(w, SALP_POLICY_PI_W1, SALP_POLICY_PI_B1, x, h1);
    out[0] = out[1] = out[2] = 0.0f;
#pragma unroll 1
    for (int j = 0; j < kPH; ++j) {
        const float* row = l2 + j * kPH;
        PolicyF2 acc = {l2[kPH * kPH + j], 0.0f};
#pragma unroll
        for (int k = 0; k < kPH; k += 4) {
            const float4 v = *reinterpret_cast<const float4*>(row + k);
            acc = __builtin_elementwise_fma(PolicyF2{v.x, v.y}, PolicyF2{h1[k], h1[k + 1]}, acc);
            acc = __builtin_elementwise_fma(PolicyF2{v.z, v.w}, PolicyF2{h1[k + 2], h1[k + 3]}, acc);
        }
        const float t = policy_tanh(acc.x + acc.y);
#pragma unroll
        for (int c = 0; c < 3; ++c) out[c] = fmaf(l2[kPH * kPH + kPH + c * kPH + j], t, out[c]);
    }
#pragma unroll
    for (int c = 0; c < 3; ++c) out[c] += w[SALP_POLICY_ACT_B + c];
}

__device__ __forceinline__ void policy_input(const float* o, int obs_dim, float* x) {
#pragma unroll
    for (int k = 0; k < kPIN; ++k) x[k] = k < obs_dim ? o[k] : 0.0f;
}

__device__ __forceinline__ float policy_value(PolicyW w, const float* x) {
    float v;
    policy_mlp<1>(w, SALP_POLICY_VF_W1, SALP_POLICY_VF_B1, SALP_POLICY_VF_W2, SALP_POLICY_VF_B2, SALP_POLICY_VAL_W,
                  SALP_POLICY_VAL_B, x, &v);
    return v;
}

// Three standard normals (Box-Muller on one Philox draw) for the exploration
// noise of env `env_id` at its env-step `step`.
#define SP_STREAM_POLICY 7u
__device__ __forceinline__ void policy_noise(uint64_t seed, uint64_t env_id, uint64_t step, float z[3]) {
    const sp_u32x4 r = sp_draw(seed, env_id, step, SP_STREAM_POLICY, 0);
    const double u1 = ((double)r.v[0] + 1.0) * 0x1.0p-32, u3 = ((double)r.v[2] + 1.0) * 0x1.0p-32;
    const double rad1 = sqrt(-2.0 * sm_log(u1)), rad2 = sqrt(-2.0 * sm_log(u3));
    double s1, c1, s2, c2;
    sm_sincos(6.283185307179586 * sp_u01_32(r.v[1]), &s1, &c1);
    sm_sincos(6.283185307179586 * sp_u01_32(r.v[3]), &s2, &c2);
    z[0] = (float)(rad1 * c1);
    z[1] = (float)(rad1 * s1);
    z[2] = (float)(rad2 * c2);
}

// The env's action for observation o: a = mean + std z (unclipped, as SB3's
// buffer holds it), V(o) and log N(a; mean, std) summed over the dims, in the
// expression order of torch.distributions.Normal.log_prob.
// value == nullptr: the value network is evaluated elsewhere (k_rollout_pair's B wave).
// l2: the actor's second layer staged in LDS (policy_actor_l2), or nullptr.
template <bool L2 = false>
__device__ __forceinline__ void policy_act(const SalpPolicyRollout& R, int obs_dim, const float* o, uint64_t env_id,
                                           uint64_t step, float a[3], float* value, float* logp,
                                           const float* l2 = nullptr) {
    const PolicyW w = (PolicyW)R.weights;
    float x[kPIN];
    policy_input(o, obs_dim, x);
    float mean[3];
    if (L2)
        policy_actor_l2(w, l2, x, mean);
    else
        policy_mlp<3>(w, SALP_POLICY_PI_W1, SALP_POLICY_PI_B1, SALP_POLICY_PI_W2, SALP_POLICY_PI_B2,
                      SALP_POLICY_ACT_W, SALP_POLICY_ACT_B, x, mean);
    if (value) *value = policy_value(w, x);
    float z[3];
    policy_noise(R.noise_seed, env_id, step, z);
    float lp = 0.0f;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        const float ls = w[SALP_POLICY_LOG_STD + c], sd = expf(ls);
        a[c] = mean[c] + sd * z[c];
        const float d = a[c] - mean[c];
        lp += -(d * d) / (2.0f * (sd * sd)) - logf(sd) - 0.91893853320467274f;
    }
    *logp = lp;
}

// Where a salp_collect boundary's value-network evaluations run: in place
// (k_rollout), or handed to the B wave of k_rollout_pair through LDS
// (ValuesToPartner, defined with that kernel) while the A wave evaluates the
// policy mean and starts the next env-step.
struct ValuesInPlace {
    static constexpr bool kDefer = false;
    static constexpr bool kL2 = false;
    __device__ __forceinline__ const float* l2() const { return nullptr; }
    __device__ __forceinline__ void start_rep() {}
    __device__ __forceinline__ void boot(const float*, int, float, int64_t) {}
    __device__ __forceinline__ void value(const float*, int, int64_t) {}
    __device__ __forceinline__ void publish() {}
};

// salp_collect: a further round of env-step boundaries within one chunk
// boundary runs only when at least this many lanes of the wave need it.  A
// clipped action of 0 for the contraction and the coast time gives a cycle of
// zero ticks, so under a fresh policy (mean ~0, std 1: half of each action
// component clipped) many boundaries would otherwise run the whole wave's
// policy evaluation again and again for a few lanes; those lanes now wait for
// the next chunk boundary (per-env results unchanged).  PPO leg 15.6 -> 16.1 M
// env-steps/s with 4 (1 / 4 / 8 / 16 / 64 measured; profiles/r4_experiments.md
// r4rep).
#ifndef SALP_COLLECT_REP_MIN
#define SALP_COLLECT_REP_MIN 4
#endif

// torch.clamp(a, low, high): NaN stays NaN
__device__ __forceinline__ float clamp_box(float a, float lo, float hi) { return a < lo ? lo : (a > hi ? hi : a); }

// Chained random-action rollout, filling the rollout buffer.  Work proceeds in
// chunks of `chunk` physics ticks: inside a chunk every lane whose cycle is
// still running ticks (a tight loop over salp::tick only); between chunks the
// lanes whose cycle ended finish that env-step and start the next one
// together, so the heavy env-step epilogue runs once per chunk for all lanes
// that need it instead of once per lane.  A lane idles at most `chunk` ticks
// per env-step.  Per-env results depend only on (seed, env id): how the work
// is cut into launches and chunks changes nothing but the count of env-steps
// a launch completes.  POL: the actions come from the policy of salp_collect
// and the outputs go to its buffers (R).
template <bool RAND, bool POL, class ST, class VS = ValuesInPlace>
__device__ __forceinline__ void rollout_boundary(Hot& h, ST S, const Params& P, int64_t i,
                                                 uint64_t env_id, bool& pending, bool& active,
                                                 int64_t& steps, int64_t max_steps,
                                                 const SalpRolloutBuffers& B, double* reward_sum,
                                                 const SalpPolicyRollout& R, salp::Cache32 c32, VS vs = VS()) {
    // o: the env's current observation once this boundary has produced one
    // (after a finished step, or the reset obs after an episode end)
    float o[SALP_OBS_DIM_MAX];
    bool have_o = false;
    float ep_start = 0.0f;   // POL: episode_start of the env's next step, once a step finished here
    // a few rounds so that zero-tick cycles chain without waiting a chunk
    for (int rep = 0; rep < 4; ++rep) {
        const bool fin = active && pending && !(h.ct < h.b2);
        vs.start_rep();
        if (fin) {
            SF(SALP_F_STEP_COUNT) = SF(SALP_F_STEP_COUNT) + 1.0;
            salp::StepOut r = salp::finish_step<RAND>(h, S, P, i, o, nullptr);
            bool reset = r.terminated || r.truncated;
            if (POL) {
                // SB3 collect_rollouts + the learner's divergence guard (ppo.py):
                // o is the terminal observation here, before any reset
                const size_t row = (size_t)steps * (size_t)P.n + (size_t)i;
                float rew = (float)r.reward;
                bool bad = false;
                if (R.diverged_obs_abs > 0.0) {
                    bad = !(fabs(r.reward) <= R.diverged_reward_abs);   // NaN too
                    for (int k = 0; k < P.obs_dim; ++k) bad = bad || !(fabsf(o[k]) <= (float)R.diverged_obs_abs);
                }
                if (bad) {
                    rew = 0.0f;
                    atomicAdd((unsigned long long*)R.diverged, 1ull);
                } else if (r.truncated && !r.terminated) {
                    if (VS::kDefer) {
                        vs.boot(o, P.obs_dim, rew, (int64_t)steps);   // the partner writes rewards[row]
                    } else {
                        float x[kPIN];
                        policy_input(o, P.obs_dim, x);
                        rew = rew + (float)R.gamma * policy_value((PolicyW)R.weights, x);
                    }
                }
                if (reset && !bad) {
                    atomicAdd(&R.ep_stats[0], SF(SALP_F_EP_RETURN));
                    atomicAdd(&R.ep_stats[1], 1.0);
                    if (r.terminated) atomicAdd(&R.ep_stats[2], 1.0);   // the target was reached
                    atomicAdd(&R.ep_stats[3], SF(SALP_F_EP_LEN));
                }
                if (!(VS::kDefer && !bad && r.truncated && !r.terminated)) R.rewards[row] = rew;
                reset = reset || bad;
                ep_start = reset ? 1.0f : 0.0f;
                R.episode_start[i] = ep_start;
            } else if (B.capacity > 0) {
                const size_t slot = (size_t)(steps % B.capacity);
                const size_t row = slot * (size_t)P.n + (size_t)i;
                if (B.obs)
                    for (int k = 0; k < P.obs_dim; ++k) B.obs[row * P.obs_dim + k] = o[k];
                if (B.actions) {
                    B.actions[row * 3 + 0] = (float)SF(SALP_F_ACT0);
                    B.actions[row * 3 + 1] = (float)SF(SALP_F_ACT1);
                    B.actions[row * 3 + 2] = (float)SF(SALP_F_ACT2);
                }
                if (B.rewards) B.rewards[row] = (float)r.reward;
                if (B.dones) B.dones[row] = (uint8_t)((r.terminated ? 1 : 0) | (r.truncated ? 2 : 0));
            }
            if (reward_sum) reward_sum[i] += r.reward;
            ++steps;
            pending = false;
            if (reset) salp::reset_env_philox(h, S, P, i, (POL || B.obs_before) ? o : nullptr);
            have_o = true;
            if (max_steps > 0 && steps >= max_steps) {
                active = false;
                if (POL)
                    for (int k = 0; k < P.obs_dim; ++k) R.last_obs[(size_t)i * P.obs_dim + k] = o[k];
            }
        }
        const bool beg = active && !pending;
        if (beg) {   // the observation the next action is taken on
            if (POL && !have_o) {
                // first step of a salp_collect call: the observation the caller
                // holds (last_obs is in/out: the previous call's last one, or the
                // reset observation; with observation noise on, the noisy one the
                // previous bootstrap value was computed from)
                for (int k = 0; k < P.obs_dim; ++k) o[k] = R.last_obs[(size_t)i * P.obs_dim + k];
                have_o = true;
            } else if (B.obs_before && !have_o) {
                // first step after create / reset / set_state / a previous call:
                // the env's observation as reset() returns it (noise-free)
                const salp::Rot Rt = salp::rot_zyx(h.e0, h.e1, h.e2);
                salp::observation(h, Rt, S, P, i, o);
                have_o = true;
            }
            if (POL && VS::kDefer) vs.value(o, P.obs_dim, (int64_t)steps);
        }
        vs.publish();
        if (beg) {
            float a[3];
            if (POL) {
                if (!fin) ep_start = R.episode_start[i];
                float raw[3], v, lp;
                policy_act<VS::kL2>(R, P.obs_dim, o, env_id, (uint64_t)SF(SALP_F_STEP_COUNT), raw,
                                    VS::kDefer ? nullptr : &v, &lp, vs.l2());
                const size_t row = (size_t)steps * (size_t)P.n + (size_t)i;
                for (int k = 0; k < P.obs_dim; ++k) R.obs[row * P.obs_dim + k] = o[k];
                R.actions[row * 3 + 0] = raw[0];
                R.actions[row * 3 + 1] = raw[1];
                R.actions[row * 3 + 2] = raw[2];
                if (!VS::kDefer) R.values[row] = v;
                R.log_probs[row] = lp;
                R.episode_starts[row] = ep_start;
                a[0] = clamp_box(raw[0], 0.0f, 1.0f);
                a[1] = clamp_box(raw[1], 0.0f, 1.0f);
                a[2] = clamp_box(raw[2], -1.0f, 1.0f);
            } else {
                if (B.obs_before && B.capacity > 0) {
                    const size_t row = (size_t)(steps % B.capacity) * (size_t)P.n + (size_t)i;
                    for (int k = 0; k < P.obs_dim; ++k) B.obs_before[row * P.obs_dim + k] = o[k];
                }
                sp_action(P.seed, env_id, (uint64_t)SF(SALP_F_STEP_COUNT), a);
            }
            salp::begin_step<RAND>(h, S, P, i, a[0], a[1], a[2], c32);
            pending = true;
        }
        if (POL && SALP_COLLECT_REP_MIN > 1) {
            // another round evaluates the policy for the whole wave again: run it
            // only for enough lanes whose new cycle already ended (zero-tick
            // cycles); the others finish that step at the next chunk boundary
            const bool again = active && pending && !(h.ct < h.b2);
            if (__popcll(__ballot(again)) < SALP_COLLECT_REP_MIN) break;
        }
        if (VS::kDefer) {   // the partner follows rep by rep: the wave leaves together
            if (!__any(fin || beg)) break;
        } else if (!fin && !beg) {
            break;
        }
    }
}

// All launch arguments in one struct: the env-step epilogue re-reads them from
// the kernarg segment (scalar loads) where it runs, so that nothing it needs
// is held in SGPRs across the tick loop — which then compiles exactly like a
// standalone tick loop (its fp64 constants pinned in VGPRs, pin_params).
struct RolloutArgs {
    double* S;
    Params P;
    int64_t n_chunks;
    int32_t chunk;
    int32_t steady_q8;   // steady ticks a wave runs per full tick of its chunk budget, x256
    int64_t max_steps;
    SalpRolloutBuffers B;
    double* reward_sum;  // += each finished env-step's reward (salp_step_random), or null
    int32_t fresh;       // 1: every env starts a new env-step (drops an in-flight cycle), as
                         // the lock-step kernels do; 0: an in-flight cycle resumes
    int32_t pad_;
    SalpPolicyRollout R;  // POL kernels (salp_collect)
};
static_assert(sizeof(RolloutArgs) % 8 == 0, "RolloutArgs is copied as 8-byte words");
typedef const __attribute__((address_space(4))) uint64_t* KernargWords;
__device__ __forceinline__ RolloutArgs fresh_args() {
    KernargWords p = (KernargWords)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(p));   // opaque: the loads below stay where they are used
    uint64_t w[sizeof(RolloutArgs) / 8];
    for (size_t k = 0; k < sizeof(RolloutArgs) / 8; ++k) w[k] = p[k];
    RolloutArgs a;
    __builtin_memcpy(&a, w, sizeof a);
    return a;
}

// Env-step boundaries park the whole wave's tick state in LDS (SpillSlot),
// not in HBM: the lanes that need a boundary load their cold fields into
// registers in one round of loads, run the epilogue/prologue there, store them
// back, and everyone reloads its tick state from LDS.  HBM sees each env's
// state once per launch plus the cold rows of the env-steps that end.
//
// Re-seating (SALP_ROLLOUT_RESEAT, the default): the workgroup's 256 envs live
// in 256 LDS slots, and at every chunk boundary each lane reloads the slot the
// workgroup hands it instead of its own.  Envs whose body still changes (REFILL,
// JET, the first COAST tick: salp::next_tick_steady false) go to the first
// lanes, the steady ones (COAST / REST, 70 % of the ticks) after them, so most
// waves hold only steady envs and run their chunk on tick<STEADY>, which keeps
// the geometry (43 % of a tick).  A wave runs full ticks while any of its
// ticking lanes is unsteady, then steady ticks for the rest of its budget
// (steady_q8 / 256 steady ticks per full tick left), so that the four waves
// of a workgroup reach the next boundary at about the same time.  Per-env
// results do not depend on the lane or the chunk an env runs in.
#ifndef SALP_ROLLOUT_RESEAT
#define SALP_ROLLOUT_RESEAT 1
#endif

// Position of the k-th set bit of the kBlock-bit mask m[0..kBlock/64-1] (k < popcount).
__device__ __forceinline__ int nth_set_lane(const uint64_t* m, int k) {
    constexpr int NW = kBlock / 64;
    int base = 0;
    uint64_t w = m[NW - 1];
#pragma unroll
    for (int j = 0; j < NW - 1; ++j) {
        const int c = __popcll(m[j]);
        if (k < c) {
            w = m[j];
            base = 64 * j;
            break;
        }
        k -= c;
        base = 64 * (j + 1);
    }
    int pos = 0;
#pragma unroll
    for (int half = 32; half > 0; half >>= 1) {
        const uint64_t lo = w & ((1ull << half) - 1ull);
        const int c = __popcll(lo);
        if (k >= c) {
            k -= c;
            w >>= half;
            pos += half;
        } else {
            w = lo;
        }
    }
    return base + pos;
}

// Does this env's next tick need the geometry (it ticks and its body is not
// yet the steady one)?
__device__ __forceinline__ bool unsteady(const Hot& h, const Params& P, bool active) {
    return active && h.ct < h.b2 && !salp::next_tick_steady(h, P);
}

// The env-step boundary of one lane of k_rollout (cold fields into registers,
// the whole Hot from its LDS slot, rollout_boundary, back).  The randomised
// kernels run it as a separate (non-inlined) function: inlined into
// k_rollout<true, true> (salp_collect with randomisation), the compiler's
// register allocation of round 5's build stored two LDS addresses in place of
// the discharge coefficient's slot (tests/test_gpu_collect.py, rand case;
// tools/debug_collect_rand.py); the call keeps the boundary's registers apart
// from the tick loop's.  The plain kernels keep it inline (the bench path).
template <bool RAND, bool POL>
__device__ __forceinline__ bool lane_boundary(const RolloutArgs& a, salp::SpillSlot sp, int64_t i, bool& pending,
                                              bool& active, int64_t& steps, double* c32p) {
    const uint64_t env_id = (uint64_t)(a.P.env_offset + i);
    salp::ColdRegs<RAND> C;
    salp::load_cold<RAND>(C, a.S, a.P, i);
    Hot hb;
    salp::unspill<RAND>(hb, sp, a.P, env_id);
    rollout_boundary<RAND, POL>(hb, &C, a.P, i, env_id, pending, active, steps, a.max_steps, a.B,
                                a.reward_sum, a.R, salp::Cache32{c32p});
    salp::store_cold<RAND>(C, a.S, a.P, i);
    salp::spill<RAND>(hb, sp);
    return unsteady(hb, a.P, active);
}
template <bool RAND, bool POL>
__device__ __noinline__ bool lane_boundary_call(const RolloutArgs* a, double* spp, int64_t i, bool* pending,
                                                bool* active, int64_t* steps, double* c32p) {
    return lane_boundary<RAND, POL>(*a, salp::SpillSlot{spp}, i, *pending, *active, *steps, c32p);
}

// SALP_ROLLOUT_PROF=1 (experiment builds only, tools/rollout_phase_prof.py):
// per wave, s_memtime cycles and loop iterations of each part of k_rollout's
// chunk loop, summed over the launch's waves into g_roll_prof (read back by
// salp_debug_rollout_prof): boundary + re-seat, full ticks, steady ticks,
// settled ticks.
#ifndef SALP_ROLLOUT_PROF
#define SALP_ROLLOUT_PROF 0
#endif
enum { RP_BOUNDARY, RP_FULL, RP_STEADY, RP_SETTLED, RP_BARRIER, RP_RESEAT, RP_N };
__device__ unsigned long long g_roll_prof[2][RP_N];   // [cycles | iterations][part]
struct RollProf {
    unsigned long long cyc[RP_N] = {}, its[RP_N] = {};
    unsigned long long t = 0;
    __device__ __forceinline__ void start() {
        if (SALP_ROLLOUT_PROF) t = __builtin_amdgcn_s_memtime();
    }
    __device__ __forceinline__ void lap(int part, int64_t iterations = 0) {
        if (SALP_ROLLOUT_PROF) {
            const unsigned long long now = __builtin_amdgcn_s_memtime();
            cyc[part] += now - t;
            its[part] += (unsigned long long)iterations;
            t = now;
        }
    }
    __device__ __forceinline__ void flush() {
        if (SALP_ROLLOUT_PROF && (threadIdx.x & 63) == 0)
            for (int k = 0; k < RP_N; ++k) {
                atomicAdd(&g_roll_prof[0][k], cyc[k]);
                atomicAdd(&g_roll_prof[1][k], its[k]);
            }
    }
};

#if SALP_ROLLOUT_RESEAT
template <bool RAND, bool POL>
__global__ __launch_bounds__(kBlock) void k_rollout(RolloutArgs A) {
    double* const S = A.S;
    const Params& P = A.P;
    const int64_t base = (int64_t)blockIdx.x * blockDim.x;
    const int lane = (int)threadIdx.x;
    __shared__ double s_cache32[salp::C32_N * salp::LANES];
    __shared__ double s_spill[salp::SPILL_N * salp::LANES];
    __shared__ int64_t s_steps[kBlock];
    __shared__ uint8_t s_flags[kBlock];              // pending | active << 1, per slot
    __shared__ int16_t s_slot[2][kBlock];            // slot each lane held (double-buffered)
    __shared__ uint64_t s_mask[2][kBlock / 64];      // unsteady ballots per wave (double-buffered)
    __shared__ uint64_t s_amask[2][kBlock / 64];     // active ballots per wave (double-buffered)
    int s = lane;                                    // this lane runs env base + s
    int64_t i = base + s;
    bool pending = false, active = false;
    int64_t steps = 0;
    Hot h{};
    if (i < P.n) {
        pending = !A.fresh && SF(SALP_F_PENDING) != 0.0;
        steps = A.B.steps_done ? A.B.steps_done[i] : 0;
        active = !(A.max_steps > 0 && steps >= A.max_steps);
        salp::load_hot<RAND>(h, S, P, i);
        salp::resume_cycle(h, S, P, i);
        salp::fill_cache32(P, h.c, salp::Cache32{s_cache32 + s});
    }
    // slots past the end of the batch hold no env: never active, never stored
    if (!active) h.b2 = -INFINITY;
    bool all_done = false;   // no env of the workgroup has an env-step left (max_steps)
    RollProf prof;
    prof.start();
    for (int64_t c = 0;; ++c) {
        const bool last = c == A.n_chunks || all_done;
        const salp::SpillSlot sp{s_spill + s};
        // Env-step boundary of the lanes whose cycle ended (or that start one)
        const bool need = active && (!pending || !(h.ct < h.b2));
        bool uns = unsteady(h, P, active);
        salp::spill<RAND>(h, sp);
        if (need) {
            if (RAND) {
                uns = lane_boundary_call<RAND, POL>(&A, s_spill + s, i, &pending, &active, &steps, s_cache32 + s);
            } else {
                const RolloutArgs a = fresh_args();
                uns = lane_boundary<RAND, POL>(a, sp, i, pending, active, steps, s_cache32 + s);
            }
        }
        if (last) {
            const RolloutArgs a = fresh_args();
            salp::unspill<RAND>(h, sp, a.P, (uint64_t)(a.P.env_offset + i));
            if (i < a.P.n) salp::store_hot<RAND>(h, a.S, a.P, i);
            break;
        }
        // Re-seat: lane k of the workgroup takes the k-th env in the order
        // (unsteady envs by lane, then steady envs by lane).  One barrier; the
        // double buffers keep the next boundary's writes off this one's reads.
        const int b = (int)(c & 1);
        s_steps[s] = steps;
        s_flags[s] = (uint8_t)((pending ? 1 : 0) | (active ? 2 : 0));
        s_slot[b][lane] = (int16_t)s;
        const uint64_t ballot = __ballot(uns);
        const uint64_t aballot = __ballot(active);
        if ((lane & 63) == 0) {
            s_mask[b][lane >> 6] = ballot;
            s_amask[b][lane >> 6] = aballot;
        }
        prof.lap(RP_BOUNDARY);
        __syncthreads();
        prof.lap(RP_BARRIER);
        uint64_t m[kBlock / 64];
        int n_uns = 0;
        uint64_t any_active = 0;
#pragma unroll
        for (int w = 0; w < kBlock / 64; ++w) {
            m[w] = s_mask[b][w];
            n_uns += __popcll(m[w]);
            any_active |= s_amask[b][w];
        }
        all_done = any_active == 0;   // the same for every lane of the workgroup
        int from;
        if (lane < n_uns) {
            from = nth_set_lane(m, lane);
        } else {
#pragma unroll
            for (int w = 0; w < kBlock / 64; ++w) m[w] = ~m[w];
            from = nth_set_lane(m, lane - n_uns);
        }
        s = s_slot[b][from];
        i = base + s;
        const int fl = s_flags[s];
        pending = (fl & 1) != 0;
        active = (fl & 2) != 0;
        steps = s_steps[s];
        {
            const RolloutArgs a = fresh_args();
            salp::unspill<RAND>(h, salp::SpillSlot{s_spill + s}, a.P, (uint64_t)(a.P.env_offset + i));
        }
        if (!active) h.b2 = -INFINITY;   // a finished lane (or an empty slot) ticks no more
        if (all_done) continue;          // next pass stores the state and leaves
        prof.lap(RP_RESEAT);
        const salp::Cache32 c32{s_cache32 + s};
        const Params PV = salp::pin_params(P);
        int32_t k = 0;
        for (; k < A.chunk; ++k) {
            if (__all(!(h.ct < h.b2) || salp::next_tick_steady(h, PV))) break;
            if (h.ct < h.b2) salp::tick<false, RAND, true>(h, PV, c32);
        }
        prof.lap(RP_FULL, k);
        const int32_t ks = (int32_t)(((int64_t)(A.chunk - k) * A.steady_q8) >> 8);
        // steady ticks until every ticking lane of the wave is settled, then
        // settled ticks (salp_device.h tick; lanes whose cycle has ended idle)
        int32_t j = 0;
        for (; j < ks; ++j) {
            bool settled = true;
            if (h.ct < h.b2) settled = salp::tick<false, RAND, true, true>(h, PV, c32);
            if (__all(settled)) {
                ++j;
                break;
            }
        }
        prof.lap(RP_STEADY, j);
        const int32_t j0 = j;
        for (; j < ks; ++j)
            if (h.ct < h.b2) salp::tick<false, RAND, true, true, true>(h, PV, c32);
        prof.lap(RP_SETTLED, j - j0);
    }
    prof.flush();
    if (A.B.steps_done && i < P.n) A.B.steps_done[i] = steps;
}
#else
template <bool RAND, bool POL>
__global__ __launch_bounds__(kBlock) void k_rollout(RolloutArgs A) {
    double* const S = A.S;
    const Params& P = A.P;
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P.n) return;
    bool pending = !A.fresh && SF(SALP_F_PENDING) != 0.0;
    int64_t steps = A.B.steps_done ? A.B.steps_done[i] : 0;
    bool active = !(A.max_steps > 0 && steps >= A.max_steps);
    LANE_CACHE32();
    __shared__ double s_spill[salp::SPILL_N * salp::LANES];
    const salp::SpillSlot sp{s_spill + threadIdx.x};
    Hot h;
    salp::load_hot<RAND>(h, S, P, i);
    salp::resume_cycle(h, S, P, i);
    salp::fill_cache32(P, h.c, c32);
    if (!active) h.b2 = -INFINITY;
    for (int64_t c = 0; c <= A.n_chunks; ++c) {
        // Env-step boundary, taken by the whole wave when any lane needs it.
        const bool need = active && (!pending || !(h.ct < h.b2));
        const bool last = c == A.n_chunks || !__any(active || need);
        if (__any(need) || last) {
            salp::spill<RAND>(h, sp);
            if (need) {
                const RolloutArgs a = fresh_args();
                const uint64_t env_id = (uint64_t)(a.P.env_offset + i);
                // cold loads first: their HBM latency hides under the LDS unspill
                salp::ColdRegs<RAND> C;
                salp::load_cold<RAND>(C, a.S, a.P, i);
                Hot hb;
                salp::unspill<RAND>(hb, sp, a.P, env_id);
                rollout_boundary<RAND, POL>(hb, &C, a.P, i, env_id, pending, active, steps, a.max_steps, a.B,
                                            a.reward_sum, a.R, c32);
                salp::store_cold<RAND>(C, a.S, a.P, i);
                salp::spill<RAND>(hb, sp);
            }
            {
                const RolloutArgs a = fresh_args();
                salp::unspill<RAND>(h, sp, a.P, (uint64_t)(a.P.env_offset + i));
                if (last) {
                    salp::store_hot<RAND>(h, a.S, a.P, i);
                    break;
                }
            }
            if (!active) h.b2 = -INFINITY;   // a finished lane ticks no more
        }
        const Params PV = salp::pin_params(P);
        for (int32_t k = 0; k < A.chunk; ++k)
            if (h.ct < h.b2) salp::tick<false, RAND, true>(h, PV, c32);
    }
    if (A.B.steps_done) A.B.steps_done[i] = steps;
}
#endif

// ----------------------------------------------------------------------
// k_rollout_pair: the chained rollout with every env on TWO waves
// (salp_pair.h).  A workgroup is 4 waves = 2 groups of 64 envs; wave 2g is
// group g's A wave, wave 2g + 1 its B wave, and lane l of both holds the same
// env.  128 env slots per workgroup, re-seated at every chunk boundary like
// k_rollout (unsteady envs first).  Env-step boundaries run on the A waves
// with the whole state assembled in the slot; inside a chunk the two waves of
// a group meet once per tick through LDS (two packet buffers per direction,
// a release/acquire counter per wave; no workgroup barrier), and the A wave
// decides each tick's kind (full / steady / settled / end of chunk) exactly as
// k_rollout's loops do and sends it with its packet.  Same per-env results as
// k_rollout.
constexpr int kPairEnvs = 128;
constexpr int kXchAB = 5;    // A -> B: v x (M_a v) (3), jet torque y, z
constexpr int kXchBA = 13;   // B -> A: w (3), alpha y, z, sin/cos of roll, pitch, yaw (6), drag-force coefficients (2)
constexpr int kXchBase = 4 * kXchAB * 64;                           // first double of the B -> A packets
constexpr int kXchDoubles = kXchBase + 4 * kXchBA * 64;
static_assert(kXchDoubles <= salp::SPILL_N * kPairEnvs, "the packets live in the spill slots' LDS");
// A wave gives up on its partner after this many polls (s_sleep 1 = 64 cycles
// each: 2^21 x 64 = 134 M cycles, ~56 ms at 2.4 GHz, against ~1 us for a
// tick's round trip and ~50 us for the longest legitimate wait, a boundary
// round of value jobs): the kernel always ends instead of hanging the GPU.
// Such an env's results are invalid; g_pair_timeouts counts the give-ups and
// salp_pair_timeouts reads it (the Python layer raises on a nonzero count).
constexpr int kPairSpin = 1 << 21;
__device__ unsigned int g_pair_timeouts;

// SALP_PAIR_PROF=1 (experiment builds only, tools/build_variant.py): s_memtime
// cycles per wave and phase, summed over the launch's waves into
// g_pair_prof[role][phase] (read back by salp_debug_pair_prof).
#ifndef SALP_PAIR_PROF
#define SALP_PAIR_PROF 0
#endif
enum { PP_BOUNDARY, PP_TICK, PP_PUBLISH, PP_WAIT, PP_READ, PP_WORLD, PP_BARRIER, PP_N };
__device__ unsigned long long g_pair_prof[2][PP_N];
struct PairProf {
    unsigned long long acc[PP_N] = {};
    unsigned long long t = 0;
    __device__ __forceinline__ void start() {
        if (SALP_PAIR_PROF) t = __builtin_amdgcn_s_memtime();
    }
    __device__ __forceinline__ void lap(int phase) {
        if (SALP_PAIR_PROF) {
            const unsigned long long now = __builtin_amdgcn_s_memtime();
            acc[phase] += now - t;
            t = now;
        }
    }
    __device__ __forceinline__ void flush(int role) {
        if (SALP_PAIR_PROF && (threadIdx.x & 63) == 0)
            for (int k = 0; k < PP_N; ++k) atomicAdd(&g_pair_prof[role][k], acc[k]);
    }
};

struct PairShared {
    double cache32[salp::C32_N * kPairEnvs];
    double big[salp::SPILL_N * kPairEnvs];   // spill slots between chunks | tick packets inside a chunk
    int64_t steps[kPairEnvs];
    int16_t slot[2][kPairEnvs];
    uint64_t mask[2][2], amask[2][2];
    int cnt[2][2];                            // [group][role]: packets published
    int mode[2][2];                           // [group][buffer]: the tick kind wave A sent
    uint8_t flags[kPairEnvs];
};

// salp_collect boundaries in k_rollout_pair: the A wave runs the env-steps and
// the policy mean; the value-network evaluations (SB3's V(obs) of every new
// step and gamma V(terminal obs) of a timeout's bootstrap) go to the B wave as
// jobs, one LDS buffer per boundary round ("rep" of rollout_boundary), which
// the B wave evaluates while the A wave goes on (ValuesToPartner).  Same
// expressions, same results.
struct PairJobs {
    __attribute__((aligned(16))) float pi_l2[kPolL2];   // the actor's second layer and heads (policy_actor_l2)
    float boot_obs[4][kPIN][kPairEnvs];
    float val_obs[4][kPIN][kPairEnvs];
    float boot_rew[4][kPairEnvs];
    int32_t boot_step[4][kPairEnvs];
    int32_t val_step[4][kPairEnvs];
    uint8_t flags[4][kPairEnvs];   // 1: bootstrap job, 2: value job
    int cnt[2];                    // [group]: job buffers the A wave published
    int done[2];                   // [group]: boundaries whose jobs are all published (chunk index + 1)
};

// Polls with s_sleep 1 (64 cycles) between them: s_sleep 0, 2 or none measured
// the same, 4 slower (profiles/r4_experiments.md r4t).
__device__ __forceinline__ bool pair_wait(int* flag, int target) {
    for (int it = 0; it < kPairSpin; ++it) {
        if (__hip_atomic_load(flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) >= target) return true;
        __builtin_amdgcn_s_sleep(1);
    }
    if ((threadIdx.x & 63) == 0) atomicAdd(&g_pair_timeouts, 1u);
    return false;
}
__device__ __forceinline__ void pair_publish(int* flag, int value) {
    __hip_atomic_store(flag, value, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// k_step_wave's LDS: the geometry table (wave 0), the velocity ring (wave 0 ->
// wave 1) with its two counters, and wave 1's hand-over of the angle chain.
constexpr int kWaveRing = 64;                       // ticks wave 0 may run ahead
enum { WR_V0, WR_V1, WR_V2, WR_W0, WR_W1, WR_W2, WR_STRIDE = 6 };
enum { WX_E0, WX_E1, WX_E2, WX_P0, WX_P1, WX_P2, WX_SP, WX_CP, WX_ST, WX_CTH, WX_FAIL, WX_N };
struct WaveShared {
    double rows[kWave * WG_STRIDE];
    double ring[kWaveRing * WR_STRIDE];
    double xchg[WX_N];
    double c32[salp::C32_N];
    int produced, consumed;   // ticks of this cycle wave 0 has published / wave 1 has read
};

// One breathing cycle of the env both waves hold (Robot.step_through_cycle's
// loop, src/robot.py:750-765).  Both waves run the same clock (the same sums),
// so they agree on the cycle's tick count.  Returns false if a wait gave up
// (g_pair_timeouts counts it; the env's results are then invalid).
template <bool RAND>
__device__ __forceinline__ bool run_cycle_split(Hot& h, const Params& P, salp::Cache32 c32, WaveShared& W) {
    const bool kin = threadIdx.x >= kWave;
    bool ok = true;
    int g = 0;
    if (!kin) {
        while (h.ct < h.b2 && g < kMaxTicksPerCycle) {
            wave_geometry_rows(h, P, c32, W.rows);
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");   /* rows of the other lanes */
            int last = 0;
            for (int j = 0; j < kWave && h.ct < h.b2 && g < kMaxTicksPerCycle; ++j, ++g) {
                /* the row is read before the forces, so that its LDS latency hides under them */
                double x[WG_RI1 + 1];
                const double* r = W.rows + j * WG_STRIDE;
#pragma unroll
                for (int k = 0; k <= WG_RI1; ++k) x[k] = r[k];
                /* the forces' SETTLED instance where its constants are the values the lane holds
                 * (jet force off, water-mass rate, centre-of-mass rate and acceleration
                 * +0, inertia unchanged): the same results with less arithmetic (tick) */
                const bool settled = h.phase != salp::JET &&
                                     (__double_as_longlong(h.geo.mr) | __double_as_longlong(h.comr) |
                                      __double_as_longlong(h.coma)) == 0 &&
                                     h.geo.I0 == h.pI0 && h.geo.I1 == h.pI1 && h.pI2 == h.pI1;
                if (settled)
                    salp::tick_dynamics<false, RAND, true, salp::TD_FORCES | salp::TD_POSITIONS>(h, P, nullptr, 0);
                else
                    salp::tick_dynamics<false, RAND, false, salp::TD_FORCES | salp::TD_POSITIONS>(h, P, nullptr, 0);
                /* this tick's velocities to wave 1 (a slot it has read) */
                if (g >= kWaveRing) ok = pair_wait(&W.consumed, g - kWaveRing + 1) && ok;
                double* q = W.ring + (g % kWaveRing) * WR_STRIDE;
                q[WR_V0] = h.v0; q[WR_V1] = h.v1; q[WR_V2] = h.v2;
                q[WR_W0] = h.w0; q[WR_W1] = h.w1; q[WR_W2] = h.w2;
                pair_publish(&W.produced, g + 1);
                h.ct = x[WG_CT]; h.time = x[WG_TIME]; h.phase = (int)x[WG_PHASE]; h.W = x[WG_W];
                h.com = x[WG_COM]; h.comr = x[WG_COMR]; h.coma = x[WG_COMA];
                salp::Geo& q2 = h.geo;
                q2.m = x[WG_M]; q2.mr = x[WG_MR]; q2.I0 = x[WG_I0]; q2.I1 = x[WG_I1];
                q2.kc0 = x[WG_KC0]; q2.kc1 = x[WG_KC1]; q2.ra0 = x[WG_RA0]; q2.ra1 = x[WG_RA1];
                q2.dimx = x[WG_DIMX]; q2.dimy = x[WG_DIMY]; q2.speed = x[WG_SPEED]; q2.rx = x[WG_RX];
                q2.rm = x[WG_RM]; q2.rI0 = x[WG_RI0]; q2.rI1 = x[WG_RI1];
                last = j;
            }
            const double* r = W.rows + last * WG_STRIDE;
            h.L = r[WG_L]; h.V = r[WG_V]; h.pV = r[WG_PV];
            h.g32 = r[WG_G32] != 0.0; h.pv32 = r[WG_PV32] != 0.0;
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");   /* the table is rewritten next */
        }
    } else {
        double ct = h.ct;
        for (; ct < h.b2 && g < kMaxTicksPerCycle; ++g) {
            ok = pair_wait(&W.produced, g + 1) && ok;
            const double* q = W.ring + (g % kWaveRing) * WR_STRIDE;
            h.v0 = q[WR_V0]; h.v1 = q[WR_V1]; h.v2 = q[WR_V2];
            h.w0 = q[WR_W0]; h.w1 = q[WR_W1]; h.w2 = q[WR_W2];
            pair_publish(&W.consumed, g + 1);
            salp::tick_dynamics<false, RAND, false, salp::TD_KINEMATICS>(h, P, nullptr, 0);
            ct += salp::DT;
        }
    }
    return ok;
}

// SalpRobotEnv.step with one env per workgroup of two waves (run_cycle_split):
// env = blockIdx.x; both waves load the env and run begin_step identically
// (wave 0 stores), run the cycle split, and wave 1 hands the angle chain to
// wave 0, which ends the env-step (k_step's epilogue) and stores.
template <bool RAND>
__global__ __launch_bounds__(2 * kWave) void k_step_wave(double* S, Params P, const float* actions,
                                                         float* obs_out, double* reward_out,
                                                         uint8_t* term_out, uint8_t* trunc_out,
                                                         int auto_reset, float* term_obs_out, double* info_out) {
    const int64_t i = blockIdx.x;
    if (i >= P.n) return;
    __shared__ __attribute__((aligned(16))) WaveShared W;
    const salp::Cache32 c32{W.c32, 1};
    const bool kin = threadIdx.x >= kWave;
    if (threadIdx.x == 0) {
        W.produced = 0;
        W.consumed = 0;
    }
    Hot h;
    salp::load_hot<RAND>(h, S, P, i);
    {
        salp::ColdRegs<RAND> C;
        salp::load_cold<RAND>(C, S, P, i);
        salp::begin_step<RAND>(h, &C, P, i, actions[3 * i], actions[3 * i + 1], actions[3 * i + 2], c32);
        if (!kin) salp::store_cold<RAND>(C, S, P, i);
    }
    __syncthreads();
    const bool ok = run_cycle_split<RAND>(h, P, c32, W);
    __syncthreads();
    if (kin) {
        if (threadIdx.x == kWave) {
            double* x = W.xchg;
            x[WX_E0] = h.e0; x[WX_E1] = h.e1; x[WX_E2] = h.e2;
            x[WX_P0] = h.p0; x[WX_P1] = h.p1; x[WX_P2] = h.p2;
            x[WX_SP] = h.sp; x[WX_CP] = h.cp; x[WX_ST] = h.st; x[WX_CTH] = h.cth;
            x[WX_FAIL] = ok ? 0.0 : 1.0;
        }
    }
    __syncthreads();
    if (kin) return;
    {
        const double* x = W.xchg;
        h.e0 = x[WX_E0]; h.e1 = x[WX_E1]; h.e2 = x[WX_E2];
        h.p0 = x[WX_P0]; h.p1 = x[WX_P1]; h.p2 = x[WX_P2];
        h.sp = x[WX_SP]; h.cp = x[WX_CP]; h.st = x[WX_ST]; h.cth = x[WX_CTH];
        /* a partner wait that gave up (g_pair_timeouts counted it) leaves this env's
         * cycle unfinished: its state is not the reference's, so mark it invalid
         * rather than hand it on as a result -- NaN motion state, which every
         * caller already treats as a diverged env (NaN obs and reward, the
         * learner's divergence guard resets it, salp_pair_timeouts says why) */
        if (!ok || x[WX_FAIL] != 0.0) salp::poison_motion(h);
    }
    float o[SALP_OBS_DIM_MAX];
    double* info = info_out ? info_out + (size_t)SALP_INFO_DIM * i : nullptr;
    salp::ColdRegs<RAND> C;
    salp::load_cold<RAND>(C, S, P, i);
    double& sc = salp::sref(&C, P, i, SALP_F_STEP_COUNT);
    sc = sc + 1.0;
    const salp::StepOut r = salp::finish_step<RAND>(h, &C, P, i, o, info);
    if (term_obs_out)
        for (int k = 0; k < P.obs_dim; ++k) term_obs_out[(size_t)i * P.obs_dim + k] = o[k];
    if (auto_reset && (r.terminated || r.truncated)) salp::reset_env_philox(h, &C, P, i, o);
    salp::store_cold<RAND>(C, S, P, i);
    if (reward_out) reward_out[i] = r.reward;
    if (term_out) term_out[i] = r.terminated;
    if (trunc_out) trunc_out[i] = r.truncated;
    if (obs_out)
        for (int k = 0; k < P.obs_dim; ++k) obs_out[(size_t)i * P.obs_dim + k] = o[k];
    salp::store_hot<RAND>(h, S, P, i);
}

struct ValuesToPartner {
    static constexpr bool kDefer = true;
    static constexpr bool kL2 = true;
    PairJobs* J;
    int grp, s, buf;
    __device__ __forceinline__ const float* l2() const { return J->pi_l2; }
    __device__ __forceinline__ void start_rep() {
        buf = __hip_atomic_load(&J->cnt[grp], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) & 3;
    }
    __device__ __forceinline__ void boot(const float* o, int od, float rew, int64_t step) {
        for (int k = 0; k < od; ++k) J->boot_obs[buf][k][s] = o[k];
        J->boot_rew[buf][s] = rew;
        J->boot_step[buf][s] = (int32_t)step;
        J->flags[buf][s] |= 1;
    }
    __device__ __forceinline__ void value(const float* o, int od, int64_t step) {
        for (int k = 0; k < od; ++k) J->val_obs[buf][k][s] = o[k];
        J->val_step[buf][s] = (int32_t)step;
        J->flags[buf][s] |= 2;
    }
    __device__ __forceinline__ void publish() {
        const int c = __hip_atomic_load(&J->cnt[grp], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        pair_publish(&J->cnt[grp], c + 1);
    }
};

// The B wave's side: evaluate the published jobs of the boundary of chunk c
// until the A wave marks it done.  `taken`: job buffers evaluated so far.
__device__ __forceinline__ void pair_value_jobs(PairJobs& J, const RolloutArgs& A, int grp, int s, int64_t c,
                                                int& taken) {
    const PolicyW w = (PolicyW)A.R.weights;
    const int64_t i = (int64_t)blockIdx.x * kPairEnvs + s;
    const int od = A.P.obs_dim;
    for (int it = 0; it < kPairSpin; ++it) {
        const int pub = __hip_atomic_load(&J.cnt[grp], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (taken < pub) {
            const int b = taken & 3;
            const int f = J.flags[b][s];
            if (f & 1) {
                float x[kPIN];
#pragma unroll
                for (int k = 0; k < kPIN; ++k) x[k] = k < od ? J.boot_obs[b][k][s] : 0.0f;
                const float rew = J.boot_rew[b][s] + (float)A.R.gamma * policy_value(w, x);
                A.R.rewards[(size_t)J.boot_step[b][s] * (size_t)A.P.n + (size_t)i] = rew;
            }
            if (f & 2) {
                float x[kPIN];
#pragma unroll
                for (int k = 0; k < kPIN; ++k) x[k] = k < od ? J.val_obs[b][k][s] : 0.0f;
                A.R.values[(size_t)J.val_step[b][s] * (size_t)A.P.n + (size_t)i] = policy_value(w, x);
            }
            ++taken;
            continue;
        }
        if (__hip_atomic_load(&J.done[grp], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) >= (int)(c + 1)) {
            if (taken < __hip_atomic_load(&J.cnt[grp], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP)) continue;
            return;
        }
        __builtin_amdgcn_s_sleep(1);
    }
    if ((threadIdx.x & 63) == 0) atomicAdd(&g_pair_timeouts, 1u);
}

// Position of the k-th set bit of the 128-bit mask m[0..1] (k < popcount).
__device__ __forceinline__ int nth_set_seat(const uint64_t* m, int k) {
    const int c0 = __popcll(m[0]);
    uint64_t w = k < c0 ? m[0] : m[1];
    int base = k < c0 ? 0 : 64;
    if (k >= c0) k -= c0;
    int pos = 0;
#pragma unroll
    for (int half = 32; half > 0; half >>= 1) {
        const uint64_t lo = w & ((1ull << half) - 1ull);
        const int c = __popcll(lo);
        if (k >= c) {
            k -= c;
            w >>= half;
            pos += half;
        } else {
            w = lo;
        }
    }
    return base + pos;
}

// The slot state's unsteady flag (k_rollout's `unsteady`), read from the slot.
__device__ __forceinline__ bool slot_unsteady(salp::SpillSlot sl, const Params& P, bool active) {
    double mx, b1, b2;
    salp::cycle_bounds_of(sl[salp::SP_REFILL], sl[salp::SP_TURN], sl[salp::SP_JET], sl[salp::SP_COAST], &mx, &b1,
                          &b2);
    const double ct = sl[salp::SP_CT];
    const bool g32 = (((int)sl[salp::SP_FLAGS]) & 4) != 0;
    return active && ct < b2 && !salp::pair_next_steady(ct, sl[salp::SP_L], sl[salp::SP_WID], g32, b1, mx, P);
}

// Re-seat after the boundary: the seat's new slot and its bookkeeping (both
// waves of a group compute the same assignment).
__device__ __forceinline__ void pair_reseat(PairShared& sh, int b, int seat, int& s, int64_t& steps, bool& pending,
                                            bool& active, bool& all_done) {
    uint64_t m[2] = {sh.mask[b][0], sh.mask[b][1]};
    const int n_uns = __popcll(m[0]) + __popcll(m[1]);
    all_done = (sh.amask[b][0] | sh.amask[b][1]) == 0;
    int from;
    if (seat < n_uns) {
        from = nth_set_seat(m, seat);
    } else {
        m[0] = ~m[0];
        m[1] = ~m[1];
        from = nth_set_seat(m, seat - n_uns);
    }
    s = sh.slot[b][from];
    const int fl = sh.flags[s];
    pending = (fl & 1) != 0;
    active = (fl & 2) != 0;
    steps = sh.steps[s];
}

// k_rollout_split (SPLIT): the same workgroup, slots, re-seating and
// boundaries as k_rollout_pair, but the tick is split along its one-way
// dependences instead of Newton <-> Euler: the A wave runs whole ticks without
// the angle chain (tick<..., TD_FORCES | TD_POSITIONS>: forces, v / w
// integration, clock, phase, geometry, the steady / settled decisions), and
// the B wave follows with the angle chain (TD_KINEMATICS: Euler-angle rates,
// angles, their sin / cos, the world-frame position), which nothing the A wave
// computes reads.  Per wave-tick the A wave writes every lane's v and w into an
// LDS ring of kSplitRing ticks; it waits only when the B wave is a whole ring
// behind, so there is no per-tick round trip.  Each value is the expression
// tick() computes: results equal k_rollout's and the oracle's bit for bit.
constexpr int kSplitRing = 8;            // wave-ticks the A wave may run ahead
constexpr int kSplitEnd = 1 << 30;       // the A wave's counter: end of its chunk
static_assert(2 * kSplitRing * 6 * 64 <= salp::SPILL_N * kPairEnvs, "the rings live in the spill slots' LDS");
constexpr int kSplitParts = salp::TD_FORCES | salp::TD_POSITIONS;

template <bool POL, bool SPLIT = false>
__device__ __forceinline__ void pair_wave_a(PairShared& sh, PairJobs* jobs, const RolloutArgs& A, int grp, int lane) {
    const Params& P = A.P;
    const int seat = grp * 64 + lane;
    const int64_t base = (int64_t)blockIdx.x * kPairEnvs;
    int s = seat;
    int64_t i = base + s;
    bool pending = false, active = false;
    int64_t steps = 0;
    {   // load this seat's env into its slot (the whole state)
        double* const S = A.S;
        Hot h{};
        if (i < P.n) {
            pending = !A.fresh && SF(SALP_F_PENDING) != 0.0;
            steps = A.B.steps_done ? A.B.steps_done[i] : 0;
            active = !(A.max_steps > 0 && steps >= A.max_steps);
            salp::load_hot<false>(h, S, P, i);
            salp::resume_cycle(h, S, P, i);
            salp::fill_cache32(P, h.c, salp::Cache32{sh.cache32 + s, kPairEnvs});
        }
        salp::spill<false>(h, salp::SpillSlot{sh.big + s, kPairEnvs});
        if (lane < 2) sh.cnt[grp][lane] = 0;
        if (POL && lane == 0) {
            jobs->cnt[grp] = 0;
            jobs->done[grp] = 0;
        }
    }
    __syncthreads();   // #0
    int pub = 0, rcv = 0;
    bool all_done = false;
    PairProf prof;
    prof.start();
    for (int64_t c = 0;; ++c) {
        const bool last = c == A.n_chunks || all_done;
        const salp::SpillSlot sl{sh.big + s, kPairEnvs};
        bool need;
        {
            double mx, b1, b2;
            salp::cycle_bounds_of(sl[salp::SP_REFILL], sl[salp::SP_TURN], sl[salp::SP_JET], sl[salp::SP_COAST], &mx,
                                  &b1, &b2);
            need = active && (!pending || !(sl[salp::SP_CT] < b2));
        }
        if (POL)
#pragma unroll
            for (int b = 0; b < 4; ++b) jobs->flags[b][s] = 0;
        if (need) {
            const RolloutArgs a = fresh_args();
            const uint64_t env_id = (uint64_t)(a.P.env_offset + i);
            salp::ColdRegs<false> C;
            salp::load_cold<false>(C, a.S, a.P, i);
            Hot hb;
            salp::unspill<false>(hb, sl, a.P, env_id);
            if (POL)
                rollout_boundary<false, POL>(hb, &C, a.P, i, env_id, pending, active, steps, a.max_steps, a.B,
                                             a.reward_sum, a.R, salp::Cache32{sh.cache32 + s, kPairEnvs},
                                             ValuesToPartner{jobs, grp, s, 0});
            else
                rollout_boundary<false, POL>(hb, &C, a.P, i, env_id, pending, active, steps, a.max_steps, a.B,
                                             a.reward_sum, a.R, salp::Cache32{sh.cache32 + s, kPairEnvs});
            salp::store_cold<false>(C, a.S, a.P, i);
            salp::spill<false>(hb, sl);
        }
        if (POL) pair_publish(&jobs->done[grp], (int)c + 1);   // this boundary's jobs are all out
        if (last) {
            const RolloutArgs a = fresh_args();
            Hot h;
            salp::unspill<false>(h, sl, a.P, (uint64_t)(a.P.env_offset + i));
            if (i < a.P.n) {
                salp::store_hot<false>(h, a.S, a.P, i);
                if (a.B.steps_done) a.B.steps_done[i] = steps;
            }
            prof.lap(PP_BOUNDARY);
            prof.flush(0);
            return;
        }
        const bool uns = slot_unsteady(sl, P, active);
        const int b = (int)(c & 1);
        sh.steps[s] = steps;
        sh.flags[s] = (uint8_t)((pending ? 1 : 0) | (active ? 2 : 0));
        sh.slot[b][seat] = (int16_t)s;
        const uint64_t ballot = __ballot(uns), aballot = __ballot(active);
        if (lane == 0) {
            sh.mask[b][grp] = ballot;
            sh.amask[b][grp] = aballot;
        }
        prof.lap(PP_BOUNDARY);
        __syncthreads();   // #1
        prof.lap(PP_BARRIER);
        pair_reseat(sh, b, seat, s, steps, pending, active, all_done);
        i = base + s;
        if (all_done) continue;
        const salp::SpillSlot ns{sh.big + s, kPairEnvs};
        const salp::Cache32 c32{sh.cache32 + s, kPairEnvs};
        if constexpr (SPLIT) {
            Hot h;
            salp::unspill<false>(h, ns, P, (uint64_t)(P.env_offset + i));
            if (!active) h.b2 = -INFINITY;
            prof.lap(PP_BOUNDARY);
            __syncthreads();   // #2: slots read; the ring may overwrite them now
            prof.lap(PP_BARRIER);
            {
                const Params PV = salp::pin_params(P);
                double2* const ring = reinterpret_cast<double2*>(sh.big) + grp * kSplitRing * 3 * 64 + lane;
                int g = 0;           // wave-ticks published
                int freed = kSplitRing;   // slots below this count are free (the B wave read them)
                bool ok = true;
                const auto publish = [&]() {
                    if (g >= freed) {
                        prof.lap(PP_TICK);
                        const int want = g - kSplitRing + 1;
                        ok = pair_wait(&sh.cnt[grp][1], want) && ok;
                        freed = __hip_atomic_load(&sh.cnt[grp][1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) +
                                kSplitRing;
                        freed = freed > g ? freed : g + 1;
                        prof.lap(PP_WAIT);
                    }
                    double2* const q = ring + (g % kSplitRing) * 3 * 64;
                    q[0] = make_double2(h.v0, h.v1);
                    q[64] = make_double2(h.v2, h.w0);
                    q[128] = make_double2(h.w1, h.w2);
                    pair_publish(&sh.cnt[grp][0], ++g);
                };
                // k_rollout's chunk: full ticks while a ticking lane is unsteady, then
                // the steady budget (settled once every ticking lane is)
                int32_t k = 0;
                for (; k < A.chunk && ok; ++k) {
                    if (__all(!(h.ct < h.b2) || salp::next_tick_steady(h, PV))) break;
                    if (h.ct < h.b2) salp::tick<false, false, true, false, false, kSplitParts>(h, PV, c32);
                    publish();
                }
                const int32_t ks = (int32_t)(((int64_t)(A.chunk - k) * A.steady_q8) >> 8);
                int32_t j = 0;
                for (; j < ks && ok; ++j) {
                    bool settled = true;
                    if (h.ct < h.b2) settled = salp::tick<false, false, true, true, false, kSplitParts>(h, PV, c32);
                    publish();
                    if (__all(settled)) {
                        ++j;
                        break;
                    }
                }
                for (; j < ks && ok; ++j) {
                    if (h.ct < h.b2) salp::tick<false, false, true, true, true, kSplitParts>(h, PV, c32);
                    publish();
                }
                pair_publish(&sh.cnt[grp][0], g | kSplitEnd);
                prof.lap(PP_TICK);
            }
            __syncthreads();   // #3: the B wave has read the ring
            prof.lap(PP_BARRIER);
            if (lane == 0) {   /* the next chunk counts from 0 (neither wave reads them before #2) */
                sh.cnt[grp][0] = 0;
                sh.cnt[grp][1] = 0;
            }
            salp::spill<false>(h, ns);   // the angle chain's fields are stale here: the B wave's follow
            __syncthreads();   // #3b
            prof.lap(PP_BOUNDARY);
            __syncthreads();   // #4: slots whole again
            prof.lap(PP_BARRIER);
            continue;
        }
        salp::HotA h;
        salp::unspill_a(h, ns);
        if (!active) h.b2 = -INFINITY;
        prof.lap(PP_BOUNDARY);
        __syncthreads();   // #2: slots read; the packets may overwrite them now
        prof.lap(PP_BARRIER);
        {
            const Params PV = salp::pin_params(P);
            const int chunk = A.chunk, q8 = A.steady_q8;
            double* const ab = sh.big + grp * 2 * kXchAB * 64 + lane;
            double* const ba = sh.big + kXchBase + grp * 2 * kXchBA * 64 + lane;
            int k = 0, j = 0, ks = 0, stage = 0;
            const auto decide = [&]() -> int {
                if (stage == 0) {
                    if (k < chunk && !__all(!(h.ct < h.b2) ||
                                            salp::pair_next_steady(h.ct, h.L, h.W, h.g32, h.b1, h.mx, PV))) {
                        ++k;
                        return salp::PM_FULL;
                    }
                    ks = (int32_t)(((int64_t)(chunk - k) * q8) >> 8);
                    stage = 1;
                }
                if (j >= ks) return salp::PM_END;
                ++j;
                return stage == 1 ? salp::PM_STEADY : salp::PM_SETTLED;
            };
            const auto publish = [&](int mode) {
                double X[3], jt[2];
                salp::a_prepare(h, PV, X, jt);
                double* const o = ab + (pub & 1) * kXchAB * 64;
                o[0 * 64] = X[0]; o[1 * 64] = X[1]; o[2 * 64] = X[2]; o[3 * 64] = jt[0]; o[4 * 64] = jt[1];
                if (lane == 0) sh.mode[grp][pub & 1] = mode;
                pair_publish(&sh.cnt[grp][0], ++pub);
            };
            bool ok = true;
            const auto recv = [&]() {
                prof.lap(PP_PUBLISH);
                ok = pair_wait(&sh.cnt[grp][1], rcv + 1) && ok;
                prof.lap(PP_WAIT);
                const double* const q = ba + (rcv & 1) * kXchBA * 64;
                h.w0 = q[0 * 64]; h.w1 = q[1 * 64]; h.w2 = q[2 * 64]; h.al1 = q[3 * 64]; h.al2 = q[4 * 64];
                h.sp = q[5 * 64]; h.cp = q[6 * 64]; h.st = q[7 * 64]; h.cth = q[8 * 64]; h.ss = q[9 * 64];
                h.cs = q[10 * 64]; h.kc0 = q[11 * 64]; h.kc1 = q[12 * 64];
                ++rcv;
                prof.lap(PP_READ);
            };
            prof.lap(PP_BOUNDARY);
            int mode = decide();
            publish(mode);
            recv();
            // pend: the lane's last tick still owes its world-frame position
            // update (step_a does it at the start of the next tick, with the
            // roll / pitch / yaw the partner sent after that tick)
            bool pend = false;
            while (mode != salp::PM_END && ok) {
                const bool ticks = h.ct < h.b2;
                if (mode == salp::PM_FULL) {
                    if (ticks) salp::step_a<salp::PM_FULL>(h, PV, c32, pend);
                } else if (mode == salp::PM_STEADY) {
                    bool settled = true;
                    if (ticks) settled = salp::step_a<salp::PM_STEADY>(h, PV, c32, pend);
                    if (__all(settled)) stage = 2;
                } else {
                    if (ticks) salp::step_a<salp::PM_SETTLED>(h, PV, c32, pend);
                }
                pend = pend || ticks;
                mode = decide();
                prof.lap(PP_TICK);
                publish(mode);
                recv();
            }
            if (pend) salp::a_world(h, PV);
            prof.lap(PP_WORLD);
        }
        prof.lap(PP_BOUNDARY);
        __syncthreads();   // #3: packets done
        prof.lap(PP_BARRIER);
        salp::spill_a(h, ns, P);
        prof.lap(PP_BOUNDARY);
        __syncthreads();   // #4: slots whole again
        prof.lap(PP_BARRIER);
    }
}

template <bool POL, bool SPLIT = false>
__device__ __forceinline__ void pair_wave_b(PairShared& sh, PairJobs* jobs, const RolloutArgs& A, int grp, int lane) {
    const Params& P = A.P;
    const int seat = grp * 64 + lane;
    int s = seat;
    bool pending = false, active = false;
    int64_t steps = 0;
    {   // the A wave loaded the slots; the bookkeeping comes with the re-seat
        const int64_t i = (int64_t)blockIdx.x * kPairEnvs + s;
        if (i < P.n) {
            steps = A.B.steps_done ? A.B.steps_done[i] : 0;
            active = !(A.max_steps > 0 && steps >= A.max_steps);
        }
    }
    __syncthreads();   // #0
    int pub = 0, rcv = 0;
    bool all_done = false;
    PairProf prof;
    prof.start();
    int taken = 0;   // POL: job buffers evaluated
    for (int64_t c = 0;; ++c) {
        const bool last = c == A.n_chunks || all_done;
        if (POL) pair_value_jobs(*jobs, A, grp, s, c, taken);   // while the A wave runs this boundary
        if (last) {
            prof.lap(PP_BOUNDARY);
            prof.flush(1);
            return;
        }
        const int b = (int)(c & 1);
        prof.lap(PP_BOUNDARY);
        __syncthreads();   // #1
        prof.lap(PP_BARRIER);
        pair_reseat(sh, b, seat, s, steps, pending, active, all_done);
        if (all_done) continue;
        const salp::SpillSlot ns{sh.big + s, kPairEnvs};
        const salp::Cache32 c32{sh.cache32 + s, kPairEnvs};
        if constexpr (SPLIT) {
            // the angle chain's state from the slot; the clock decides which
            // wave-ticks this lane ticks, exactly as the A wave's copy does
            const double sct = ns[salp::SP_CT];
            double mx, b1, b2;
            salp::cycle_bounds_of(ns[salp::SP_REFILL], ns[salp::SP_TURN], ns[salp::SP_JET], ns[salp::SP_COAST], &mx, &b1,
                                  &b2);
            if (!active) b2 = -INFINITY;
            salp::Kin k{ns[salp::SP_E], ns[salp::SP_E + 1], ns[salp::SP_E + 2], ns[salp::SP_P], ns[salp::SP_P + 1],
                        ns[salp::SP_P + 2], ns[salp::SP_SP], ns[salp::SP_CP], ns[salp::SP_ST], ns[salp::SP_CTH]};
            double ct = sct;
            prof.lap(PP_BOUNDARY);
            __syncthreads();   // #2
            prof.lap(PP_BARRIER);
            {
                const Params PV = salp::pin_params(P);
                const double2* const ring = reinterpret_cast<const double2*>(sh.big) + grp * kSplitRing * 3 * 64 + lane;
                for (int g = 0;; ++g) {
                    // wait for wave-tick g, or the end of the chunk before it
                    int c = 0;
                    for (int it = 0;; ++it) {
                        c = __builtin_amdgcn_readfirstlane(
                            __hip_atomic_load(&sh.cnt[grp][0], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP));
                        if ((c & ~kSplitEnd) > g || (c & kSplitEnd)) break;
                        if (it >= kPairSpin) {   /* give up: this chunk's results are invalid */
                            if (lane == 0) atomicAdd(&g_pair_timeouts, 1u);
                            c = g | kSplitEnd;
                            break;
                        }
                        __builtin_amdgcn_s_sleep(1);
                    }
                    prof.lap(PP_WAIT);
                    if ((c & ~kSplitEnd) <= g) break;
                    const double2* const q = ring + (g % kSplitRing) * 3 * 64;
                    const double2 x0 = q[0], x1 = q[64], x2 = q[128];
                    pair_publish(&sh.cnt[grp][1], g + 1);   // slot read: the A wave may refill it
                    prof.lap(PP_READ);
                    if (ct < b2) {
                        double r[3];
                        salp::kinematics(k, x0.x, x0.y, x1.x, x1.y, x2.x, x2.y, PV, r);
                        ct += salp::DT;
                    }
                    prof.lap(PP_TICK);
                }
            }
            __syncthreads();   // #3
            prof.lap(PP_BARRIER);
            __syncthreads();   // #3b: the A wave spilled its fields
            prof.lap(PP_BARRIER);
            ns[salp::SP_E] = k.e0; ns[salp::SP_E + 1] = k.e1; ns[salp::SP_E + 2] = k.e2;
            ns[salp::SP_P] = k.p0; ns[salp::SP_P + 1] = k.p1; ns[salp::SP_P + 2] = k.p2;
            ns[salp::SP_SP] = k.sp; ns[salp::SP_CP] = k.cp; ns[salp::SP_ST] = k.st; ns[salp::SP_CTH] = k.cth;
            prof.lap(PP_BOUNDARY);
            __syncthreads();   // #4
            prof.lap(PP_BARRIER);
            continue;
        }
        salp::HotB h;
        salp::unspill_b(h, ns, P);
        if (!active) h.b2 = -INFINITY;
        prof.lap(PP_BOUNDARY);
        __syncthreads();   // #2
        prof.lap(PP_BARRIER);
        {
            const Params PV = salp::pin_params(P);
            double* const ab = sh.big + grp * 2 * kXchAB * 64 + lane;
            double* const ba = sh.big + kXchBase + grp * 2 * kXchBA * 64 + lane;
            const auto publish = [&]() {
                double* const o = ba + (pub & 1) * kXchBA * 64;
                o[0 * 64] = h.w0; o[1 * 64] = h.w1; o[2 * 64] = h.w2; o[3 * 64] = h.al1; o[4 * 64] = h.al2;
                o[5 * 64] = h.sp; o[6 * 64] = h.cp; o[7 * 64] = h.st; o[8 * 64] = h.cth; o[9 * 64] = h.ss;
                o[10 * 64] = h.cs; o[11 * 64] = h.kc0; o[12 * 64] = h.kc1;
                pair_publish(&sh.cnt[grp][1], ++pub);
            };
            // a bound on the ticks of one chunk (A ends it earlier)
            const int64_t cap = 4 + (int64_t)A.chunk + (((int64_t)A.chunk * A.steady_q8) >> 8);
            prof.lap(PP_BOUNDARY);
            publish();
            prof.lap(PP_PUBLISH);
            for (int64_t it = 0; it < cap; ++it) {
                const bool ok = pair_wait(&sh.cnt[grp][0], rcv + 1);
                prof.lap(PP_WAIT);
                const double* const q = ab + (rcv & 1) * kXchAB * 64;
                h.X0 = q[0 * 64]; h.X1 = q[1 * 64]; h.X2 = q[2 * 64]; h.jt1 = q[3 * 64]; h.jt2 = q[4 * 64];
                const int mode = __builtin_amdgcn_readfirstlane(sh.mode[grp][rcv & 1]);
                ++rcv;
                prof.lap(PP_READ);
                if (mode == salp::PM_END || !ok) break;
                if (h.ct < h.b2) {
                    if (mode == salp::PM_FULL) salp::step_b<salp::PM_FULL>(h, PV, c32);
                    else if (mode == salp::PM_STEADY) salp::step_b<salp::PM_STEADY>(h, PV, c32);
                    else salp::step_b<salp::PM_SETTLED>(h, PV, c32);
                }
                prof.lap(PP_TICK);
                publish();
                prof.lap(PP_PUBLISH);
            }
        }
        prof.lap(PP_BOUNDARY);
        __syncthreads();   // #3
        prof.lap(PP_BARRIER);
        salp::spill_b(h, ns);
        prof.lap(PP_BOUNDARY);
        __syncthreads();   // #4
        prof.lap(PP_BARRIER);
    }
}

// The job buffers exist (LDS) in the salp_collect instance only.
template <bool POL>
__device__ __forceinline__ PairJobs* pair_jobs_lds() {
    __shared__ PairJobs j;
    return &j;
}
template <>
__device__ __forceinline__ PairJobs* pair_jobs_lds<false>() { return nullptr; }

template <bool POL>
__global__ __launch_bounds__(kBlock) void k_rollout_pair(RolloutArgs A) {
    __shared__ PairShared sh;
    const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int lane = (int)(threadIdx.x & 63);
    PairJobs* const jobs = pair_jobs_lds<POL>();
    if (POL) {   /* the actor's second layer into LDS, once per workgroup */
        const float* src = (const float*)A.R.weights + SALP_POLICY_PI_W2;
        for (int k = (int)threadIdx.x; k < kPolL2; k += kBlock) jobs->pi_l2[k] = src[k];
        __syncthreads();
    }
    if (wave & 1) pair_wave_b<POL>(sh, jobs, A, wave >> 1, lane);
    else pair_wave_a<POL>(sh, jobs, A, wave >> 1, lane);
}

// k_rollout_split: k_rollout_pair's workgroup with the tick split one way
// (pair_wave_a / pair_wave_b, SPLIT).
template <bool POL>
__global__ __launch_bounds__(kBlock) void k_rollout_split(RolloutArgs A) {
    __shared__ PairShared sh;
    const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int lane = (int)(threadIdx.x & 63);
    PairJobs* const jobs = pair_jobs_lds<POL>();
    if (POL) {   /* the actor's second layer into LDS, once per workgroup */
        const float* src = (const float*)A.R.weights + SALP_POLICY_PI_W2;
        for (int k = (int)threadIdx.x; k < kPolL2; k += kBlock) jobs->pi_l2[k] = src[k];
        __syncthreads();
    }
    if (wave & 1) pair_wave_b<POL, true>(sh, jobs, A, wave >> 1, lane);
    else pair_wave_a<POL, true>(sh, jobs, A, wave >> 1, lane);
}

// The ABI's field-major state (state[f * n + i]) <-> the handle's layout
// (field-major rows + env-major cold block, salp_device.h "state layout").
// One env per lane; the field-major side is coalesced per field.
template <bool TO_HANDLE>
__global__ __launch_bounds__(kBlock) void k_state_copy(double* S, Params P, double* flat) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P.n) return;
    for (int f = 0; f < SALP_NUM_FIELDS; ++f) {
        const size_t a = (size_t)f * (size_t)P.n + (size_t)i;
        if (TO_HANDLE) SF(f) = flat[a];
        else flat[a] = SF(f);
    }
}

// ------------------------------------------------ Robot / Nozzle level
__global__ __launch_bounds__(kBlock) void k_calm(double* S, Params P, int coefficients, int ou) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P.n) return;
    salp::calm_env(S, P, i, coefficients != 0, ou != 0);
}

__global__ __launch_bounds__(kBlock) void k_robot_reset(double* S, Params P, const uint8_t* mask) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P.n || (mask && !mask[i])) return;
    Hot h;
    salp::load_hot(h, S, P, i, false);
    salp::robot_reset(h, S, P, i);
    salp::store_hot(h, S, P, i);
}

__global__ __launch_bounds__(kBlock) void k_nozzle_set_angles(double* S, Params P, const double* ang) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P.n) return;
    (void)salp::nozzle_set_angles(S, P, i, ang[2 * i], ang[2 * i + 1]);
}

__global__ __launch_bounds__(kBlock) void k_nozzle_solve(double* S, Params P, const double* yaw,
                                                         int yaw32) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P.n) return;
    salp::nozzle_solve(S, P, i, yaw[i], yaw32 != 0);
}

template <bool RAND>
__global__ __launch_bounds__(kBlock) void k_robot_set_control(double* S, Params P, const double* ctl,
                                                              int c32) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P.n) return;
    Hot h;
    salp::load_hot(h, S, P, i, false);
    salp::set_control<RAND>(h, S, P, i, ctl[4 * i], ctl[4 * i + 1], ctl[4 * i + 2], ctl[4 * i + 3], c32 != 0);
    salp::store_hot(h, S, P, i);
}

template <bool REC, bool RAND>
__global__ __launch_bounds__(kBlock) void k_robot_cycle(double* S, Params P, SalpTraceBuffer T) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P.n) return;
    LANE_CACHE32();
    Hot h;
    salp::load_hot<RAND>(h, S, P, i);
    salp::resume_cycle(h, S, P, i);
    salp::fill_cache32(P, h.c, c32);
    salp::cycle_prologue(h, S, P, i);
    if (REC) run_cycle_recorded<RAND>(h, S, P, c32, T, i);
    else run_cycle<RAND>(h, P, c32);
    SF(SALP_F_PENDING) = 0.0;
    salp::store_hot<RAND>(h, S, P, i);
}

// Diagnostic: n_ticks physics ticks on every lane with no env-step boundaries
// (cycles simply run on in REST), to time the tick body alone.
__global__ __launch_bounds__(kBlock) void k_tick_bench(double* S, Params P, int32_t n_ticks) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P.n) return;
    LANE_CACHE32();
    Hot h;
    salp::load_hot(h, S, P, i);
    salp::resume_cycle(h, S, P, i);
    salp::fill_cache32(P, h.c, c32);
    const Params PV = salp::pin_params(P);
    for (int32_t k = 0; k < n_ticks; ++k) salp::tick<false, false>(h, PV, c32);
    salp::store_hot(h, S, P, i);
}

__global__ void k_math_selftest(const double* x, const double* y, int64_t n, double* out) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
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
    out[11 * n + i] = salp::qdiv(x[i], salp::rcp_of(y[i]));   /* the tick's shared-reciprocal division */
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

const char* const kFieldNames[SALP_NUM_FIELDS] = {
    "v0", "v1", "v2", "w0", "w1", "w2", "acc0", "acc1", "acc2", "alpha0", "alpha1", "alpha2",
    "eta0", "eta1", "eta2", "pw0", "pw1", "pw2", "pos0", "pos1", "pos2", "ang0", "ang1", "ang2",
    "ppos0", "ppos1", "ppos2", "pang0", "pang1", "pang2", "avgv0", "avgv1", "avgv2",
    "avgw0", "avgw1", "avgw2",
    "length", "width", "volume", "prev_volume", "com", "com_rate", "com_acc",
    "prev_I0", "prev_I1", "prev_I2", "geom32", "pvol32",
    "cycle_time", "time", "refill_time", "jet_time", "coast_time", "contraction",
    "contract_rate", "release_rate", "phase", "cycle", "contr32",
    "angle1", "angle2", "prev_angle1", "prev_angle2", "yaw", "prev_yaw", "turn_time",
    "target0", "target1", "obst0", "obst1", "obst2", "obst3", "obst4", "obst5", "obst6", "obst7",
    "n_obst", "prev_dist", "prev_a2",
    "ep_len", "ep_return", "path_len", "last_px", "last_py", "sum_a0", "sum_a1", "sum_abs_a2",
    "sum_vel", "init_dist", "sum_r0", "sum_r1", "sum_r2", "sum_r3", "sum_r4", "sum_r5", "sum_r6",
    "act0", "act1", "act2", "pending", "step_count", "episode",
    "cd", "dfr", "dtr", "amf0", "amf1", "amf2", "amrf0", "amrf1", "amrf2",
    "amt0", "amt1", "amt2", "amrt0", "amrt1", "amrt2",
    "ouf0", "ouf1", "ouf2", "out0", "out1", "out2", "rng_ctl", "rng_tick"};

thread_local std::string g_last_error;

}  // namespace

struct SalpEnv {
    int device = 0;
    int64_t n = 0;
    SalpParams params{};
    Params dp{};
    double* state = nullptr;
    SalpTraceBuffer trace{};   // max_samples 0: not recording
    std::string err;
    // lock-step launch order (salp_sort.hip): -1 auto, 0 env order, 1 sorted
    int order_mode = -1;
    uint32_t *sort_keys = nullptr, *sort_keys_out = nullptr;
    int32_t *sort_ids = nullptr, *sort_order = nullptr;
    void* sort_temp = nullptr;
    size_t sort_temp_bytes = 0;
    int64_t* step_counts = nullptr;   // per-env env-step counter of a chained salp_step_random
    int rollout_kernel = -1;          // salp_set_rollout_kernel: -1 auto, 0 k_rollout, 1 k_rollout_pair, 2 k_rollout_split
    int step_kernel = -1;             // salp_set_step_kernel: -1 auto, 0 k_step, 1 k_step_wave
    int cu_count = 256;               // compute units of the device (the auto choice)
};

namespace {

int fail(SalpEnv* h, int code, const std::string& msg) {
    if (h) h->err = msg;
    g_last_error = msg;
    return code;
}

int check_hip(SalpEnv* h, hipError_t e, const char* what) {
    if (e == hipSuccess) return SALP_OK;
    return fail(h, SALP_EHIP, std::string(what) + ": " + hipGetErrorString(e));
}

int launched(SalpEnv* h, const char* what) { return check_hip(h, hipGetLastError(), what); }

unsigned blocks_for(int64_t n) { return (unsigned)((n + kBlock - 1) / kBlock); }

// k_rollout's steady ticks per full tick of a wave's chunk budget (x256): a
// steady tick costs ~0.8 of a full one in the round-2 kernel (q = 360,
// profiles/r2_experiments.md r2l-r2o); with the fused arithmetic and settled
// ticks ~0.65 (q = 480 best of 360..580, profiles/r3_experiments.md r3f);
// round 5's cheaper settled tick (1 500 vs 3 760 cycles a full one, phase
// profile r5f) moved it to q = 560 (480..900 swept, profiles/r5_experiments.md
// r5g).  SALP_STEADY_Q8 overrides it for tuning runs; it changes throughput only.
int32_t rollout_steady_q8() {
    static const int32_t q = [] {
        const char* e = std::getenv("SALP_STEADY_Q8");
        const long v = e ? std::strtol(e, nullptr, 10) : 0;
        return (int32_t)(v > 0 && v < (1 << 16) ? v : 560);
    }();
    return q;
}
// The same budget for k_rollout_pair, whose steady ticks cost relatively more
// (the per-tick packet exchange is the same for every kind of tick): q = 320 in
// round 4 (32 768 envs, profiles/r4_experiments.md r4h / r4q / r4x); round 5's
// cheaper settled tick: q = 400 (320 / 360 / 400 / 440 / 480 x chunk 96-256,
// collect_bench at 32 768 envs 25.4 -> 26.3-26.7 M at chunk 192,
// profiles/r5_experiments.md r5n-r5o).  SALP_PAIR_STEADY_Q8 overrides it.
int32_t pair_steady_q8() {
    static const int32_t q = [] {
        const char* e = std::getenv("SALP_PAIR_STEADY_Q8");
        const long v = e ? std::strtol(e, nullptr, 10) : 0;
        return (int32_t)(v > 0 && v < (1 << 16) ? v : 400);
    }();
    return q;
}

// salp_collect's steady budget on the pair kernel: the policy's actions make
// other cycles than uniform random ones, and the bench's PPO leg (config 5,
// 32 768 envs, n_steps 256) runs best at q = 340 with 176-tick chunks (16.9 vs
// 16.4 M env-steps/s at round 4's 400 / 192; chunk 160-224 x q 280-440,
// profiles/r5_experiments.md r5aa-r5ac).  SALP_PAIR_COLLECT_Q8 overrides it.
int32_t pair_collect_steady_q8() {
    static const int32_t q = [] {
        const char* e = std::getenv("SALP_PAIR_COLLECT_Q8");
        const long v = e ? std::strtol(e, nullptr, 10) : 0;
        return (int32_t)(v > 0 && v < (1 << 16) ? v : 340);
    }();
    return q;
}

// Any randomisation switch on: launch the RAND instantiation of the kernels.
bool randomized(const Params& d) { return d.rand_dyn || d.rand_dist || d.rand_act || d.rand_obs || d.latency; }

// The chained kernels (salp_rollout, salp_collect, chained salp_step_random):
// k_rollout_pair (two waves per env, salp_pair.h) or k_rollout (one lane per
// env).  Auto: the pair kernel while one env per lane would leave SIMDs
// without a wave (n <= 64 lanes x 4 SIMDs x CUs / 2, e.g. config 5's 32 768
// envs); SALP_ROLLOUT_KERNEL=0/1 overrides the auto choice (A/B runs).
// The pair kernel has no randomised instance.
bool use_pair(const SalpEnv* h) {
    if (randomized(h->dp)) return false;
    if (h->rollout_kernel >= 0) return h->rollout_kernel >= 1;
    static const int forced = [] {
        const char* e = std::getenv("SALP_ROLLOUT_KERNEL");
        return e && (e[0] == '0' || e[0] == '1') ? e[0] - '0' : -1;
    }();
    if (forced >= 0) return forced == 1;
    return h->n <= (int64_t)h->cu_count * 128;
}
unsigned pair_blocks_for(int64_t n) { return (unsigned)((n + kPairEnvs - 1) / kPairEnvs); }
// Of the two-wave kernels: the one-way split (k_rollout_split) in mode 2, the
// Newton <-> Euler pair in mode 1.  The auto choice's two-wave kernel is the
// split (round 6: config 5's collection 27.2-27.9 vs 25.4-25.7 M env-steps/s,
// PPO leg 20.3 vs 19.7 M on one box, profiles/r6_experiments.md r6d);
// SALP_TWO_WAVE_KERNEL=pair selects the pair (A/B runs).
bool use_split(const SalpEnv* h) {
    if (h->rollout_kernel >= 1) return h->rollout_kernel == 2;
    static const bool pair = [] {
        const char* e = std::getenv("SALP_TWO_WAVE_KERNEL");
        return e && e[0] == 'p';
    }();
    return !pair;
}
// k_rollout_split's steady budgets (SALP_SPLIT_STEADY_Q8 / SALP_SPLIT_COLLECT_Q8
// override them): its steady ticks lose the angle chain as its full ones do,
// so k_rollout's ratio (560) is the rollout's; salp_collect's, swept on the
// bench's PPO leg (chunk 128 / 144 / 176 / 208 / 256 x q 340 .. 1100,
// profiles/r6_experiments.md r6g): q = 700 with the 176-tick chunk, PPO leg
// 20.65 M (q 560: 20.30 M; q 900: 20.22 M).
int32_t split_steady_q8() {
    static const int32_t q = [] {
        const char* e = std::getenv("SALP_SPLIT_STEADY_Q8");
        const long v = e ? std::strtol(e, nullptr, 10) : 0;
        return (int32_t)(v > 0 && v < (1 << 16) ? v : 560);
    }();
    return q;
}
int32_t split_collect_steady_q8() {
    static const int32_t q = [] {
        const char* e = std::getenv("SALP_SPLIT_COLLECT_Q8");
        const long v = e ? std::strtol(e, nullptr, 10) : 0;
        return (int32_t)(v > 0 && v < (1 << 16) ? v : 700);
    }();
    return q;
}

// salp_step's kernel: one wave per env (k_step_wave) for small batches - the
// per-env SalpRobotEnv and small vector envs, where a lane per env leaves the
// chip idle and the step is the latency of one cycle - and while not
// recording (the trace is written by k_step<true>); one lane per env above
// kStepWaveMaxEnvs, where the waves would share SIMDs.
constexpr int64_t kStepWaveMaxEnvs = 1024;
bool use_step_wave(const SalpEnv* h) {
    if (h->trace.max_samples > 0 || h->n > (int64_t)UINT32_MAX) return false;
    if (h->step_kernel == 0 || h->step_kernel == 1) return h->step_kernel == 1;
    return h->n <= kStepWaveMaxEnvs;
}

// One chained launch on the kernel use_pair chooses.
int launch_chained(SalpEnv* h, const RolloutArgs& args, bool pol, hipStream_t st, const char* what) {
    if (use_pair(h)) {
        RolloutArgs pa = args;
        if (use_split(h)) {
            pa.steady_q8 = pol ? split_collect_steady_q8() : split_steady_q8();
            hipLaunchKernelGGL(pol ? k_rollout_split<true> : k_rollout_split<false>, dim3(pair_blocks_for(h->n)),
                               dim3(kBlock), 0, st, pa);
            return launched(h, what);
        }
        pa.steady_q8 = pol ? pair_collect_steady_q8() : pair_steady_q8();
        hipLaunchKernelGGL(pol ? k_rollout_pair<true> : k_rollout_pair<false>, dim3(pair_blocks_for(h->n)),
                           dim3(kBlock), 0, st, pa);
    } else if (pol) {
        hipLaunchKernelGGL((randomized(h->dp) ? k_rollout<true, true> : k_rollout<false, true>),
                           dim3(blocks_for(h->n)), dim3(kBlock), 0, st, args);
    } else {
        hipLaunchKernelGGL((randomized(h->dp) ? k_rollout<true, false> : k_rollout<false, false>),
                           dim3(blocks_for(h->n)), dim3(kBlock), 0, st, args);
    }
    return launched(h, what);
}

// Launch-invariant constants; the same IEEE expressions as the oracle.
Params derive(const SalpParams& p, int64_t n, uint64_t seed, int64_t offset) {
    Params d{};
    const double PI = salp::PI;
    d.L0 = p.init_length; d.W0 = p.init_width; d.maxc = p.max_contraction;
    d.sk = sm_poly();
    d.dry_mass = p.dry_mass; d.nozzle_mass = p.nozzle_mass; d.density = p.density;
    d.nozzle_area = p.nozzle_area;
    d.mid_x = -(p.nozzle_length1 + p.nozzle_length2);
    d.tube_volume = PI * (0.029 * 0.029) * 0.15;
    d.tube_volume_I = 3.14159265358979 * (0.029 * 0.029) * 0.15;
    d.net_tube_mass = salp::TUBE_MASS - d.tube_volume_I * 1000.0;
    d.com_mass_sum = salp::TUBE_MASS + p.nozzle_mass + salp::BUOY_MASS + salp::SKIN_MASS;
    d.P1000tv = 1000.0 * d.tube_volume;
    d.init_aspect = p.init_length / p.init_width;
    double cl = p.init_length - p.max_contraction;
    double cw = p.init_length - cl + p.init_width;
    d.end_aspect = cl / cw;
    d.aspect_den = d.init_aspect - d.end_aspect;
    d.angle_speed = 31 * PI / 30;
    d.obstacle_radius = p.obstacle_radius;
    const double scale = 200.0, margin = 50;
    d.x_min = (-p.width / 2.0 + margin) / scale;
    d.x_max = (p.width / 2.0 - margin) / scale;
    d.y_min = (-p.height / 2.0 + margin) / scale;
    d.y_max = (p.height / 2.0 - margin) / scale;
    d.sep = 2 * p.obstacle_radius + 0.1;
    d.init_angle1 = p.init_angle1; d.init_angle2 = p.init_angle2;
    d.num_obstacles = p.num_obstacles;
    d.max_cycles = p.max_cycles;
    d.obs_dim = 6 + 2 * p.num_obstacles;
    d.rand_dyn = p.dynamics_randomization != 0;
    d.rand_dist = p.disturbances != 0;
    d.rand_act = p.action_randomization != 0;
    d.rand_obs = p.observation_randomization != 0;
    d.latency = p.latency != 0;
    d.n = n;
    d.cold_off = salp::layout_cold_off(n);
    d.env_offset = offset;
    d.seed = seed;
    return d;
}

}  // namespace

extern "C" __attribute__((visibility("hidden"))) hipError_t salp_ppo_loss_launch(
    int64_t B, const float* mu, const float* log_std, const float* value, const float* actions,
    const float* old_logp, const float* adv, const float* returns, double clip_range, double ent_coef,
    double vf_coef, int normalize_advantage, double* workspace, float* out, float* dmu, float* dvalue,
    void* stream);

extern "C" __attribute__((visibility("hidden"))) int64_t salp_ppo_mlp_params_impl(int obs_dim);
extern "C" __attribute__((visibility("hidden"))) int64_t salp_ppo_mlp_offset_impl(int obs_dim, int tensor);
extern "C" __attribute__((visibility("hidden"))) int64_t salp_ppo_mlp_workspace_impl(int64_t batch, int obs_dim);
extern "C" __attribute__((visibility("hidden"))) hipError_t salp_ppo_mlp_adv_partials_launch(
    int64_t B, int64_t n_mb, const int64_t* idx, const float* adv, double* out, void* stream);
extern "C" __attribute__((visibility("hidden"))) hipError_t salp_ppo_mlp_grads_launch(const SalpPpoMinibatch* m,
                                                                                       void* stream);
extern "C" __attribute__((visibility("hidden"))) hipError_t salp_ppo_mlp_apply_launch(const SalpPpoAdam* a,
                                                                                       void* stream);

extern "C" __attribute__((visibility("hidden"))) hipError_t salp_lstm_fwd_launch(
    int64_t m, int H, const float* G, const float* GX, const float* c_prev, const float* keep, const float* keep_next,
    float* h, float* c, float* act, float* hk, void* stream);
extern "C" __attribute__((visibility("hidden"))) hipError_t salp_lstm_bwd_launch(
    int64_t m, int H, const float* act, const float* c_prev, const float* keep, const float* c, const float* dh,
    const float* dhk_next, const float* keep_next, const float* dc, float* dG, float* dc_prev, void* stream);

extern "C" __attribute__((visibility("hidden"))) hipError_t salp_sort_temp_bytes(int64_t n, size_t* bytes);
extern "C" __attribute__((visibility("hidden"))) hipError_t salp_sort_launch(
    void* temp, size_t temp_bytes, const uint32_t* keys_in, uint32_t* keys_out, const int32_t* ids_in,
    int32_t* order, int64_t n, void* stream);

extern "C" __attribute__((visibility("hidden"))) hipError_t salp_gae_launch(
    int64_t n_steps, int64_t n_envs, const float* rewards, const float* values, const float* episode_starts,
    const float* last_values, const float* last_dones, double gamma, double gae_lambda, float* advantages,
    float* returns, void* stream);

extern "C" {

int salp_abi_version(void) { return SALP_ABI_VERSION; }

void salp_default_params(SalpParams* p) {
    std::memset(p, 0, sizeof *p);
    p->nozzle_length1 = 0.05; p->nozzle_length2 = 0.05; p->nozzle_length3 = 0.05;
    p->nozzle_area = 0.00016; p->nozzle_mass = 1.0;
    p->dry_mass = 1.0; p->init_length = 0.3; p->init_width = 0.15; p->max_contraction = 0.06;
    p->density = 1000.0; p->init_angle1 = 0.0; p->init_angle2 = 0.0;
    p->obstacle_radius = 0.2; p->width = 900; p->height = 700; p->num_obstacles = 2;
    p->max_cycles = 500;
}

int salp_create(const SalpParams* p, int64_t n_envs, uint64_t seed, int64_t env_id_offset,
                int device, SalpEnv** out) {
    if (!p || !out) return fail(nullptr, SALP_EINVAL, "salp_create: null argument");
    *out = nullptr;
    if (n_envs <= 0) return fail(nullptr, SALP_EINVAL, "salp_create: n_envs must be positive");
    if (p->num_obstacles < 0 || p->num_obstacles > SALP_MAX_OBSTACLES)
        return fail(nullptr, SALP_EINVAL, "salp_create: num_obstacles must be in [0, 4]");
    if (!(p->init_length > 0) || !(p->init_width > 0) || !(p->nozzle_area > 0))
        return fail(nullptr, SALP_EINVAL, "salp_create: non-positive body dimensions");
    auto* h = new SalpEnv();
    h->device = device;
    h->n = n_envs;
    h->params = *p;
    h->dp = derive(*p, n_envs, seed, env_id_offset);
    int rc = check_hip(nullptr, hipSetDevice(device), "hipSetDevice");
    if (rc) { delete h; return rc; }
    {
        int cus = 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess && cus > 0)
            h->cu_count = cus;
    }
    rc = check_hip(nullptr, hipMalloc(&h->state, sizeof(double) * (size_t)salp::layout_doubles(n_envs)),
                   "hipMalloc(state)");
    if (rc) { delete h; return SALP_ENOMEM; }
    {   // lock-step ordering buffers (small: 16 B per env + the sort's scratch)
        size_t tb = 0;
        rc = check_hip(nullptr, salp_sort_temp_bytes(n_envs, &tb), "salp_sort_temp_bytes");
        if (!rc) rc = check_hip(nullptr, hipMalloc(&h->sort_keys, sizeof(uint32_t) * n_envs), "hipMalloc(sort)");
        if (!rc) rc = check_hip(nullptr, hipMalloc(&h->sort_keys_out, sizeof(uint32_t) * n_envs), "hipMalloc(sort)");
        if (!rc) rc = check_hip(nullptr, hipMalloc(&h->sort_ids, sizeof(int32_t) * n_envs), "hipMalloc(sort)");
        if (!rc) rc = check_hip(nullptr, hipMalloc(&h->sort_order, sizeof(int32_t) * n_envs), "hipMalloc(sort)");
        if (!rc) rc = check_hip(nullptr, hipMalloc(&h->sort_temp, tb > 0 ? tb : 1), "hipMalloc(sort)");
        if (!rc) rc = check_hip(nullptr, hipMalloc(&h->step_counts, sizeof(int64_t) * n_envs), "hipMalloc(steps)");
        h->sort_temp_bytes = tb;
        if (rc) { g_last_error = h->err.empty() ? g_last_error : h->err; salp_destroy(h); return SALP_ENOMEM; }
    }
    hipLaunchKernelGGL(k_construct, dim3(blocks_for(n_envs)), dim3(kBlock), 0, nullptr, h->state, h->dp);
    if ((rc = launched(h, "k_construct"))) { g_last_error = h->err; salp_destroy(h); return rc; }
    // SalpRobotEnv.__init__ ends with self.reset() (src/salp_robot_env.py:112)
    hipLaunchKernelGGL(k_reset, dim3(blocks_for(n_envs)), dim3(kBlock), 0, nullptr, h->state, h->dp,
                       (const uint8_t*)nullptr, (float*)nullptr);
    if ((rc = launched(h, "k_reset"))) { g_last_error = h->err; salp_destroy(h); return rc; }
    if ((rc = check_hip(h, hipDeviceSynchronize(), "salp_create sync"))) {
        g_last_error = h->err; salp_destroy(h); return rc;
    }
    *out = h;
    return SALP_OK;
}

int salp_destroy(SalpEnv* h) {
    if (!h) return SALP_OK;
    (void)hipSetDevice(h->device);
    for (void* p : {(void*)h->state, (void*)h->sort_keys, (void*)h->sort_keys_out, (void*)h->sort_ids,
                    (void*)h->sort_order, h->sort_temp, (void*)h->step_counts})
        if (p) (void)hipFree(p);
    delete h;
    return SALP_OK;
}

const char* salp_last_error(const SalpEnv* h) {
    return h ? h->err.c_str() : g_last_error.c_str();
}

int64_t salp_num_envs(const SalpEnv* h) { return h ? h->n : -1; }
int salp_obs_dim(const SalpEnv* h) { return h ? h->dp.obs_dim : -1; }
int salp_num_fields(void) { return SALP_NUM_FIELDS; }
int salp_trace_dim(void) { return SALP_TRACE_DIM; }
const char* salp_field_name(int f) {
    return (f >= 0 && f < SALP_NUM_FIELDS) ? kFieldNames[f] : nullptr;
}

int salp_reset(SalpEnv* h, const uint8_t* mask, float* obs_out, void* stream) {
    if (!h) return fail(nullptr, SALP_EINVAL, "salp_reset: null handle");
    hipLaunchKernelGGL(k_reset, dim3(blocks_for(h->n)), dim3(kBlock), 0, (hipStream_t)stream,
                       h->state, h->dp, mask, obs_out);
    return launched(h, "k_reset");
}

int salp_reset_to(SalpEnv* h, const uint8_t* mask, const float* targets, const float* obstacles,
                  const int32_t* n_obstacles, float* obs_out, void* stream) {
    if (!h) return fail(nullptr, SALP_EINVAL, "salp_reset_to: null handle");
    if (!targets || !obstacles || !n_obstacles)
        return fail(h, SALP_EINVAL, "salp_reset_to: targets, obstacles and n_obstacles are required");
    hipLaunchKernelGGL(k_reset_to, dim3(blocks_for(h->n)), dim3(kBlock), 0, (hipStream_t)stream,
                       h->state, h->dp, mask, targets, obstacles, n_obstacles, obs_out);
    return launched(h, "k_reset_to");
}

// The launch order of a lock-step call: nullptr (env order) or the sorted
// permutation, computed on `stream` ahead of the step kernel.
static const int32_t* lockstep_order(SalpEnv* h, const float* actions, int32_t n_steps, void* stream, int* rc) {
    *rc = SALP_OK;
    // auto: sorted from a few waves on (measured: +10 % with every wave
    // resident, 1.8x at two waves per SIMD; profiles/r2_experiments.md r2e)
    const bool sort = h->order_mode == 1 || (h->order_mode == -1 && h->n >= kSortMinEnvs);
    if (!sort) return nullptr;
    hipLaunchKernelGGL(k_predict_ticks, dim3(blocks_for(h->n)), dim3(kBlock), 0, (hipStream_t)stream, h->state,
                       h->dp, actions, n_steps, h->sort_keys, h->sort_ids);
    if ((*rc = launched(h, "k_predict_ticks"))) return nullptr;
    *rc = check_hip(h, salp_sort_launch(h->sort_temp, h->sort_temp_bytes, h->sort_keys, h->sort_keys_out,
                                        h->sort_ids, h->sort_order, h->n, stream),
                    "lock-step order sort");
    return *rc ? nullptr : h->sort_order;
}

int salp_step(SalpEnv* h, const float* actions, float* obs_out, double* reward_out,
              uint8_t* terminated_out, uint8_t* truncated_out, int auto_reset,
              float* terminal_obs_out, double* info_out, void* stream) {
    if (!h) return fail(nullptr, SALP_EINVAL, "salp_step: null handle");
    if (!actions) return fail(h, SALP_EINVAL, "salp_step: actions is required");
    if (use_step_wave(h)) {
        hipLaunchKernelGGL(randomized(h->dp) ? k_step_wave<true> : k_step_wave<false>, dim3((unsigned)h->n),
                           dim3(2 * kWave), 0, (hipStream_t)stream, h->state, h->dp, actions, obs_out, reward_out,
                           terminated_out, truncated_out, auto_reset, terminal_obs_out, info_out);
        return launched(h, "k_step_wave");
    }
    auto kern = h->trace.max_samples > 0 ? (randomized(h->dp) ? k_step<true, true> : k_step<true, false>)
                                         : (randomized(h->dp) ? k_step<false, true> : k_step<false, false>);
    int rc;
    const int32_t* order = lockstep_order(h, actions, 1, stream, &rc);
    if (rc) return rc;
    hipLaunchKernelGGL(kern, dim3(blocks_for(h->n)), dim3(kBlock), 0, (hipStream_t)stream, h->state, h->dp,
                       actions, obs_out, reward_out, terminated_out, truncated_out, auto_reset, terminal_obs_out,
                       info_out, h->trace, order);
    return launched(h, "k_step");
}

// salp_step_random with n_steps >= kChainedMinSteps runs on the chained kernel:
// every env does its n_steps env-steps back to back and stops (max_steps),
// instead of the whole wave waiting for its slowest cycle at every env-step.
// Same per-env results (the actions are keyed by env id and step index either
// way).  The chained launch lasts as long as the workgroup whose slowest env
// has the longest sum of n_steps cycles, so it only pays for long calls
// (65 536 envs, M env-steps/s lock-step / chained: k 4 32.0 / 27.1, k 16
// 34.9 / 34.8, k 32 35.2 / 37.2; profiles/r2_experiments.md r2q).
// SALP_STEP_RANDOM_LOCKSTEP=1 keeps the lock-step kernel for every n_steps.
constexpr int32_t kChainedMinSteps = 32;
static bool step_random_chained(int32_t n_steps) {
    static const bool lock = [] {
        const char* e = std::getenv("SALP_STEP_RANDOM_LOCKSTEP");
        return e && e[0] == '1';
    }();
    return n_steps >= kChainedMinSteps && !lock;
}

int salp_step_random(SalpEnv* h, int32_t n_steps, double* reward_sum_out, void* stream) {
    if (!h) return fail(nullptr, SALP_EINVAL, "salp_step_random: null handle");
    if (n_steps < 0) return fail(h, SALP_EINVAL, "salp_step_random: n_steps < 0");
    int rc;
    if (step_random_chained(n_steps)) {
        hipStream_t st = (hipStream_t)stream;
        rc = check_hip(h, hipMemsetAsync(h->step_counts, 0, sizeof(int64_t) * h->n, st), "salp_step_random memset");
        if (!rc && reward_sum_out)
            rc = check_hip(h, hipMemsetAsync(reward_sum_out, 0, sizeof(double) * h->n, st), "salp_step_random memset");
        if (rc) return rc;
        SalpRolloutBuffers b{};
        b.steps_done = h->step_counts;
        b.max_steps = n_steps;
        static const int32_t chunk = [] {   // SALP_STEP_RANDOM_CHUNK: tuning runs only
            const char* e = std::getenv("SALP_STEP_RANDOM_CHUNK");
            const long v = e ? std::strtol(e, nullptr, 10) : 0;
            return (int32_t)(v > 0 && v < 4096 ? v : 64);
        }();
        // bound: n_steps cycles of the longest legitimate length (the lock-step guard)
        const int64_t n_chunks = ((int64_t)n_steps * kMaxTicksPerCycle + chunk - 1) / chunk;
        RolloutArgs args{h->state, h->dp, n_chunks, chunk, rollout_steady_q8(), n_steps, b, reward_sum_out, 1, 0};
        return launch_chained(h, args, false, st, "k_rollout(step_random)");
    }
    const int32_t* order = lockstep_order(h, nullptr, n_steps, stream, &rc);
    if (rc) return rc;
    hipLaunchKernelGGL(randomized(h->dp) ? k_step_random<true> : k_step_random<false>, dim3(blocks_for(h->n)),
                       dim3(kBlock), 0, (hipStream_t)stream, h->state, h->dp, n_steps, reward_sum_out, order);
    return launched(h, "k_step_random");
}

int salp_rollout(SalpEnv* h, int64_t tick_budget, const SalpRolloutBuffers* buf, void* stream) {
    if (!h) return fail(nullptr, SALP_EINVAL, "salp_rollout: null handle");
    if (tick_budget < 0) return fail(h, SALP_EINVAL, "salp_rollout: tick_budget < 0");
    SalpRolloutBuffers b{};
    if (buf) b = *buf;
    if (b.capacity < 0) return fail(h, SALP_EINVAL, "salp_rollout: capacity < 0");
    // chunk 64 with q = 560 (round 5: the cheaper settled tick made shorter
    // chunks pay; 48 / 64 / 80 / 96 / 112 / 128 swept, profiles/r5_experiments.md r5j-r5k)
    int32_t chunk = b.chunk > 0 ? b.chunk : 64;
    int64_t n_chunks = (tick_budget + chunk - 1) / chunk;
    RolloutArgs args{h->state, h->dp, n_chunks, chunk, rollout_steady_q8(), b.max_steps, b, nullptr, 0, 0};
    return launch_chained(h, args, false, (hipStream_t)stream, "k_rollout");
}

int salp_collect(SalpEnv* h, const SalpPolicyRollout* r, void* stream) {
    if (!h) return fail(nullptr, SALP_EINVAL, "salp_collect: null handle");
    if (!r || !r->weights || r->n_steps <= 0)
        return fail(h, SALP_EINVAL, "salp_collect: weights and n_steps > 0 are required");
    if (!r->obs || !r->actions || !r->rewards || !r->episode_starts || !r->values || !r->log_probs ||
        !r->episode_start || !r->last_obs || !r->ep_stats || !r->diverged)
        return fail(h, SALP_EINVAL, "salp_collect: every buffer is required");
    if (r->n_steps > (int64_t)1 << 24) return fail(h, SALP_EINVAL, "salp_collect: n_steps too large");
    hipStream_t st = (hipStream_t)stream;
    int rc = check_hip(h, hipMemsetAsync(h->step_counts, 0, sizeof(int64_t) * h->n, st), "salp_collect memset");
    if (rc) return rc;
    SalpRolloutBuffers b{};
    b.steps_done = h->step_counts;
    b.max_steps = r->n_steps;
    // Longer chunks than the rollout's 64: every wave evaluates the policy at
    // most once per chunk, and that evaluation is on its critical path
    // (k_rollout, 65 536 envs, M env-steps/s by chunk 128 / 192 / 256 / 384 /
    // 512 / 768: 26.3 / 28.3 / 28.3 / 29.2 / 28.6 / 24.6; profiles/
    // r2_experiments.md r2x).  k_rollout_pair, whose B wave takes the value
    // network off the A wave's boundary: 192 (32 768 envs, chunk 96 / 128 / 160
    // / 192 / 224 / 256 / 384: 20.2 / 21.3 / 21.5 / 21.9 / 21.6 / 21.2 / 20.9;
    // profiles/r4_experiments.md r4x); round 5: 176 with q = 340
    // (pair_collect_steady_q8).  SALP_COLLECT_CHUNK overrides both.
    static const int32_t forced_chunk = [] {
        const char* e = std::getenv("SALP_COLLECT_CHUNK");
        const long v = e ? std::strtol(e, nullptr, 10) : 0;
        return (int32_t)(v > 0 && v < 4096 ? v : 0);
    }();
    const int32_t chunk = forced_chunk ? forced_chunk : use_pair(h) ? 176 : 384;
    const int64_t n_chunks = (r->n_steps * kMaxTicksPerCycle + chunk - 1) / chunk;
    RolloutArgs args{h->state, h->dp, n_chunks, chunk, rollout_steady_q8(), r->n_steps, b, nullptr, 1, 0, *r};
    return launch_chained(h, args, true, st, "k_rollout(collect)");
}

int salp_robot_reset(SalpEnv* h, const uint8_t* mask, void* stream) {
    if (!h) return fail(nullptr, SALP_EINVAL, "salp_robot_reset: null handle");
    hipLaunchKernelGGL(k_robot_reset, dim3(blocks_for(h->n)), dim3(kBlock), 0, (hipStream_t)stream,
                       h->state, h->dp, mask);
    return launched(h, "k_robot_reset");
}

int salp_nozzle_set_angles(SalpEnv* h, const double* angles, void* stream) {
    if (!h) return fail(nullptr, SALP_EINVAL, "salp_nozzle_set_angles: null handle");
    if (!angles) return fail(h, SALP_EINVAL, "salp_nozzle_set_angles: angles is required");
    hipLaunchKernelGGL(k_nozzle_set_angles, dim3(blocks_for(h->n)), dim3(kBlock), 0, (hipStream_t)stream,
                       h->state, h->dp, angles);
    return launched(h, "k_nozzle_set_angles");
}

int salp_nozzle_solve(SalpEnv* h, const double* yaw, int yaw_is_f32, void* stream) {
    if (!h) return fail(nullptr, SALP_EINVAL, "salp_nozzle_solve: null handle");
    if (!yaw) return fail(h, SALP_EINVAL, "salp_nozzle_solve: yaw is required");
    hipLaunchKernelGGL(k_nozzle_solve, dim3(blocks_for(h->n)), dim3(kBlock), 0, (hipStream_t)stream,
                       h->state, h->dp, yaw, yaw_is_f32);
    return launched(h, "k_nozzle_solve");
}

int salp_robot_set_control(SalpEnv* h, const double* control, int contraction_is_f32, void* stream) {
    if (!h) return fail(nullptr, SALP_EINVAL, "salp_robot_set_control: null handle");
    if (!control) return fail(h, SALP_EINVAL, "salp_robot_set_control: control is required");
    hipLaunchKernelGGL(randomized(h->dp) ? k_robot_set_control<true> : k_robot_set_control<false>,
                       dim3(blocks_for(h->n)), dim3(kBlock), 0, (hipStream_t)stream, h->state, h->dp, control,
                       contraction_is_f32);
    return launched(h, "k_robot_set_control");
}

int salp_robot_step_through_cycle(SalpEnv* h, void* stream) {
    if (!h) return fail(nullptr, SALP_EINVAL, "salp_robot_step_through_cycle: null handle");
    auto kern = h->trace.max_samples > 0
                    ? (randomized(h->dp) ? k_robot_cycle<true, true> : k_robot_cycle<true, false>)
                    : (randomized(h->dp) ? k_robot_cycle<false, true> : k_robot_cycle<false, false>);
    hipLaunchKernelGGL(kern, dim3(blocks_for(h->n)), dim3(kBlock), 0, (hipStream_t)stream, h->state, h->dp,
                       h->trace);
    return launched(h, "k_robot_cycle");
}

int salp_set_lockstep_order(SalpEnv* h, int mode) {
    if (!h) return fail(nullptr, SALP_EINVAL, "salp_set_lockstep_order: null handle");
    if (mode < -1 || mode > 1) return fail(h, SALP_EINVAL, "salp_set_lockstep_order: mode must be -1, 0 or 1");
    h->order_mode = mode;
    return SALP_OK;
}

#if SALP_ROLLOUT_PROF
// experiment builds only (not in include/salp.h): read and clear g_roll_prof
int salp_debug_rollout_prof(unsigned long long* out) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_roll_prof), sizeof(g_roll_prof)) != hipSuccess) return -1;
    static const unsigned long long zero[2][RP_N] = {};
    return hipMemcpyToSymbol(HIP_SYMBOL(g_roll_prof), zero, sizeof zero) == hipSuccess ? 0 : -1;
}
#endif

#if SALP_PAIR_PROF
// experiment builds only (not in include/salp.h): read and clear g_pair_prof
int salp_debug_pair_prof(unsigned long long* out) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_pair_prof), sizeof(g_pair_prof)) != hipSuccess) return -1;
    static const unsigned long long zero[2][PP_N] = {};
    return hipMemcpyToSymbol(HIP_SYMBOL(g_pair_prof), zero, sizeof zero) == hipSuccess ? 0 : -1;
}
#endif

int salp_pair_timeouts(SalpEnv* h, uint64_t* count_out, void* stream) {
    if (!h || !count_out) return fail(h, SALP_EINVAL, "salp_pair_timeouts: null argument");
    unsigned int c = 0;
    const hipStream_t s = (hipStream_t)stream;
    hipError_t e = hipMemcpyFromSymbolAsync(&c, HIP_SYMBOL(g_pair_timeouts), sizeof c, 0, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    static const unsigned int zero = 0;
    if (e == hipSuccess && c != 0) e = hipMemcpyToSymbolAsync(HIP_SYMBOL(g_pair_timeouts), &zero, sizeof zero, 0,
                                                               hipMemcpyHostToDevice, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    *count_out = c;
    return check_hip(h, e, "salp_pair_timeouts");
}

int salp_set_step_kernel(SalpEnv* h, int mode) {
    if (!h) return fail(nullptr, SALP_EINVAL, "salp_set_step_kernel: null handle");
    if (mode < -1 || mode > 1) return fail(h, SALP_EINVAL, "salp_set_step_kernel: mode must be -1, 0 or 1");
    h->step_kernel = mode;
    return SALP_OK;
}

int salp_set_rollout_kernel(SalpEnv* h, int mode) {
    if (!h) return fail(nullptr, SALP_EINVAL, "salp_set_rollout_kernel: null handle");
    if (mode < -1 || mode > 2) return fail(h, SALP_EINVAL, "salp_set_rollout_kernel: mode must be -1, 0, 1 or 2");
    h->rollout_kernel = mode;
    return SALP_OK;
}

int salp_set_trace(SalpEnv* h, const SalpTraceBuffer* buf) {
    if (!h) return fail(nullptr, SALP_EINVAL, "salp_set_trace: null handle");
    if (!buf || buf->max_samples <= 0) {
        h->trace = SalpTraceBuffer{};
        return SALP_OK;
    }
    if (!buf->rows || !buf->n_samples)
        return fail(h, SALP_EINVAL, "salp_set_trace: rows and n_samples are required");
    h->trace = *buf;
    return SALP_OK;
}

int salp_set_randomization(SalpEnv* h, int dynamics, int disturbances, int actions, int observations,
                           int latency) {
    if (!h) return fail(nullptr, SALP_EINVAL, "salp_set_randomization: null handle");
    // a feature switched off leaves the reference's defaults behind: mean
    // coefficients, calm disturbance processes (what the plain kernels assume)
    const bool calm_coef = h->dp.rand_dyn && !dynamics, calm_ou = h->dp.rand_dist && !disturbances;
    if (calm_coef || calm_ou) {
        hipLaunchKernelGGL(k_calm, dim3(blocks_for(h->n)), dim3(kBlock), 0, nullptr, h->state, h->dp,
                           (int)calm_coef, (int)calm_ou);
        int rc = launched(h, "k_calm");
        if (rc) return rc;
        if ((rc = check_hip(h, hipDeviceSynchronize(), "salp_set_randomization sync"))) return rc;
    }
    h->params.dynamics_randomization = h->dp.rand_dyn = dynamics != 0;
    h->params.disturbances = h->dp.rand_dist = disturbances != 0;
    h->params.action_randomization = h->dp.rand_act = actions != 0;
    h->params.observation_randomization = h->dp.rand_obs = observations != 0;
    h->params.latency = h->dp.latency = latency != 0;
    return SALP_OK;
}

int salp_get_state(SalpEnv* h, double* state_out, void* stream) {
    if (!h || !state_out) return fail(h, SALP_EINVAL, "salp_get_state: null argument");
    hipLaunchKernelGGL(k_state_copy<false>, dim3(blocks_for(h->n)), dim3(kBlock), 0, (hipStream_t)stream, h->state,
                       h->dp, state_out);
    return launched(h, "salp_get_state");
}

int salp_set_state(SalpEnv* h, const double* state_in, void* stream) {
    if (!h || !state_in) return fail(h, SALP_EINVAL, "salp_set_state: null argument");
    hipLaunchKernelGGL(k_state_copy<true>, dim3(blocks_for(h->n)), dim3(kBlock), 0, (hipStream_t)stream, h->state,
                       h->dp, const_cast<double*>(state_in));
    return launched(h, "salp_set_state");
}

int salp_math_selftest(const double* x, const double* y, int64_t n, double* out, void* stream) {
    if (!x || !y || !out || n < 0) return fail(nullptr, SALP_EINVAL, "salp_math_selftest: bad argument");
    hipLaunchKernelGGL(k_math_selftest, dim3(blocks_for(n)), dim3(kBlock), 0, (hipStream_t)stream, x, y,
                       n, out);
    return check_hip(nullptr, hipGetLastError(), "k_math_selftest");
}

int salp_bench_ticks(SalpEnv* h, int32_t n_ticks, void* stream) {
    if (!h || n_ticks < 0) return fail(h, SALP_EINVAL, "salp_bench_ticks: bad argument");
    hipLaunchKernelGGL(k_tick_bench, dim3(blocks_for(h->n)), dim3(kBlock), 0, (hipStream_t)stream,
                       h->state, h->dp, n_ticks);
    return launched(h, "k_tick_bench");
}

int64_t salp_state_ptr(SalpEnv* h) { return h ? (int64_t)(intptr_t)h->state : 0; }

int salp_ppo_loss(int64_t batch, const float* mu, const float* log_std, const float* value,
                  const float* actions, const float* old_logp, const float* advantages, const float* returns,
                  double clip_range, double ent_coef, double vf_coef, int normalize_advantage,
                  double* workspace, float* out, float* dmu, float* dvalue, void* stream) {
    if (batch <= 0) return fail(nullptr, SALP_EINVAL, "salp_ppo_loss: batch must be positive");
    if (!mu || !log_std || !value || !actions || !old_logp || !advantages || !returns || !workspace || !out ||
        !dmu || !dvalue)
        return fail(nullptr, SALP_EINVAL, "salp_ppo_loss: null buffer");
    if (!(clip_range >= 0)) return fail(nullptr, SALP_EINVAL, "salp_ppo_loss: clip_range must be >= 0");
    const hipError_t e = salp_ppo_loss_launch(batch, mu, log_std, value, actions, old_logp, advantages, returns,
                                              clip_range, ent_coef, vf_coef, normalize_advantage, workspace, out, dmu,
                                              dvalue, stream);
    return check_hip(nullptr, e, "k_ppo");
}

int64_t salp_ppo_mlp_num_params(int obs_dim) {
    return (obs_dim > 0 && obs_dim <= SALP_OBS_DIM_MAX) ? salp_ppo_mlp_params_impl(obs_dim) : -1;
}
int64_t salp_ppo_mlp_offset(int obs_dim, int tensor) {
    if (obs_dim <= 0 || obs_dim > SALP_OBS_DIM_MAX || tensor < 0 || tensor > SALP_MLP_N_TENSORS) return -1;
    return salp_ppo_mlp_offset_impl(obs_dim, tensor);
}
int64_t salp_ppo_mlp_workspace_doubles(int64_t batch, int obs_dim) {
    if (batch <= 0 || obs_dim <= 0 || obs_dim > SALP_OBS_DIM_MAX) return -1;
    return salp_ppo_mlp_workspace_impl(batch, obs_dim);
}

int salp_ppo_mlp_grads(const SalpPpoMinibatch* m, void* stream) {
    if (!m || m->batch <= 0) return fail(nullptr, SALP_EINVAL, "salp_ppo_mlp_grads: batch must be positive");
    if (m->obs_dim <= 0 || m->obs_dim > SALP_OBS_DIM_MAX)
        return fail(nullptr, SALP_EINVAL, "salp_ppo_mlp_grads: obs_dim out of range");
    if (!m->idx || !m->obs || !m->actions || !m->old_log_prob || !m->advantages || !m->returns || !m->grads ||
        !m->workspace)
        return fail(nullptr, SALP_EINVAL, "salp_ppo_mlp_grads: null buffer");
    for (int t = 0; t < SALP_MLP_N_TENSORS; ++t)
        if (!m->params[t]) return fail(nullptr, SALP_EINVAL, "salp_ppo_mlp_grads: null parameter tensor");
    if (!(m->clip_range >= 0)) return fail(nullptr, SALP_EINVAL, "salp_ppo_mlp_grads: clip_range must be >= 0");
    return check_hip(nullptr, salp_ppo_mlp_grads_launch(m, stream), "k_mlp");
}

int salp_ppo_mlp_adv_partials(int64_t batch, int64_t n_minibatches, const int64_t* idx, const float* advantages,
                              double* out, void* stream) {
    if (batch <= 0 || n_minibatches <= 0 || n_minibatches > 65535)
        return fail(nullptr, SALP_EINVAL, "salp_ppo_mlp_adv_partials: batch > 0 and 0 < n_minibatches <= 65535");
    if (!idx || !advantages || !out) return fail(nullptr, SALP_EINVAL, "salp_ppo_mlp_adv_partials: null buffer");
    return check_hip(nullptr, salp_ppo_mlp_adv_partials_launch(batch, n_minibatches, idx, advantages, out, stream),
                     "k_mlp_adv_sums");
}

int salp_ppo_mlp_apply(const SalpPpoAdam* a, void* stream) {
    if (!a || a->obs_dim <= 0 || a->obs_dim > SALP_OBS_DIM_MAX)
        return fail(nullptr, SALP_EINVAL, "salp_ppo_mlp_apply: obs_dim out of range");
    if (!a->grads || !a->exp_avg || !a->exp_avg_sq || !a->step)
        return fail(nullptr, SALP_EINVAL, "salp_ppo_mlp_apply: null buffer");
    for (int t = 0; t < SALP_MLP_N_TENSORS; ++t)
        if (!a->params[t]) return fail(nullptr, SALP_EINVAL, "salp_ppo_mlp_apply: null parameter tensor");
    return check_hip(nullptr, salp_ppo_mlp_apply_launch(a, stream), "k_mlp_apply");
}

int salp_lstm_cell_forward(int64_t rows, int32_t hidden, const float* gates, const float* c_prev, const float* keep,
                           float* h, float* c, float* act, void* stream) {
    if (rows < 0 || hidden <= 0) return fail(nullptr, SALP_EINVAL, "salp_lstm_cell_forward: bad size");
    if (!gates || !c_prev || !keep || !h || !c || !act)
        return fail(nullptr, SALP_EINVAL, "salp_lstm_cell_forward: null buffer");
    if (rows == 0) return SALP_OK;
    return check_hip(nullptr, salp_lstm_fwd_launch(rows, hidden, gates, nullptr, c_prev, keep, nullptr, h, c, act,
                                                   nullptr, stream), "k_lstm_fwd");
}

int salp_lstm_step_forward(int64_t rows, int32_t hidden, const float* gates, const float* gx, const float* c_prev,
                           const float* keep, const float* keep_next, float* h, float* c, float* act, float* hk_next,
                           void* stream) {
    if (rows < 0 || hidden <= 0) return fail(nullptr, SALP_EINVAL, "salp_lstm_step_forward: bad size");
    if (!gates || !c_prev || !keep || !h || !c || !act)
        return fail(nullptr, SALP_EINVAL, "salp_lstm_step_forward: null buffer");
    if (!keep_next != !hk_next)
        return fail(nullptr, SALP_EINVAL, "salp_lstm_step_forward: keep_next and hk_next go together");
    if (rows == 0) return SALP_OK;
    return check_hip(nullptr, salp_lstm_fwd_launch(rows, hidden, gates, gx, c_prev, keep, keep_next, h, c, act,
                                                   hk_next, stream), "k_lstm_fwd");
}

int salp_lstm_cell_backward(int64_t rows, int32_t hidden, const float* act, const float* c_prev, const float* keep,
                            const float* c, const float* dh, const float* dc, float* dgates, float* dc_prev,
                            void* stream) {
    if (rows < 0 || hidden <= 0) return fail(nullptr, SALP_EINVAL, "salp_lstm_cell_backward: bad size");
    if (!act || !c_prev || !keep || !c || !dh || !dgates || !dc_prev)
        return fail(nullptr, SALP_EINVAL, "salp_lstm_cell_backward: null buffer");
    if (rows == 0) return SALP_OK;
    return check_hip(nullptr, salp_lstm_bwd_launch(rows, hidden, act, c_prev, keep, c, dh, nullptr, nullptr, dc, dgates,
                                                   dc_prev, stream), "k_lstm_bwd");
}

int salp_lstm_step_backward(int64_t rows, int32_t hidden, const float* act, const float* c_prev, const float* keep,
                            const float* c, const float* d_out, const float* dhk_next, const float* keep_next,
                            const float* dc, float* dgates, float* dc_prev, void* stream) {
    if (rows < 0 || hidden <= 0) return fail(nullptr, SALP_EINVAL, "salp_lstm_step_backward: bad size");
    if (!act || !c_prev || !keep || !c || !d_out || !dgates || !dc_prev)
        return fail(nullptr, SALP_EINVAL, "salp_lstm_step_backward: null buffer");
    if (!dhk_next != !keep_next)
        return fail(nullptr, SALP_EINVAL, "salp_lstm_step_backward: dhk_next and keep_next go together");
    if (rows == 0) return SALP_OK;
    return check_hip(nullptr, salp_lstm_bwd_launch(rows, hidden, act, c_prev, keep, c, d_out, dhk_next, keep_next, dc,
                                                   dgates, dc_prev, stream), "k_lstm_bwd");
}

int salp_gae(int64_t n_steps, int64_t n_envs, const float* rewards, const float* values,
             const float* episode_starts, const float* last_values, const float* last_dones, double gamma,
             double gae_lambda, float* advantages, float* returns, void* stream) {
    if (n_steps < 0 || n_envs < 0) return fail(nullptr, SALP_EINVAL, "salp_gae: negative size");
    if (!rewards || !values || !episode_starts || !last_values || !last_dones || !advantages || !returns)
        return fail(nullptr, SALP_EINVAL, "salp_gae: null buffer");
    if (n_steps == 0 || n_envs == 0) return SALP_OK;
    const hipError_t e = salp_gae_launch(n_steps, n_envs, rewards, values, episode_starts, last_values, last_dones,
                                         gamma, gae_lambda, advantages, returns, stream);
    return check_hip(nullptr, e, "k_gae");
}

}  // extern "C"
