// salp_gae.hip — GAE / return scan over a device rollout buffer (gfx950).
//
// Restates stable_baselines3's RolloutBuffer.compute_returns_and_advantage
// (stable-baselines3 >= 2.0, requirements.txt:6-7; used with gamma 0.99,
// gae_lambda 0.95 by src/train_robot_recurrent_ppo.py:94-95) for buffers of
// shape [n_steps][n_envs] float32:
//
//   for step in reversed(range(n_steps)):
//       nnt, nv = (1 - dones, last_values) if step == n_steps - 1
//                 else (1 - episode_starts[step + 1], values[step + 1])
//       delta = rewards[step] + gamma * nv * nnt - values[step]
//       last  = delta + gamma * gae_lambda * nnt * last
//       advantages[step] = last
//   returns = advantages + values
//
// in float32 with NumPy 2's promotion of the Python-float coefficients
// (float32(gamma), float32(gamma * gae_lambda)) and the same left-to-right
// operation order, no FMA contraction: bit-identical to the NumPy code.
//
// One env per lane; the time loop runs backwards in blocks of kU steps whose
// loads are all issued before the block's dependent chain, so each wave keeps
// 3 * kU coalesced 256 B loads in flight (the scan is HBM-bound: 12 B read and
// 8 B written per (step, env)).
#include <hip/hip_runtime.h>

#include <cstdint>

#pragma clang fp contract(off)

namespace {

#ifndef GAE_BLOCK
#define GAE_BLOCK 256
#endif
constexpr int kGaeBlock = GAE_BLOCK;
constexpr int kU = 16;

__device__ __forceinline__ void gae_load(const float* __restrict__ rew, const float* __restrict__ val,
                                         const float* __restrict__ starts, int64_t t, int64_t n, int64_t e,
                                         float* rb, float* vb, float* sb) {
#pragma unroll
    for (int u = 0; u < kU; ++u) {
        const size_t k = (size_t)(t - u) * (size_t)n + (size_t)e;
        rb[u] = rew[k];
        vb[u] = val[k];
        sb[u] = starts[k];
    }
}

__global__ __launch_bounds__(kGaeBlock) void k_gae(int64_t T, int64_t n, const float* __restrict__ rew,
                                                   const float* __restrict__ val,
                                                   const float* __restrict__ starts,
                                                   const float* __restrict__ last_val,
                                                   const float* __restrict__ last_done, float g, float gl,
                                                   float* __restrict__ adv, float* __restrict__ ret) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= n) return;
    float last = 0.0f;
    float nv = last_val[e];
    float nnt = 1.0f - last_done[e];
    int64_t t = T - 1;
    // ragged top block first so that the rest are whole blocks of kU
    for (int64_t r = T % kU; r > 0; --r, --t) {
        const size_t k = (size_t)t * (size_t)n + (size_t)e;
        const float v = val[k];
        const float delta = (rew[k] + (g * nv) * nnt) - v;
        last = delta + (gl * nnt) * last;
        adv[k] = last;
        ret[k] = last + v;
        nv = v;
        nnt = 1.0f - starts[k];
    }
    for (; t >= 0; t -= kU) {
        float rb[kU], vb[kU], sb[kU];
        gae_load(rew, val, starts, t, n, e, rb, vb, sb);
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            const size_t k = (size_t)(t - u) * (size_t)n + (size_t)e;
            const float delta = (rb[u] + (g * nv) * nnt) - vb[u];
            last = delta + (gl * nnt) * last;
            adv[k] = last;
            ret[k] = last + vb[u];
            nv = vb[u];
            nnt = 1.0f - sb[u];
        }
    }
}

}  // namespace

// Returns the launch status; the caller reports it (salp_kernels.hip).
extern "C" __attribute__((visibility("hidden"))) hipError_t salp_gae_launch(int64_t n_steps, int64_t n_envs, const float* rewards, const float* values,
                               const float* episode_starts, const float* last_values,
                               const float* last_dones, double gamma, double gae_lambda, float* advantages,
                               float* returns, void* stream) {
    // NumPy 2: python float * float32 array -> the float is cast to float32;
    // gamma * gae_lambda is a python (double) product first.
    const float g = (float)gamma;
    const float gl = (float)(gamma * gae_lambda);
    // Each wave streams its envs' columns serially in time, so the scan needs
    // every CU busy: the largest block (<= kGaeBlock) that still gives one
    // block per CU (256 CUs).  Measured: n = 32768 at 128 lanes 0.71 of HBM
    // peak vs 0.59 at 256 (profiles/r1k_gae_variants.jsonl).
    int64_t bs = kGaeBlock;
    while (bs > 64 && (n_envs + bs - 1) / bs < 256) bs /= 2;
    const unsigned blocks = (unsigned)((n_envs + bs - 1) / bs);
    hipLaunchKernelGGL(k_gae, dim3(blocks), dim3((unsigned)bs), 0, (hipStream_t)stream, n_steps, n_envs, rewards,
                       values, episode_starts, last_values, last_dones, g, gl, advantages, returns);
    return hipGetLastError();
}
