/*
 * salp_tanh.h — the float32 tanh of the 64-64 tanh MlpPolicy's hidden units,
 * shared by the in-kernel policy of salp_collect (salp_kernels.hip) and the
 * fused PPO minibatch step (salp_ppo_mlp.hip), so that the collection and the
 * update evaluate the same function.
 *
 * Branch-free: below |x| = 0.625 the odd polynomial the device library uses
 * there (x + x^3 P(x^2)), above it 1 - 2 / (1 + 2^(2|x| log2 e)) on the
 * hardware exp2 and reciprocal.  About 1e-7 from torch's tanh (the library's
 * tanhf is ~1 ulp, and runs both of its paths in a wave holding small and large
 * units: 35 instructions against 17 here).  The collection tests hold values
 * and log-probabilities to the torch policy, tests/test_gpu_ppo_mlp.py the
 * update's gradients and Adam steps.
 */
#ifndef SALP_TANH_H
#define SALP_TANH_H

#include <hip/hip_runtime.h>

__device__ __forceinline__ float salp_tanhf(float x) {
    const float a = fabsf(x), z = x * x;
    float p = fmaf(__builtin_bit_cast(float, 0xbbbac73du), z, __builtin_bit_cast(float, 0x3ca908c9u));
    p = fmaf(z, p, __builtin_bit_cast(float, 0xbd5c1c4eu));
    p = fmaf(z, p, __builtin_bit_cast(float, 0x3e088382u));
    p = fmaf(z, p, __builtin_bit_cast(float, 0xbeaaaa99u));
    const float small = fmaf(z, a * p, a);
    const float e = __builtin_amdgcn_exp2f(a * 2.88539008177792681f);
    const float large = fmaf(-2.0f, __builtin_amdgcn_rcpf(1.0f + e), 1.0f);
    return copysignf(a < 0.625f ? small : large, x);
}

#endif /* SALP_TANH_H */
