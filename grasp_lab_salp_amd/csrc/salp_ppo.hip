// salp_ppo.hip — fused PPO loss head and its gradient (gfx950).
//
// Restates the loss of stable_baselines3 PPO.train (stable-baselines3 >= 2.0,
// requirements.txt:6-7) for a diagonal-Gaussian policy with state-independent
// log-std, as grasp_lab_salp_amd/ppo.py computes it with torch ops:
//
//   adv    = (adv - mean(adv)) / (std(adv, unbiased) + 1e-8)     (optional)
//   logp_b = sum_j -(a - mu)^2 / (2 sigma^2) - log sigma - log sqrt(2 pi)
//   ratio  = exp(logp - old_logp)
//   pg     = -mean(min(adv * ratio, adv * clamp(ratio, 1 - c, 1 + c)))
//   vf     = mean((returns - value)^2)
//   ent    = mean(sum_j 0.5 + 0.5 log(2 pi) + log sigma)
//   loss   = pg - ent_coef * ent + vf_coef * vf
//
// and, in the same pass, d loss / d mu [B,3], d loss / d value [B] and
// d loss / d log_std [3] with torch's subgradient conventions (minimum: ties
// split the gradient; clamp: the gradient passes on the closed interval).
// Three launches replace the ~45 elementwise/reduction kernels (and their
// autograd backward kernels) the torch expression costs per minibatch:
//   k_ppo_adv_sums   block partials of sum(adv), sum(adv^2) (fp64)
//   k_ppo_rows       every block folds the partials into mean/std, then one
//                    row per thread: loss terms, per-row gradients, block
//                    partials of the sums (fp64)
//   k_ppo_final      one block: scalars and d loss / d log_std
// Row math is float32 like the torch code; sums are accumulated in fp64, so
// results agree with torch to float32 rounding, not bit for bit.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>

namespace {

constexpr int kPpoBlock = 256;
constexpr int kPpoGrid = 256;          // one block per CU
constexpr int kRowSums = 6;            // surrogate, squared error, clipped, 3 x d/dlog_std
constexpr float kLogSqrt2Pi = 0.91893853320467274178f;

__device__ __forceinline__ double block_sum(double v, double* sh) {
    // wave reduction by DPP-free shuffles, then across the block's waves
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    const int w = threadIdx.x / 64, l = threadIdx.x % 64;
    __syncthreads();
    if (l == 0) sh[w] = v;
    __syncthreads();
    double t = 0.0;
    if (threadIdx.x == 0)
        for (int k = 0; k < kPpoBlock / 64; ++k) t += sh[k];
    return t;   // valid in thread 0
}

__global__ __launch_bounds__(kPpoBlock) void k_ppo_adv_sums(int64_t B, const float* __restrict__ adv,
                                                            double* __restrict__ part) {
    __shared__ double sh[kPpoBlock / 64];
    double s = 0.0, q = 0.0;
    for (int64_t b = (int64_t)blockIdx.x * kPpoBlock + threadIdx.x; b < B; b += (int64_t)gridDim.x * kPpoBlock) {
        const double x = adv[b];
        s += x;
        q += x * x;
    }
    s = block_sum(s, sh);
    q = block_sum(q, sh);
    if (threadIdx.x == 0) {
        part[2 * blockIdx.x] = s;
        part[2 * blockIdx.x + 1] = q;
    }
}

__global__ __launch_bounds__(kPpoBlock) void k_ppo_rows(
    int64_t B, const float* __restrict__ mu, const float* __restrict__ log_std, const float* __restrict__ value,
    const float* __restrict__ act, const float* __restrict__ old_logp, const float* __restrict__ adv,
    const float* __restrict__ ret, float clip, float vf_coef, int normalize, const double* __restrict__ adv_part,
    double* __restrict__ row_part, float* __restrict__ dmu, float* __restrict__ dvalue) {
    __shared__ double sh[kPpoBlock / 64];
    __shared__ float s_stats[2];
    if (threadIdx.x == 0) {
        float m = 0.0f, inv = 1.0f;
        if (normalize && B > 1) {
            double s = 0.0, q = 0.0;
            for (int k = 0; k < kPpoGrid; ++k) { s += adv_part[2 * k]; q += adv_part[2 * k + 1]; }
            const double mean = s / (double)B;
            const double var = fmax(q - s * mean, 0.0) / (double)(B - 1);
            m = (float)mean;
            inv = 1.0f / ((float)sqrt(var) + 1e-8f);
        }
        s_stats[0] = m;
        s_stats[1] = inv;
    }
    __syncthreads();
    const float amean = s_stats[0], ainv = s_stats[1];
    float ls[3], var[3];
    for (int j = 0; j < 3; ++j) {
        ls[j] = log_std[j];
        const float sd = expf(ls[j]);
        var[j] = sd * sd;
    }
    const float invB = 1.0f / (float)B;
    double acc[kRowSums] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
    for (int64_t b = (int64_t)blockIdx.x * kPpoBlock + threadIdx.x; b < B; b += (int64_t)gridDim.x * kPpoBlock) {
        float d[3], lp = 0.0f;
        for (int j = 0; j < 3; ++j) {
            d[j] = act[3 * b + j] - mu[3 * b + j];
            lp += -(d[j] * d[j]) / (2.0f * var[j]) - ls[j] - kLogSqrt2Pi;
        }
        const float A = normalize ? (adv[b] - amean) * ainv : adv[b];
        const float r = expf(lp - old_logp[b]);
        const float rc = fminf(fmaxf(r, 1.0f - clip), 1.0f + clip);
        const float p1 = A * r, p2 = A * rc;
        const float g1 = p1 < p2 ? 1.0f : (p1 == p2 ? 0.5f : 0.0f);
        const float g2 = p2 < p1 ? 1.0f : (p1 == p2 ? 0.5f : 0.0f);
        const bool inside = r >= 1.0f - clip && r <= 1.0f + clip;
        const float dL_dr = g1 * A + (inside ? g2 * A : 0.0f);
        const float dlp = -invB * dL_dr * r;          // d pg / d logp_b
        for (int j = 0; j < 3; ++j) {
            dmu[3 * b + j] = dlp * d[j] / var[j];
            acc[3 + j] += (double)(dlp * (d[j] * d[j] / var[j] - 1.0f));
        }
        const float e = ret[b] - value[b];
        dvalue[b] = vf_coef * (-2.0f * e * invB);
        acc[0] += (double)fminf(p1, p2);
        acc[1] += (double)(e * e);
        acc[2] += fabsf(r - 1.0f) > clip ? 1.0 : 0.0;
    }
    for (int k = 0; k < kRowSums; ++k) {
        const double t = block_sum(acc[k], sh);
        if (threadIdx.x == 0) row_part[kRowSums * blockIdx.x + k] = t;
    }
}

__global__ __launch_bounds__(kPpoBlock) void k_ppo_final(int64_t B, const float* __restrict__ log_std,
                                                         float ent_coef, float vf_coef,
                                                         const double* __restrict__ row_part,
                                                         float* __restrict__ out) {
    __shared__ double sh[kPpoBlock / 64];
    double t[kRowSums];
    for (int k = 0; k < kRowSums; ++k) {
        const double v = threadIdx.x < kPpoGrid ? row_part[kRowSums * threadIdx.x + k] : 0.0;
        t[k] = block_sum(v, sh);
    }
    if (threadIdx.x == 0) {
        const float pg = (float)(-t[0] / (double)B);
        const float vf = (float)(t[1] / (double)B);
        float ent = 0.0f;
        for (int j = 0; j < 3; ++j) ent += 0.5f + kLogSqrt2Pi + log_std[j];
        out[0] = pg - ent_coef * ent + vf_coef * vf;   // loss
        out[1] = pg;
        out[2] = vf;
        out[3] = ent;
        out[4] = (float)(t[2] / (double)B);            // clip fraction
        for (int j = 0; j < 3; ++j) out[5 + j] = (float)t[3 + j] - ent_coef;   // d loss / d log_std
    }
}

static_assert(kPpoGrid <= kPpoBlock, "k_ppo_final reduces one partial per thread");

}  // namespace

// Returns the launch status (hipSuccess or the error the launches left); the
// caller builds its message from this value, not from a second
// hipGetLastError() (which would read the already-cleared error).
extern "C" __attribute__((visibility("hidden"))) hipError_t salp_ppo_loss_launch(
    int64_t B, const float* mu, const float* log_std, const float* value, const float* actions,
    const float* old_logp, const float* adv, const float* returns, double clip_range, double ent_coef,
    double vf_coef, int normalize_advantage, double* workspace, float* out, float* dmu, float* dvalue,
    void* stream) {
    hipStream_t s = (hipStream_t)stream;
    double* adv_part = workspace;
    double* row_part = workspace + 2 * kPpoGrid;
    hipLaunchKernelGGL(k_ppo_adv_sums, dim3(kPpoGrid), dim3(kPpoBlock), 0, s, B, adv, adv_part);
    hipLaunchKernelGGL(k_ppo_rows, dim3(kPpoGrid), dim3(kPpoBlock), 0, s, B, mu, log_std, value, actions, old_logp,
                       adv, returns, (float)clip_range, (float)vf_coef, normalize_advantage, adv_part, row_part, dmu,
                       dvalue);
    hipLaunchKernelGGL(k_ppo_final, dim3(1), dim3(kPpoBlock), 0, s, B, log_std, (float)ent_coef, (float)vf_coef,
                       row_part, out);
    return hipGetLastError();
}
