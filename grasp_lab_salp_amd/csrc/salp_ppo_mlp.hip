// salp_ppo_mlp.hip — one PPO minibatch step of the built-in MlpPolicy, fused
// (gfx950).
//
// What it replaces: the minibatch step of stable_baselines3 PPO.train
// (stable-baselines3 >= 2.0, requirements.txt:6-7) for SB3's MlpPolicy
// (separate 64-64 tanh actor and critic, diagonal Gaussian with
// state-independent log-std), as grasp_lab_salp_amd/ppo.py runs it with torch
// ops: forward of both networks, the clipped-surrogate / value / entropy loss
// (salp_ppo.hip's head), backward, clip_grad_norm_(max_norm) and Adam.  In
// torch that is ~60 small kernels per minibatch (GEMMs, elementwise, reduce,
// foreach); here it is four launches on one rank:
//
//   k_mlp_adv_sums   block partials of sum(adv), sum(adv^2) over the gathered
//                    rows (the advantage normalisation's mean / std)
//   k_mlp_fwd_bwd    every block takes a contiguous slice of the minibatch in
//                    tiles of 64 rows: forward through both networks (weights
//                    and activations in LDS, the products on the f32 matrix
//                    cores), the loss head per row, backward to the weight
//                    gradients, which the block accumulates in registers over
//                    its tiles and writes as one fp32 partial per parameter
//   k_mlp_reduce     sums the partials in fp64 into the flat gradient, and
//                    the loss statistics (and, on one rank, the squared
//                    norm's partials)
//   k_mlp_adam       (salp_ppo_mlp_apply) the global gradient norm, the
//                    clipping coefficient and Adam, one parameter per thread
//                    (after k_mlp_norm's norm partials on several ranks; with
//                    no workspace, k_mlp_apply does it all in one block)
//
// Between the reduction and the update a multi-GPU learner all-reduces the
// flat gradient (one RCCL message).  The hidden units' tanh is the collection's
// (salp_tanh.h: branch-free, ~1e-7 from torch's; the library's tanhf was 35
// VALU instructions of the row kernel's ~115 per unit, profiles/r6c_pmc_update_summary.json).  Row math is float32 like torch's; reductions are fp64;
// the results agree with torch to float32 rounding (tests/test_gpu_ppo_mlp.py),
// not bit for bit (different summation orders), and are deterministic (no
// floating-point atomics: k_mlp_adam's one atomic counts arriving blocks).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>

#include "../../include/salp.h"
#include "salp_tanh.h"

namespace {

constexpr int H = SALP_POLICY_HIDDEN;   // 64 hidden units per layer
constexpr int NA = 3;                   // action dims
constexpr int DP = 16;                  // observation columns in LDS (SALP_OBS_DIM_MAX <= 16)
constexpr int TR = 64;                  // rows per tile
constexpr int NT = 512;                 // threads per block of the row kernel (8 waves)
constexpr int NB_MAX = 256;             // row blocks (partials) at most
constexpr int NADV = 256;               // blocks of k_mlp_adv_sums
constexpr int NSTAT = 6;                // stats partials: pg, vf, clip, d log_std x 3
constexpr float kLogSqrt2Pi = 0.91893853320467274178f;
static_assert(SALP_OBS_DIM_MAX <= DP, "observation columns fit the LDS tile");

// Offsets of the tensors in the flat gradient / Adam-state layout.
struct Layout {
    int64_t off[SALP_MLP_N_TENSORS + 1];
};
__host__ __device__ inline int64_t tensor_size(int t, int d) {
    switch (t) {
        case SALP_MLP_PI_W1: case SALP_MLP_VF_W1: return (int64_t)H * d;
        case SALP_MLP_PI_W2: case SALP_MLP_VF_W2: return (int64_t)H * H;
        case SALP_MLP_ACT_W: return (int64_t)NA * H;
        case SALP_MLP_ACT_B: case SALP_MLP_LOG_STD: return NA;
        case SALP_MLP_VAL_W: return H;
        case SALP_MLP_VAL_B: return 1;
        default: return H;   // hidden-layer biases
    }
}
__host__ __device__ inline Layout make_layout(int d) {
    Layout L;
    L.off[0] = 0;
    for (int t = 0; t < SALP_MLP_N_TENSORS; ++t) L.off[t + 1] = L.off[t] + tensor_size(t, d);
    return L;
}

struct RowArgs {
    SalpPpoMinibatch m;
    Layout L;
    int64_t rows_per_block;   // multiple of TR
    float* part;              // [gridDim.x][n_params]
    double* stat_part;        // [gridDim.x][NSTAT]
    const double* adv_part;   // [NADV][2]
};

__device__ __forceinline__ double block_sum_d(double v, double* sh, int nthreads) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    const int w = threadIdx.x / 64, l = threadIdx.x % 64;
    __syncthreads();
    if (l == 0) sh[w] = v;
    __syncthreads();
    double t = 0.0;
    if (threadIdx.x == 0)
        for (int k = 0; k < nthreads / 64; ++k) t += sh[k];
    __syncthreads();
    return t;   // valid in thread 0
}

// K block sums at once, in a fixed order (the wave's xor tree, then the
// waves in order), broadcast to every thread through sh [nthreads / 64][K].
template <int K>
__device__ __forceinline__ void block_sums(double (&v)[K], double* sh, int nthreads) {
    for (int o = 32; o > 0; o >>= 1)
#pragma unroll
        for (int k = 0; k < K; ++k) v[k] += __shfl_xor(v[k], o, 64);
    const int w = threadIdx.x / 64, l = threadIdx.x % 64;
    __syncthreads();
    if (l == 0)
#pragma unroll
        for (int k = 0; k < K; ++k) sh[w * K + k] = v[k];
    __syncthreads();
#pragma unroll
    for (int k = 0; k < K; ++k) {
        double t = 0.0;
        for (int ww = 0; ww < nthreads / 64; ++ww) t += sh[ww * K + k];
        v[k] = t;
    }
}

// The same sums in the same order, valid in thread 0 only (no broadcast: the
// other threads skip the K x waves LDS reads).
template <int K>
__device__ __forceinline__ void block_sums0(double (&v)[K], double* sh, int nthreads) {
    for (int o = 32; o > 0; o >>= 1)
#pragma unroll
        for (int k = 0; k < K; ++k) v[k] += __shfl_xor(v[k], o, 64);
    const int w = threadIdx.x / 64, l = threadIdx.x % 64;
    __syncthreads();
    if (l == 0)
#pragma unroll
        for (int k = 0; k < K; ++k) sh[w * K + k] = v[k];
    __syncthreads();
    if (threadIdx.x == 0)
#pragma unroll
        for (int k = 0; k < K; ++k) {
            double t = 0.0;
            for (int ww = 0; ww < nthreads / 64; ++ww) t += sh[ww * K + k];
            v[k] = t;
        }
}

// blockIdx.y: minibatch (rows idx[y * B ...]), part + y * 2 * NADV (one launch
// per epoch, salp_ppo_mlp_adv_partials; gridDim.y = 1 for one minibatch).
__global__ __launch_bounds__(256) void k_mlp_adv_sums(int64_t B, const int64_t* __restrict__ idx,
                                                      const float* __restrict__ adv, double* __restrict__ part) {
    __shared__ double sh[4];
    idx += (int64_t)blockIdx.y * B;
    part += (int64_t)blockIdx.y * 2 * NADV;
    double s = 0.0, q = 0.0;
    for (int64_t b = (int64_t)blockIdx.x * 256 + threadIdx.x; b < B; b += (int64_t)gridDim.x * 256) {
        const double x = adv[idx[b]];
        s += x;
        q += x * x;
    }
    s = block_sum_d(s, sh, 256);
    q = block_sum_d(q, sh, 256);
    if (threadIdx.x == 0) {
        part[2 * blockIdx.x] = s;
        part[2 * blockIdx.x + 1] = q;
    }
}

// The four GEMM shapes of a 64-row tile run on the f32-input matrix cores
// (v_mfma_f32_32x32x2_f32 / 16x16x4_f32: exact f32, one fmaf chain in k order
// per output, the VALU's numerics).  Waves 0-3 take the actor, 4-7 the
// critic; wave quadrant (qa, qb) owns one 32x32 output tile of every 64x64
// product.  Lane l supplies A[row l&31][k] and B[k][col l&31] of a step, k
// from its own half l>>5 of the step's k range (any pairing of k over the
// steps is a valid sum); results come back with the column on the lane and
// rows crow(reg, half) in the 16 accumulator registers.
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4v __attribute__((ext_vector_type(4)));
constexpr int HS2 = H + 4;   // LDS row stride: rows 16-B aligned, rows 8 apart 32 banks apart
__device__ __forceinline__ f32x16 mfma32(float a, float b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x4v mfma16(float a, float b, f32x4v c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
// row of accumulator register r of a 32x32 result, lane half h
__device__ __forceinline__ int crow(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

__global__ __launch_bounds__(NT) void k_mlp_fwd_bwd(RowArgs a) {
    const SalpPpoMinibatch& m = a.m;
    const int D = m.obs_dim;
    const int64_t B = m.batch;
    const int tid = threadIdx.x;
    const int64_t r_begin = (int64_t)blockIdx.x * a.rows_per_block;
    const int64_t r_end = r_begin + a.rows_per_block < B ? r_begin + a.rows_per_block : B;
    static_assert(TR * DP == 2 * NT, "two observation entries per thread and tile");
    // The gathered rows come in two dependent round trips (the index, then the
    // row), so each is issued a tile ahead of the other: a tile's phase 0 stores
    // the observations loaded during the previous tile, loads the next tile's
    // rows through indices loaded during the previous tile, and loads the
    // indices of the tile after that (r6t: one round trip per tile used to stall
    // phase 0 ~3.7 k cycles).  Entries tid and tid + NT of the [TR][DP] tile;
    // padding rows are zero (index -1).
    auto load_idx = [&](int64_t row0, int64_t* xi) {
        const int64_t n = r_end - row0;
        for (int u = 0; u < 2; ++u) {
            const int r = (tid + u * NT) / DP;
            xi[u] = r < n ? m.idx[row0 + r] : -1;
        }
    };
    auto load_rows = [&](const int64_t* xi, float* xv) {
        for (int u = 0; u < 2; ++u) {
            const int k = (tid + u * NT) % DP;
            xv[u] = (xi[u] >= 0 && k < D) ? m.obs[xi[u] * D + k] : 0.0f;
        }
    };
    // the loss head's row of this thread (hp == 0: one thread per row)
    const int hr = tid / 8, hp = tid % 8;
    auto head_idx = [&](int64_t row0) -> int64_t {
        return (hp == 0 && hr < r_end - row0) ? m.idx[row0 + hr] : -1;
    };
    float xv[2];
    int64_t xi[2] = {-1, -1};           // row indices of the next tile's entries
    int64_t hb = -1, hb_next = -1;      // the head row's index: this tile, the next
    // the first tile's gather is issued before the weight staging, so the two
    // latencies overlap; the second tile's indices with it
    if (r_begin < r_end) {
        int64_t x0[2];
        load_idx(r_begin, x0);
        load_rows(x0, xv);
        hb = head_idx(r_begin);
        if (r_begin + TR < r_end) {
            load_idx(r_begin + TR, xi);
            hb_next = head_idx(r_begin + TR);
        }
    }
    // and so are the advantage partials (summed after it)
    static_assert(NADV <= NT, "one advantage partial per thread");
    const bool norm_adv = m.normalize_advantage && B > 1;
    double sq[2] = {0.0, 0.0};
    if (norm_adv && tid < NADV) {
        sq[0] = a.adv_part[2 * tid];
        sq[1] = a.adv_part[2 * tid + 1];
    }
    // weights (nets: 0 = actor / pi, 1 = critic / vf)
    __shared__ float sW1[2][H][DP];       // [net][unit][input]
    __shared__ float sB1[2][H];
    __shared__ __attribute__((aligned(16))) float sW2[2][H][HS2];   // [net][unit j][input k]
    __shared__ float sB2[2][H];
    __shared__ float sAw[NA][H], sAb[NA], sLs[NA], sVw[H], sVb;
    // one tile of rows
    __shared__ float sX[TR][DP];
    __shared__ __attribute__((aligned(16))) float sH1[2][TR][HS2];  // h1, then dz1 in place
    __shared__ __attribute__((aligned(16))) float sH2[2][TR][HS2];  // h2, then dz2 in place
    __shared__ float sDmu[TR][NA], sDv[TR];
    __shared__ float sNorm[2];
    __shared__ double sRed[NT / 64 * (NA + 1 + NSTAT)];

    // weights into LDS: every load of a thread is issued before its stores
    // (one L2 round trip instead of one per element)
    {
        constexpr int N1 = 2 * H * DP / NT, N2 = 2 * H * H / NT;
        static_assert(N1 * NT == 2 * H * DP && N2 * NT == 2 * H * H, "whole staging rounds");
        float v1[N1], v2[N2];
#pragma unroll
        for (int q = 0; q < N1; ++q) {
            const int e = tid + q * NT, net = e / (H * DP), u = (e / DP) % H, k = e % DP;
            v1[q] = k < D ? m.params[net ? SALP_MLP_VF_W1 : SALP_MLP_PI_W1][u * D + k] : 0.0f;
        }
#pragma unroll
        for (int q = 0; q < N2; ++q) {
            const int e = tid + q * NT, net = e / (H * H);
            v2[q] = m.params[net ? SALP_MLP_VF_W2 : SALP_MLP_PI_W2][e % (H * H)];
        }
#pragma unroll
        for (int q = 0; q < N1; ++q) {
            const int e = tid + q * NT;
            sW1[e / (H * DP)][(e / DP) % H][e % DP] = v1[q];
        }
#pragma unroll
        for (int q = 0; q < N2; ++q) {
            const int e = tid + q * NT;
            sW2[e / (H * H)][(e / H) % H][e % H] = v2[q];
        }
    }
    for (int e = tid; e < 2 * H; e += NT) {
        const int net = e / H, j = e % H;
        sB1[net][j] = m.params[net ? SALP_MLP_VF_B1 : SALP_MLP_PI_B1][j];
        sB2[net][j] = m.params[net ? SALP_MLP_VF_B2 : SALP_MLP_PI_B2][j];
    }
    for (int e = tid; e < NA * H; e += NT) sAw[e / H][e % H] = m.params[SALP_MLP_ACT_W][e];
    if (tid < H) sVw[tid] = m.params[SALP_MLP_VAL_W][tid];
    if (tid < NA) {
        sAb[tid] = m.params[SALP_MLP_ACT_B][tid];
        sLs[tid] = m.params[SALP_MLP_LOG_STD][tid];
    }
    if (tid == 0) sVb = m.params[SALP_MLP_VAL_B][0];
    // advantage mean / std of the minibatch from k_mlp_adv_sums' partials, summed by the block
    if (norm_adv) {
        block_sums0(sq, sRed, NT);
        if (tid == 0) {
            const double mu = sq[0] / (double)B;
            const double var = fmax(sq[1] - sq[0] * mu, 0.0) / (double)(B - 1);
            sNorm[0] = (float)mu;
            sNorm[1] = 1.0f / ((float)sqrt(var) + 1e-8f);
        }
    } else if (tid == 0) {
        sNorm[0] = 0.0f;
        sNorm[1] = 1.0f;
    }
    __syncthreads();

    const int w = tid / 64, l = tid % 64, net = w >> 2, q = w & 3, qa = q >> 1, qb = q & 1;
    const int lc = l & 31, lh = l >> 5;
    // gradient accumulators, kept over the block's tiles
    f32x16 gW2 = {};           // dW2[net][32 qa + crow(r, lh)][32 qb + lc]
    f32x4v gW1 = {};           // dW1[net][16 q + 4 (l >> 4) + r][l & 15]
    float gB2 = 0.0f;          // db2[net][32 qa + lc], partial over this lane half's rows (qb == 0 waves)
    float gB1 = 0.0f;          // db1[net][16 q + (l & 15)], partial over this lane group's rows
    float gH[NA] = {0.0f, 0.0f, 0.0f};   // dWa[c][32 qb + lc] (actor) / dVw (critic, gH[0]): this lane's rows
    double gHb[NA + 1] = {0.0, 0.0, 0.0, 0.0};   // dab[c], dvb: the rows of this heads thread
    double st[NSTAT] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
    float ls[NA], var[NA];
    for (int j = 0; j < NA; ++j) {
        ls[j] = sLs[j];
        const float sd = expf(ls[j]);
        var[j] = sd * sd;
    }
    // this lane's columns of the heads (dz2 of its tile from registers)
    const float aw0 = sAw[0][32 * qb + lc], aw1 = sAw[1][32 * qb + lc], aw2 = sAw[2][32 * qb + lc];
    const float vw = sVw[32 * qb + lc];
    const float invB = 1.0f / (float)B, clip = (float)m.clip_range, vfc = (float)m.vf_coef;
    const float amean = sNorm[0], ainv = sNorm[1];

    for (int64_t row0 = r_begin; row0 < r_end; row0 += TR) {
        const int nrows = (int)(r_end - row0 < TR ? r_end - row0 : TR);
        for (int u = 0; u < 2; ++u) sX[(tid + u * NT) / DP][(tid + u * NT) % DP] = xv[u];
        if (row0 + TR < r_end) {
            load_rows(xi, xv);
            if (row0 + 2 * TR < r_end) load_idx(row0 + 2 * TR, xi);
        }
        // the loss head's per-row inputs, issued now, used after both layers
        float r_act[NA] = {0.0f, 0.0f, 0.0f}, r_adv = 0.0f, r_olp = 0.0f, r_ret = 0.0f;
        if (hb >= 0) {
            for (int j = 0; j < NA; ++j) r_act[j] = m.actions[3 * hb + j];
            r_adv = m.advantages[hb];
            r_olp = m.old_log_prob[hb];
            r_ret = m.returns[hb];
        }
        hb = hb_next;
        hb_next = row0 + 2 * TR < r_end ? head_idx(row0 + 2 * TR) : -1;
        __syncthreads();
        // ---- layer 1: h1 = tanh(x W1^T + b1)     (K = 16: 8 steps)
        {
            const float b = sB1[net][32 * qb + lc];
            f32x16 acc = {b, b, b, b, b, b, b, b, b, b, b, b, b, b, b, b};
#pragma unroll
            for (int s = 0; s < DP / 2; ++s) {
                const int k = (DP / 2) * lh + s;
                acc = mfma32(sX[32 * qa + lc][k], sW1[net][32 * qb + lc][k], acc);
            }
#pragma unroll
            for (int r = 0; r < 16; ++r) sH1[net][32 * qa + crow(r, lh)][32 * qb + lc] = salp_tanhf(acc[r]);
        }
        __syncthreads();
        // ---- layer 2: h2 = tanh(h1 W2^T + b2)    (K = 64: 32 steps, k = 32 half + 4 s4 + e); h2 kept
        float h2r[16];
        {
            const float b = sB2[net][32 * qb + lc];
            f32x16 acc = {b, b, b, b, b, b, b, b, b, b, b, b, b, b, b, b};
#pragma unroll
            for (int s4 = 0; s4 < 8; ++s4) {
                const float4 x = *reinterpret_cast<const float4*>(&sH1[net][32 * qa + lc][32 * lh + 4 * s4]);
                const float4 y = *reinterpret_cast<const float4*>(&sW2[net][32 * qb + lc][32 * lh + 4 * s4]);
                acc = mfma32(x.x, y.x, acc);
                acc = mfma32(x.y, y.y, acc);
                acc = mfma32(x.z, y.z, acc);
                acc = mfma32(x.w, y.w, acc);
            }
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                h2r[r] = salp_tanhf(acc[r]);
                sH2[net][32 * qa + crow(r, lh)][32 * qb + lc] = h2r[r];
            }
        }
        __syncthreads();
        // ---- heads and the loss head: 8 threads per row
        {
            const int r = hr, p = hp;
            float s[4] = {0.0f, 0.0f, 0.0f, 0.0f};
            for (int qq = 0; qq < 8; ++qq) {
                const int j = p * 8 + qq;
                const float h_p = sH2[0][r][j], h_v = sH2[1][r][j];
                s[0] = fmaf(h_p, sAw[0][j], s[0]);
                s[1] = fmaf(h_p, sAw[1][j], s[1]);
                s[2] = fmaf(h_p, sAw[2][j], s[2]);
                s[3] = fmaf(h_v, sVw[j], s[3]);
            }
            for (int o = 1; o < 8; o <<= 1)
                for (int c = 0; c < 4; ++c) s[c] += __shfl_xor(s[c], o, 64);
            if (p == 0) {
                float dmu[NA] = {0.0f, 0.0f, 0.0f}, dv = 0.0f;
                if (r < nrows) {
                    float d[NA], lp = 0.0f;
                    for (int j = 0; j < NA; ++j) {
                        const float mu = s[j] + sAb[j];
                        d[j] = r_act[j] - mu;
                        lp += -(d[j] * d[j]) / (2.0f * var[j]) - ls[j] - kLogSqrt2Pi;
                    }
                    const float v = s[3] + sVb;
                    const float A = m.normalize_advantage ? (r_adv - amean) * ainv : r_adv;
                    const float rt = expf(lp - r_olp);
                    const float rc = fminf(fmaxf(rt, 1.0f - clip), 1.0f + clip);
                    const float p1 = A * rt, p2 = A * rc;
                    const float g1 = p1 < p2 ? 1.0f : (p1 == p2 ? 0.5f : 0.0f);
                    const float g2 = p2 < p1 ? 1.0f : (p1 == p2 ? 0.5f : 0.0f);
                    const bool inside = rt >= 1.0f - clip && rt <= 1.0f + clip;
                    const float dL_dr = g1 * A + (inside ? g2 * A : 0.0f);
                    const float dlp = -invB * dL_dr * rt;
                    for (int j = 0; j < NA; ++j) {
                        dmu[j] = dlp * d[j] / var[j];
                        st[3 + j] += (double)(dlp * (d[j] * d[j] / var[j] - 1.0f));
                    }
                    const float e = r_ret - v;
                    dv = vfc * (-2.0f * e * invB);
                    st[0] += (double)fminf(p1, p2);
                    st[1] += (double)(e * e);
                    st[2] += fabsf(rt - 1.0f) > clip ? 1.0 : 0.0;
                }
                for (int j = 0; j < NA; ++j) {
                    sDmu[r][j] = dmu[j];
                    gHb[j] += (double)dmu[j];
                }
                sDv[r] = dv;
                gHb[NA] += (double)dv;
            }
        }
        __syncthreads();
        // ---- head weight gradients and dz2 = (head^T d) (1 - h2^2) of this wave's
        //      tile, from the h2 it kept; dz2 replaces h2 (every reader of h2 is done)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int row = 32 * qa + crow(r, lh);
            const float h = h2r[r];
            float dh;
            if (net == 0) {
                const float d0 = sDmu[row][0], d1 = sDmu[row][1], d2 = sDmu[row][2];
                gH[0] = fmaf(d0, h, gH[0]);
                gH[1] = fmaf(d1, h, gH[1]);
                gH[2] = fmaf(d2, h, gH[2]);
                dh = fmaf(d2, aw2, fmaf(d1, aw1, d0 * aw0));
            } else {
                const float dv = sDv[row];
                gH[0] = fmaf(dv, h, gH[0]);
                dh = dv * vw;
            }
            sH2[net][row][32 * qb + lc] = dh * (1.0f - h * h);
        }
        __syncthreads();
        // ---- dW2 += dz2^T h1 (K = rows: r = 16 (s / 8) + 8 half + s % 8), db2 from the same
        //      operand, dh1 = dz2 W2 (K = units: 32 half + 4 s4 + e), dz1 = dh1 (1 - h1^2)
        float dz1[16];
        {
#pragma unroll
            for (int s = 0; s < 32; ++s) {
                const int r = 16 * (s >> 3) + 8 * lh + (s & 7);
                const float z = sH2[net][r][32 * qa + lc];
                gB2 += z;
                gW2 = mfma32(z, sH1[net][r][32 * qb + lc], gW2);
            }
            f32x16 dh = {};
#pragma unroll
            for (int s4 = 0; s4 < 8; ++s4) {
                const float4 z = *reinterpret_cast<const float4*>(&sH2[net][32 * qa + lc][32 * lh + 4 * s4]);
                const int j = 32 * lh + 4 * s4;
                dh = mfma32(z.x, sW2[net][j + 0][32 * qb + lc], dh);
                dh = mfma32(z.y, sW2[net][j + 1][32 * qb + lc], dh);
                dh = mfma32(z.z, sW2[net][j + 2][32 * qb + lc], dh);
                dh = mfma32(z.w, sW2[net][j + 3][32 * qb + lc], dh);
            }
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const float h = sH1[net][32 * qa + crow(r, lh)][32 * qb + lc];
                dz1[r] = dh[r] * (1.0f - h * h);
            }
        }
        __syncthreads();   // every read of h1 is done: dz1 replaces it
#pragma unroll
        for (int r = 0; r < 16; ++r) sH1[net][32 * qa + crow(r, lh)][32 * qb + lc] = dz1[r];
        __syncthreads();
        // ---- dW1 += dz1^T x (16x16x4: wave q takes units 16 q .. 16 q + 15; r = 16 (l >> 4) + s),
        //      db1 from the same operand
#pragma unroll
        for (int s = 0; s < TR / 4; ++s) {
            const int r = 16 * (l >> 4) + s;
            const float z = sH1[net][r][16 * q + (l & 15)];
            gB1 += z;
            gW1 = mfma16(z, sX[r][l & 15], gW1);
        }
        __syncthreads();
    }

    // ---- this block's partials, in the flat gradient layout
    float* P = a.part + (int64_t)blockIdx.x * a.L.off[SALP_MLP_N_TENSORS];
    {
        const int64_t ow2 = a.L.off[net ? SALP_MLP_VF_W2 : SALP_MLP_PI_W2];
#pragma unroll
        for (int r = 0; r < 16; ++r) P[ow2 + (32 * qa + crow(r, lh)) * H + 32 * qb + lc] = gW2[r];
        const int64_t ow1 = a.L.off[net ? SALP_MLP_VF_W1 : SALP_MLP_PI_W1];
        if ((l & 15) < D)
#pragma unroll
            for (int r = 0; r < 4; ++r) P[ow1 + (16 * q + 4 * (l >> 4) + r) * D + (l & 15)] = gW1[r];
        // db2: the two lane halves' rows (waves qb == 0 saw every unit 32 qa + lc)
        const float b2 = gB2 + __shfl_xor(gB2, 32, 64);
        if (qb == 0 && lh == 0) P[a.L.off[net ? SALP_MLP_VF_B2 : SALP_MLP_PI_B2] + 32 * qa + lc] = b2;
        // db1: the four lane groups' rows
        float b1 = gB1 + __shfl_xor(gB1, 16, 64);
        b1 += __shfl_xor(b1, 32, 64);
        if (l < 16) P[a.L.off[net ? SALP_MLP_VF_B1 : SALP_MLP_PI_B1] + 16 * q + l] = b1;
    }
    // head weights: lane halves, then the two row-tile waves (qa) of each column block, via LDS
    {
        __shared__ float sHG[2][2][NA][H];   // [net][qa][c][unit]
        float hg[NA];
        for (int c = 0; c < NA; ++c) hg[c] = gH[c] + __shfl_xor(gH[c], 32, 64);
        if (lh == 0)
            for (int c = 0; c < (net == 0 ? NA : 1); ++c) sHG[net][qa][c][32 * qb + lc] = hg[c];
        __syncthreads();
        if (tid < NA * H) {
            const int c = tid / H, j = tid % H;
            P[a.L.off[SALP_MLP_ACT_W] + tid] = sHG[0][0][c][j] + sHG[0][1][c][j];
        } else if (tid < NA * H + H) {
            const int j = tid - NA * H;
            P[a.L.off[SALP_MLP_VAL_W] + j] = sHG[1][0][0][j] + sHG[1][1][0][j];
        }
    }
    // head biases and the loss statistics: one block reduction for all ten
    double red[NA + 1 + NSTAT];
#pragma unroll
    for (int c = 0; c <= NA; ++c) red[c] = gHb[c];
#pragma unroll
    for (int k = 0; k < NSTAT; ++k) red[NA + 1 + k] = st[k];
    block_sums0(red, sRed, NT);
    if (tid == 0) {
        for (int c = 0; c <= NA; ++c) P[c < NA ? a.L.off[SALP_MLP_ACT_B] + c : a.L.off[SALP_MLP_VAL_B]] = (float)red[c];
        for (int k = 0; k < NSTAT; ++k) a.stat_part[(int64_t)blockIdx.x * NSTAT + k] = red[NA + 1 + k];
    }
}

// Flat gradient = sum of the block partials (fp64); d loss / d log_std gets its
// row sums and - ent_coef; block 0 also adds the loss statistics to stats[4].
// One block per 64 parameters: its 16 waves take every 16th partial each (at
// most 16 independent loads per lane, all in flight at once), then wave 0 adds
// the 16 wave sums in a fixed order (deterministic).
constexpr int NT_RED = 1024, RED_G = NT_RED / 64, RED_T = NB_MAX / RED_G;
__global__ __launch_bounds__(NT_RED) void k_mlp_reduce(SalpPpoMinibatch m, Layout L, int nb, const float* part,
                                                       const double* stat_part) {
    __shared__ double sh[RED_G][64];
    const int64_t P = L.off[SALP_MLP_N_TENSORS];
    const int l = threadIdx.x % 64, g = threadIdx.x / 64;
    const int64_t p = (int64_t)blockIdx.x * 64 + l;
    const int64_t ols = L.off[SALP_MLP_LOG_STD];
    const bool is_ls = p >= ols && p < ols + NA;
    double s = 0.0;
    if (p < P) {
        double v[RED_T];
#pragma unroll
        for (int t = 0; t < RED_T; ++t) {
            const int b = g + t * RED_G;
            v[t] = b >= nb ? 0.0
                 : is_ls ? stat_part[(int64_t)b * NSTAT + 3 + (p - ols)] : (double)part[(int64_t)b * P + p];
        }
#pragma unroll
        for (int t = 0; t < RED_T; ++t) s += v[t];
    }
    sh[g][l] = s;
    __syncthreads();
    float gf = 0.0f;
    if (g == 0 && p < P) {
        double t = 0.0;
#pragma unroll
        for (int k = 0; k < RED_G; ++k) t += sh[k][l];
        if (is_ls) t = (double)((float)t - (float)m.ent_coef);
        gf = (float)t;
        m.grads[p] = gf;
    }
    if (g == 0 && m.norm_part) {
        // this block's 64 parameters' share of the squared norm, in k_mlp_norm's order
        double q = (double)gf * (double)gf;
        for (int o = 32; o > 0; o >>= 1) q += __shfl_xor(q, o, 64);
        if (l == 0) m.norm_part[blockIdx.x] = q;
    }
    if (blockIdx.x == 0 && g == 1 && m.stats) {
        // every lane's partials loaded at once, then summed in the same order
        double x[NB_MAX / 64][3];
#pragma unroll
        for (int j = 0; j < NB_MAX / 64; ++j) {
            const int b = l + 64 * j;
#pragma unroll
            for (int k = 0; k < 3; ++k) x[j][k] = b < nb ? stat_part[(int64_t)b * NSTAT + k] : 0.0;
        }
        double t[3] = {0.0, 0.0, 0.0};
#pragma unroll
        for (int j = 0; j < NB_MAX / 64; ++j)
            if (l + 64 * j < nb)
                for (int k = 0; k < 3; ++k) t[k] += x[j][k];
        for (int o = 32; o > 0; o >>= 1)
            for (int k = 0; k < 3; ++k) t[k] += __shfl_xor(t[k], o, 64);
        if (l == 0) {
            const double B = (double)m.batch;
            float ent = 0.0f;
            for (int j = 0; j < NA; ++j) ent += 0.5f + kLogSqrt2Pi + m.params[SALP_MLP_LOG_STD][j];
            m.stats[0] += (float)(-t[0] / B);   // pg_loss
            m.stats[1] += (float)(t[1] / B);    // vf_loss
            m.stats[2] += ent;                  // entropy
            m.stats[3] += (float)(t[2] / B);    // clip fraction
        }
    }
}

// clip_grad_norm_(max_norm) and torch.optim.Adam (no weight decay, no
// amsgrad), over the flat gradient, in one block: every thread loads its
// parameters' gradient, moments and weights in one round (AP_MAX each), the
// block reduces the squared norm, then the thread updates them.
constexpr int NT_APPLY = 1024;
constexpr int AP_MAX = 11;   // parameters per thread
static_assert((int64_t)NT_APPLY * AP_MAX >= 2 * (H * DP + H + H * H + H) + NA * H + 2 * NA + H + 1,
              "the flat gradient of obs_dim <= 16 fits one apply block");
__global__ __launch_bounds__(NT_APPLY) void k_mlp_apply(SalpPpoAdam o, Layout L) {
    __shared__ double sh[NT_APPLY / 64];
    __shared__ float s_coef;
    __shared__ float s_adam[2];   // lr / (1 - beta1^step), sqrt(1 - beta2^step)
    __shared__ float* s_base[SALP_MLP_N_TENSORS];   // params[t] - off[t]: p indexes it directly
    __shared__ int s_off[SALP_MLP_N_TENSORS];
#pragma unroll
    for (int t = 0; t < SALP_MLP_N_TENSORS; ++t)
        if (threadIdx.x == t) {
            s_base[t] = o.params[t] - L.off[t];
            s_off[t] = (int)L.off[t];
        }
    const int P = (int)L.off[SALP_MLP_N_TENSORS];
    const float step = o.step[0] + 1.0f;   // issued with the parameter loads, not after the norm
    __syncthreads();
    float g[AP_MAX], m1[AP_MAX], v1[AP_MAX], w1[AP_MAX];
    float* wp[AP_MAX];
    double q = 0.0;
#pragma unroll
    for (int k = 0; k < AP_MAX; ++k) {
        const int p = threadIdx.x + k * NT_APPLY;
        int t = 0;
#pragma unroll
        for (int u = 1; u < SALP_MLP_N_TENSORS; ++u) t += p >= s_off[u] ? 1 : 0;
        wp[k] = s_base[t] + p;
        g[k] = m1[k] = v1[k] = w1[k] = 0.0f;
        if (p < P) {
            g[k] = o.grads[p];
            m1[k] = o.exp_avg[p];
            v1[k] = o.exp_avg_sq[p];
            w1[k] = *wp[k];
        }
    }
    // Adam's bias corrections from the step count alone: wave 0 computes them
    // while the parameter loads are in flight and hands them over with the
    // norm's barriers (two powf in all 16 waves after those barriers: ~2 us)
    const float b1 = (float)o.beta1, b2 = (float)o.beta2, lr = (float)o.lr, eps = (float)o.eps;
    if (threadIdx.x < 64) {
        const float bc1 = 1.0f - powf(b1, step), bc2 = 1.0f - powf(b2, step);
        if (threadIdx.x == 0) {
            s_adam[0] = lr / bc1;
            s_adam[1] = sqrtf(bc2);
        }
    }
#pragma unroll
    for (int k = 0; k < AP_MAX; ++k) q += (double)g[k] * (double)g[k];
    q = block_sum_d(q, sh, NT_APPLY);
    if (threadIdx.x == 0) {
        const float total = (float)sqrt(q);
        float coef = 1.0f;
        if (o.max_grad_norm > 0.0) {
            coef = (float)o.max_grad_norm / (total + 1e-6f);
            coef = coef < 1.0f ? coef : 1.0f;
        }
        s_coef = coef;
        if (o.grad_norm) o.grad_norm[0] = total;
    }
    __syncthreads();
    const float coef = s_coef;
    const float step_size = s_adam[0], bc2_sqrt = s_adam[1];
#pragma unroll
    for (int k = 0; k < AP_MAX; ++k) {
        const int p = threadIdx.x + k * NT_APPLY;
        if (p < P) {
            const float gc = g[k] * coef;
            const float m = b1 * m1[k] + (1.0f - b1) * gc;
            const float v = b2 * v1[k] + (1.0f - b2) * gc * gc;
            o.exp_avg[p] = m;
            o.exp_avg_sq[p] = v;
            *wp[k] = w1[k] - step_size * m / (sqrtf(v) / bc2_sqrt + eps);
        }
    }
    if (threadIdx.x == 0) o.step[0] = step;
}

// The same clip + Adam over many blocks (SalpPpoAdam.workspace set, ABI 13).
// The squared norm's partials, one per 64 parameters (a wave's xor tree over
// (double) g^2), come from k_mlp_reduce (SalpPpoMinibatch.norm_part: one rank)
// or from k_mlp_norm (after a multi-GPU all-reduce); the two give the same
// bits.  k_mlp_adam runs one parameter per thread; every block sums the
// partials in the same fixed order, so every block derives the same norm and
// clipping coefficient (deterministic), and the last block to arrive (a
// vector atomic count in the workspace, after every block has read the step)
// writes Adam's new step count.  r6m: the one-block kernel above took 10.6 us
// per minibatch (~60 instructions per parameter on one CU); r5v's many-block
// variant had re-read the whole gradient in every block for the norm.
constexpr int NT_ADAM = 256;
constexpr int NORM_PARTS_MAX = SALP_PPO_APPLY_WORKSPACE_DOUBLES - 1;   // the last slot: the arrival count
constexpr int NORM_LANE_PARTS = (NORM_PARTS_MAX + 63) / 64;
static_assert((2 * (H * DP + H + H * H + H) + NA * H + 2 * NA + H + 1 + 63) / 64 <= NORM_PARTS_MAX,
              "the norm partials of obs_dim <= 16 fit the workspace");
__global__ __launch_bounds__(NT_ADAM) void k_mlp_norm(SalpPpoAdam o, int P) {
    const int p = blockIdx.x * NT_ADAM + threadIdx.x;
    double q = 0.0;
    if (p < P) {
        const float g = o.grads[p];
        q = (double)g * (double)g;
    }
    for (int off = 32; off > 0; off >>= 1) q += __shfl_xor(q, off, 64);
    if (threadIdx.x % 64 == 0 && p < P) o.workspace[p / 64] = q;
}

__global__ __launch_bounds__(NT_ADAM) void k_mlp_adam(SalpPpoAdam o, Layout L) {
    __shared__ float* s_base[SALP_MLP_N_TENSORS];   // params[t] - off[t]: p indexes it directly
    __shared__ int s_off[SALP_MLP_N_TENSORS];
    __shared__ float s_k[3];                        // clipping coefficient, lr / (1 - beta1^step), sqrt(1 - beta2^step)
#pragma unroll
    for (int t = 0; t < SALP_MLP_N_TENSORS; ++t)
        if (threadIdx.x == t) {
            s_base[t] = o.params[t] - L.off[t];
            s_off[t] = (int)L.off[t];
        }
    const int P = (int)L.off[SALP_MLP_N_TENSORS];
    const int nparts = (P + 63) / 64;
    const int p = blockIdx.x * NT_ADAM + threadIdx.x;
    float g = 0.0f, m1 = 0.0f, v1 = 0.0f;
    if (p < P) {
        g = o.grads[p];
        m1 = o.exp_avg[p];
        v1 = o.exp_avg_sq[p];
    }
    const float b1 = (float)o.beta1, b2 = (float)o.beta2, lr = (float)o.lr, eps = (float)o.eps;
    if (threadIdx.x < 64) {
        // the norm: lane l adds partials l, l + 64, ... in order, then the xor tree
        double q = 0.0;
#pragma unroll
        for (int j = 0; j < NORM_LANE_PARTS; ++j) {
            const int k = threadIdx.x + 64 * j;
            q += k < nparts ? o.workspace[k] : 0.0;
        }
        for (int off = 32; off > 0; off >>= 1) q += __shfl_xor(q, off, 64);
        const float step = o.step[0] + 1.0f;
        const float bc1 = 1.0f - powf(b1, step), bc2 = 1.0f - powf(b2, step);
        if (threadIdx.x == 0) {
            const float total = (float)sqrt(q);
            float coef = 1.0f;
            if (o.max_grad_norm > 0.0) {
                coef = (float)o.max_grad_norm / (total + 1e-6f);
                coef = coef < 1.0f ? coef : 1.0f;
            }
            s_k[0] = coef;
            s_k[1] = lr / bc1;
            s_k[2] = sqrtf(bc2);
            if (blockIdx.x == 0 && o.grad_norm) o.grad_norm[0] = total;
            // every block has read the step count before it arrives; the last one advances it
            unsigned* const arrived = reinterpret_cast<unsigned*>(o.workspace + NORM_PARTS_MAX);
            if (atomicAdd(arrived, 1u) == gridDim.x - 1) {
                o.step[0] = step;
                *arrived = 0u;
            }
        }
    }
    __syncthreads();
    if (p < P) {
        int t = 0;
#pragma unroll
        for (int u = 1; u < SALP_MLP_N_TENSORS; ++u) t += p >= s_off[u] ? 1 : 0;
        float* const wp = s_base[t] + p;
        const float w1 = *wp;
        const float coef = s_k[0], step_size = s_k[1], bc2_sqrt = s_k[2];
        const float gc = g * coef;
        const float m = b1 * m1 + (1.0f - b1) * gc;
        const float v = b2 * v1 + (1.0f - b2) * gc * gc;
        o.exp_avg[p] = m;
        o.exp_avg_sq[p] = v;
        *wp = w1 - step_size * m / (sqrtf(v) / bc2_sqrt + eps);
    }
}

}  // namespace

extern "C" __attribute__((visibility("hidden"))) int64_t salp_ppo_mlp_params_impl(int obs_dim) {
    return make_layout(obs_dim).off[SALP_MLP_N_TENSORS];
}
extern "C" __attribute__((visibility("hidden"))) int64_t salp_ppo_mlp_offset_impl(int obs_dim, int tensor) {
    return make_layout(obs_dim).off[tensor];
}

// Blocks of the row kernel and the workspace they need (doubles).
static int row_blocks(int64_t B) {
    const int64_t tiles = (B + TR - 1) / TR;
    return (int)(tiles < NB_MAX ? tiles : NB_MAX);
}
extern "C" __attribute__((visibility("hidden"))) int64_t salp_ppo_mlp_workspace_impl(int64_t B, int obs_dim) {
    const int nb = row_blocks(B);
    const int64_t P = make_layout(obs_dim).off[SALP_MLP_N_TENSORS];
    // adv partials, stats partials (doubles) + fp32 parameter partials (as doubles, rounded up)
    return 2 * NADV + (int64_t)nb * NSTAT + ((int64_t)nb * P + 1) / 2;
}

extern "C" __attribute__((visibility("hidden"))) hipError_t salp_ppo_mlp_grads_launch(const SalpPpoMinibatch* mb,
                                                                                       void* stream) {
    hipStream_t s = (hipStream_t)stream;
    const SalpPpoMinibatch& m = *mb;
    const int nb = row_blocks(m.batch);
    const Layout L = make_layout(m.obs_dim);
    double* const ws_adv = m.workspace;
    double* stat_part = ws_adv + 2 * NADV;
    float* part = reinterpret_cast<float*>(stat_part + (int64_t)nb * NSTAT);
    const double* adv_part = m.adv_part;
    if (!adv_part) {
        hipLaunchKernelGGL(k_mlp_adv_sums, dim3(NADV), dim3(256), 0, s, m.batch, m.idx, m.advantages, ws_adv);
        adv_part = ws_adv;
    }
    const int64_t tiles = (m.batch + TR - 1) / TR;
    const int64_t rpb = (tiles + nb - 1) / nb * TR;
    RowArgs a{m, L, rpb, part, stat_part, adv_part};
    hipLaunchKernelGGL(k_mlp_fwd_bwd, dim3(nb), dim3(NT), 0, s, a);
    const int64_t P = L.off[SALP_MLP_N_TENSORS];
    hipLaunchKernelGGL(k_mlp_reduce, dim3((unsigned)((P + 63) / 64)), dim3(NT_RED), 0, s, m, L, nb, part, stat_part);
    return hipGetLastError();
}

static_assert(2 * NADV == SALP_PPO_ADV_PARTIAL_DOUBLES, "include/salp.h advantage partials per minibatch");
extern "C" __attribute__((visibility("hidden"))) hipError_t salp_ppo_mlp_adv_partials_launch(
        int64_t B, int64_t n_mb, const int64_t* idx, const float* adv, double* out, void* stream) {
    hipLaunchKernelGGL(k_mlp_adv_sums, dim3(NADV, (unsigned)n_mb), dim3(256), 0, (hipStream_t)stream, B, idx, adv,
                       out);
    return hipGetLastError();
}

extern "C" __attribute__((visibility("hidden"))) hipError_t salp_ppo_mlp_apply_launch(const SalpPpoAdam* o,
                                                                                       void* stream) {
    const Layout L = make_layout(o->obs_dim);
    if (o->workspace) {
        const int P = (int)L.off[SALP_MLP_N_TENSORS], nb = (P + NT_ADAM - 1) / NT_ADAM;
        if (!o->norm_ready) hipLaunchKernelGGL(k_mlp_norm, dim3(nb), dim3(NT_ADAM), 0, (hipStream_t)stream, *o, P);
        hipLaunchKernelGGL(k_mlp_adam, dim3(nb), dim3(NT_ADAM), 0, (hipStream_t)stream, *o, L);
    } else {
        hipLaunchKernelGGL(k_mlp_apply, dim3(1), dim3(NT_APPLY), 0, (hipStream_t)stream, *o, L);
    }
    return hipGetLastError();
}
