// salp_lstm.hip — the LSTM cell of RecurrentPPO's MlpLstmPolicy (gfx950).
//
// What it replaces: the elementwise part of one torch.nn.LSTM step (gates
// i, f, g, o in torch's order; c' = f c + i g, h' = o tanh(c')), with
// sb3-contrib's episode-start reset folded in (c is multiplied by keep =
// 1 - episode_start before the step, as sb3-contrib's _process_sequence
// zeroes the state), and its backward.  The gate pre-activations
// G = x W_ih^T + b + (h keep) W_hh^T stay library GEMMs (grasp_lab_salp_amd/
// recurrent_ppo.py); what these kernels fuse is the ~8 elementwise torch
// kernels of a step forward and ~12 backward, which at 2 048 sequences x 16
// steps x 2 LSTMs made RecurrentPPO's update launch-bound.
//
// One thread per (row, unit): the four gate columns of a row are H apart, so
// each gate's loads are coalesced across the wave.  float32 like torch.
#include <hip/hip_runtime.h>

#include <cstdint>

namespace {

__device__ __forceinline__ float sigm(float x) { return 1.0f / (1.0f + expf(-x)); }

// act [m][4H]: the activated gates (i, f, g, o) for the backward pass
// Sequence steps (salp_lstm_step_forward): GX (the input projection, or null)
// is added to G here instead of by a copy before the GEMM, and hk = h keep_next
// (the next step's GEMM operand, when keep_next is not null) is written too.
__global__ __launch_bounds__(256) void k_lstm_fwd(int64_t m, int H, const float* __restrict__ G,
                                                  const float* __restrict__ GX,
                                                  const float* __restrict__ c_prev, const float* __restrict__ keep,
                                                  const float* __restrict__ keep_next,
                                                  float* __restrict__ h, float* __restrict__ c,
                                                  float* __restrict__ act, float* __restrict__ hk) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= m * H) return;
    const int64_t r = e / H;
    const int u = (int)(e - r * H);
    const float* g = G + r * 4 * H;
    float gi = g[u], gf = g[H + u], gc = g[2 * H + u], go = g[3 * H + u];
    if (GX) {
        const float* x = GX + r * 4 * H;
        gi = x[u] + gi;
        gf = x[H + u] + gf;
        gc = x[2 * H + u] + gc;
        go = x[3 * H + u] + go;
    }
    const float ig = sigm(gi), fg = sigm(gf), gg = tanhf(gc), og = sigm(go);
    const float ck = c_prev[e] * keep[r];
    const float cn = fg * ck + ig * gg;
    c[e] = cn;
    const float hn = og * tanhf(cn);
    h[e] = hn;
    if (keep_next) hk[e] = hn * keep_next[r];
    float* a = act + r * 4 * H;
    a[u] = ig;
    a[H + u] = fg;
    a[2 * H + u] = gg;
    a[3 * H + u] = og;
}

// dh, dc: gradients of the step's h and c outputs (dc may be null: zero);
// dG [m][4H] the gate pre-activations' gradient, dc_prev [m][H] c_prev's
// Sequence steps (salp_lstm_step_backward): dh = d_out + dhk_next keep_next
// (the gradient through the next step's GEMM operand, when dhk_next is not null).
__global__ __launch_bounds__(256) void k_lstm_bwd(int64_t m, int H, const float* __restrict__ act,
                                                  const float* __restrict__ c_prev, const float* __restrict__ keep,
                                                  const float* __restrict__ c, const float* __restrict__ dh,
                                                  const float* __restrict__ dhk_next,
                                                  const float* __restrict__ keep_next,
                                                  const float* __restrict__ dc, float* __restrict__ dG,
                                                  float* __restrict__ dc_prev) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= m * H) return;
    const int64_t r = e / H;
    const int u = (int)(e - r * H);
    const float* a = act + r * 4 * H;
    const float ig = a[u], fg = a[H + u], gg = a[2 * H + u], og = a[3 * H + u];
    const float kp = keep[r];
    const float ck = c_prev[e] * kp;
    const float tc = tanhf(c[e]);
    const float dhe = dhk_next ? dh[e] + dhk_next[e] * keep_next[r] : dh[e];
    const float dcn = (dc ? dc[e] : 0.0f) + dhe * og * (1.0f - tc * tc);
    float* d = dG + r * 4 * H;
    d[u] = dcn * gg * ig * (1.0f - ig);
    d[H + u] = dcn * ck * fg * (1.0f - fg);
    d[2 * H + u] = dcn * ig * (1.0f - gg * gg);
    d[3 * H + u] = dhe * tc * og * (1.0f - og);
    dc_prev[e] = dcn * fg * kp;
}

}  // namespace

extern "C" __attribute__((visibility("hidden"))) hipError_t salp_lstm_fwd_launch(
    int64_t m, int H, const float* G, const float* GX, const float* c_prev, const float* keep, const float* keep_next,
    float* h, float* c, float* act, float* hk, void* stream) {
    const int64_t n = m * H;
    hipLaunchKernelGGL(k_lstm_fwd, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, m, H, G, GX,
                       c_prev, keep, keep_next, h, c, act, hk);
    return hipGetLastError();
}
extern "C" __attribute__((visibility("hidden"))) hipError_t salp_lstm_bwd_launch(
    int64_t m, int H, const float* act, const float* c_prev, const float* keep, const float* c, const float* dh,
    const float* dhk_next, const float* keep_next, const float* dc, float* dG, float* dc_prev, void* stream) {
    const int64_t n = m * H;
    hipLaunchKernelGGL(k_lstm_bwd, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, m, H,
                       act, c_prev, keep, c, dh, dhk_next, keep_next, dc, dG, dc_prev);
    return hipGetLastError();
}
