// Does a wave with part of its exec mask off issue fp64 VALU work faster?
// One wave per SIMD (1024 workgroups of 64 threads, 1 per SIMD by LDS),
// each active lane runs 8 independent fp64 FMA chains; lanes >= ACTIVE
// return at once.  Prints ms per launch and cycles per VALU instruction for
// 64, 32, 16 and 1 active lanes.  Build: hipcc -O3 --offload-arch=gfx950.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ __launch_bounds__(64) void k_fma(double* out, int iters, int active) {
    __shared__ double pad[5000];   // > 160 KB / 5: at most 4 workgroups (one per SIMD) per CU
    const int lane = threadIdx.x;
    if (lane == 0) pad[0] = 0.0;
    if (lane >= active) return;
    double a0 = lane, a1 = lane + 1, a2 = lane + 2, a3 = lane + 3, a4 = lane + 4, a5 = lane + 5, a6 = lane + 6,
           a7 = lane + 7;
    const double m = 0.999999, c = 1e-7;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            a0 = fma(a0, m, c); a1 = fma(a1, m, c); a2 = fma(a2, m, c); a3 = fma(a3, m, c);
            a4 = fma(a4, m, c); a5 = fma(a5, m, c); a6 = fma(a6, m, c); a7 = fma(a7, m, c);
        }
    }
    out[blockIdx.x * 64 + lane] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + pad[0];
}

int main() {
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const int blocks = cus * 4, iters = 4096;
    double* out;
    hipMalloc(&out, sizeof(double) * blocks * 64);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    int clk = 0;
    hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, 0);   // kHz
    const int actives[] = {64, 48, 32, 16, 1};
    for (int active : actives) {
        k_fma<<<blocks, 64>>>(out, iters, active);
        hipDeviceSynchronize();
        float best = 1e30f;
        for (int r = 0; r < 5; ++r) {
            hipEventRecord(e0);
            k_fma<<<blocks, 64>>>(out, iters, active);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            best = ms < best ? ms : best;
        }
        const double instr = (double)iters * 16 * 8;   // fp64 FMAs per wave
        const double cyc = best * 1e-3 * clk * 1e3 / instr;
        printf("{\"active_lanes\": %d, \"ms\": %.4f, \"cycles_per_fma\": %.3f, \"waves\": %d, \"clock_khz\": %d}\n",
               active, best, cyc, blocks, clk);
    }
    hipFree(out);
    return 0;
}
