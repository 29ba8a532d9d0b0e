// fp64 FMA issue rate per SIMD against waves per SIMD and independent chains.
// Workgroups of one wave; LDS padding sets how many share a CU (4 / 8 / 16 per
// CU = 1 / 2 / 4 waves per SIMD).  Each lane runs CH independent fp64 FMA
// chains.  Prints cycles per wave-instruction per SIMD (lower is better; a
// wave64 fp64 FMA at the full 16 lanes / cycle / SIMD is 4).
// Build: hipcc -O3 --offload-arch=gfx950 -o fp64_issue_probe fp64_issue_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>

template <int CH, int PAD>
__global__ __launch_bounds__(64) void k_fma(double* out, int iters) {
    __shared__ double pad[PAD];
    const int lane = threadIdx.x;
    if (lane == 0) pad[0] = 0.0;
    double a[CH];
#pragma unroll
    for (int k = 0; k < CH; ++k) a[k] = lane + k;
    const double m = 0.999999, c = 1e-7;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int r = 0; r < 128 / CH; ++r)
#pragma unroll
            for (int k = 0; k < CH; ++k) a[k] = fma(a[k], m, c);
    }
    double s = pad[0];
#pragma unroll
    for (int k = 0; k < CH; ++k) s += a[k];
    out[blockIdx.x * 64 + lane] = s;
}

template <int CH, int PAD>
void run(int cus, int per_simd, int clk_khz, double* out) {
    const int blocks = cus * 4 * per_simd, iters = 2048;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    k_fma<CH, PAD><<<blocks, 64>>>(out, iters);
    (void)hipDeviceSynchronize();
    float best = 1e30f;
    for (int r = 0; r < 5; ++r) {
        (void)hipEventRecord(e0);
        k_fma<CH, PAD><<<blocks, 64>>>(out, iters);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        best = ms < best ? ms : best;
    }
    // wave-instructions per SIMD = per_simd waves x iters x 128
    const double per_simd_instr = (double)per_simd * iters * 128;
    const double cyc = best * 1e-3 * clk_khz * 1e3 / per_simd_instr;
    printf("{\"waves_per_simd\": %d, \"chains\": %d, \"ms\": %.4f, \"cycles_per_fma_per_simd\": %.3f}\n", per_simd, CH,
           best, cyc);
}

int main() {
    int cus = 0, clk = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    (void)hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, 0);
    double* out;
    (void)hipMalloc(&out, sizeof(double) * cus * 16 * 64);
    // LDS per workgroup: 40000 B -> 4 per CU, 20000 B -> 8, 10000 B -> 16
    run<8, 5000>(cus, 1, clk, out);
    run<16, 5000>(cus, 1, clk, out);
    run<32, 5000>(cus, 1, clk, out);
    run<8, 2500>(cus, 2, clk, out);
    run<16, 2500>(cus, 2, clk, out);
    run<8, 1250>(cus, 4, clk, out);
    run<16, 1250>(cus, 4, clk, out);
    (void)hipFree(out);
    return 0;
}
