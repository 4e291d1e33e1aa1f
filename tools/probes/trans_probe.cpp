// Issue cost of the fp64 ops the closed-form ReLU uses (v_rsq_f64, v_fma_f64, v_mul_f64,
// v_min_f64) on gfx950: every thread runs 8 independent chains of K dependent ops; the
// cycles per wave-instruction follow from the wall time at full occupancy.
//   hipcc -O3 --offload-arch=gfx950 tools/probes/trans_probe.cpp -o /tmp/trans_probe
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int K = 256;

template <int OP>
__global__ __launch_bounds__(256) void probe(double* out, double seed) {
    double v[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) v[c] = seed + threadIdx.x * 1e-3 + c;
    for (int k = 0; k < K; ++k) {
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            if constexpr (OP == 0) v[c] = __builtin_amdgcn_rsq(v[c]);
            if constexpr (OP == 1) v[c] = __builtin_fma(v[c], 0.999999, 1e-9);
            if constexpr (OP == 2) v[c] = __builtin_amdgcn_rsqf((float)v[c]);
            if constexpr (OP == 3) v[c] = __builtin_amdgcn_sqrt(v[c]);
            if constexpr (OP == 4) v[c] = __builtin_amdgcn_rcp(v[c]);
        }
    }
    double s = 0;
#pragma unroll
    for (int c = 0; c < 8; ++c) s += v[c];
    if (s == 12345.0) out[threadIdx.x] = s;
}

template <int OP>
double run(const char* name, int cus) {
    double* d;
    hipMalloc(&d, 1024 * sizeof(double));
    const int blocks = cus * 8;                 // 8 x 4 waves per CU
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipLaunchKernelGGL(probe<OP>, dim3(blocks), dim3(256), 0, 0, d, 1.5);
    hipEventRecord(a);
    const int reps = 20;
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(probe<OP>, dim3(blocks), dim3(256), 0, 0, d, 1.5);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    // wave-instructions per SIMD: blocks*4 waves / (cus*4 SIMDs) * K * 8
    const double winst = (double)blocks * 4 / (cus * 4) * K * 8 * reps;
    int clk_khz = 0;
    hipDeviceGetAttribute(&clk_khz, hipDeviceAttributeClockRate, 0);
    const double cycles = ms * 1e-3 * clk_khz * 1e3;
    printf("%-10s %7.3f ms  %6.2f cycles per wave-instruction (clock %d MHz)\n", name, ms,
           cycles / winst, clk_khz / 1000);
    hipFree(d);
    return cycles / winst;
}

int main() {
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    run<1>("fma_f64", cus);
    run<0>("rsq_f64", cus);
    run<3>("sqrt_f64", cus);
    run<4>("rcp_f64", cus);
    run<2>("rsq_f32", cus);
    return 0;
}
