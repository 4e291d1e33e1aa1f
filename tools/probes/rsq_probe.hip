// Accuracy of v_rsq_f64 / v_rsq_f32 with 0, 1, 2 Newton steps against 1/sqrt in
// long double on the host.  Diagnostic only (tools/, not the product).
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <random>
#include <vector>

__global__ void probe(const double* x, double* out, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    double t = x[i];
    double y = __builtin_amdgcn_rsq(t);
    out[3 * i] = y;
    double e = __builtin_fma(-t * y, y, 1.0);
    double y1 = __builtin_fma(0.5 * y, e, y);
    out[3 * i + 1] = y1;
    e = __builtin_fma(-t * y1, y1, 1.0);
    out[3 * i + 2] = __builtin_fma(0.5 * y1, e, y1);
}
__global__ void probef(const float* x, float* out, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float t = x[i];
    float y = __builtin_amdgcn_rsqf(t);
    out[2 * i] = y;
    float e = __builtin_fmaf(-t * y, y, 1.0f);
    out[2 * i + 1] = __builtin_fmaf(0.5f * y, e, y);
}
int main() {
    const int n = 1 << 22;
    std::mt19937_64 g(1);
    std::uniform_real_distribution<double> u(-300, 300), uf(-37, 37);
    std::vector<double> x(n), o(3 * n);
    std::vector<float> xf(n), of(2 * n);
    for (int i = 0; i < n; ++i) { x[i] = std::pow(10.0, u(g)); xf[i] = (float)std::pow(10.0, uf(g)); }
    double *dx, *dout; float *fx, *fout;
    hipMalloc(&dx, n * 8); hipMalloc(&dout, 3 * n * 8); hipMalloc(&fx, n * 4); hipMalloc(&fout, 2 * n * 4);
    hipMemcpy(dx, x.data(), n * 8, hipMemcpyHostToDevice);
    hipMemcpy(fx, xf.data(), n * 4, hipMemcpyHostToDevice);
    probe<<<n / 256, 256>>>(dx, dout, n);
    probef<<<n / 256, 256>>>(fx, fout, n);
    hipMemcpy(o.data(), dout, 3 * n * 8, hipMemcpyDeviceToHost);
    hipMemcpy(of.data(), fout, 2 * n * 4, hipMemcpyDeviceToHost);
    double w[3] = {0, 0, 0}, wf[2] = {0, 0};
    for (int i = 0; i < n; ++i) {
        long double r = 1.0L / std::sqrt((long double)x[i]);
        for (int k = 0; k < 3; ++k) w[k] = std::fmax(w[k], (double)std::fabs((o[3 * i + k] - r) / r));
        long double rf = 1.0L / std::sqrt((long double)xf[i]);
        for (int k = 0; k < 2; ++k) wf[k] = std::fmax(wf[k], (double)std::fabs((of[2 * i + k] - rf) / rf));
    }
    printf("f64 rsq max rel err: raw %.3e  1 newton %.3e  2 newton %.3e  (ulp 1.1e-16)\n", w[0], w[1], w[2]);
    printf("f32 rsq max rel err: raw %.3e  1 newton %.3e  (ulp 6e-8)\n", wf[0], wf[1]);
    return 0;
}
