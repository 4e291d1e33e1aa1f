// Probe: is the VOP3 output modifier (div:2) honoured by f64 VALU ops on gfx950, and
// does it depend on the f64 denormal mode?  hipcc --offload-arch=gfx950 omod_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void probe(const double* in, double* out) {
    const double a = in[0], b = in[1], c = in[2];
    double o0, o1, o2, o3;
    asm volatile("v_fma_f64 %0, %1, %2, %3 div:2" : "=v"(o0) : "v"(a), "v"(b), "v"(c));
    asm volatile("v_add_f64 %0, %1, |%1| div:2" : "=v"(o1) : "v"(c));
    asm volatile("v_fma_f64 %0, -%1, %2, 1.0 div:2" : "=v"(o2) : "v"(a), "v"(b));
    asm volatile("v_mul_f64 %0, %1, %2 mul:2" : "=v"(o3) : "v"(a), "v"(b));
    if (threadIdx.x == 0) {
        out[0] = o0; out[1] = o1; out[2] = o2; out[3] = o3;
        out[4] = (a * b + c) * 0.5; out[5] = (c + __builtin_fabs(c)) * 0.5;
        out[6] = (1.0 - a * b) * 0.5; out[7] = a * b * 2.0;
    }
}

int main() {
    double h[3] = {1.5, 0.75, -3.25}, *d, *o, r[8];
    hipMalloc(&d, sizeof h);
    hipMalloc(&o, sizeof r);
    hipMemcpy(d, h, sizeof h, hipMemcpyHostToDevice);
    probe<<<1, 64>>>(d, o);
    hipMemcpy(r, o, sizeof r, hipMemcpyDeviceToHost);
    const char* nm[4] = {"fma div:2", "add|abs| div:2", "fma(-a,b,1) div:2", "mul mul:2"};
    int bad = 0;
    for (int k = 0; k < 4; ++k) {
        printf("%-20s got %.17g want %.17g %s\n", nm[k], r[k], r[k + 4], r[k] == r[k + 4] ? "ok" : "DIFF");
        bad += r[k] != r[k + 4];
    }
    return bad;
}
