// solve_bench.hip — time the fp64 Cholesky factor + solve variants on one MI355X.
//   hipcc --offload-arch=gfx950 -O3 tools/solve_bench.hip -lrocsolver -lrocblas -o tools/bin/solve_bench
//   tools/bin/solve_bench N [nb ...]
// Matrix: A_ij = 1/(1 + |i - j|) off the diagonal, 64 on it (diagonally dominant: SPD);
// the column-major upper triangle (= the row-major lower triangle the reference leaves
// NaN) is NaN, as in the production Kxx.  b = A·1, so the solution is x = 1.
// Variants: rocSOLVER dpotrf_64 (+ dpotrs_64, 10 right-hand sides); blocked right-looking
// Cholesky on the lower triangle with panel nb: dpotrf of the diagonal block, dtrsm of the
// panel below it, then the trailing update as dsyrk, or as dgemm column panels (which also
// write the NaN upper part of each diagonal block — never read).
#include <hip/hip_runtime.h>
#include <rocblas/rocblas.h>
#include <rocsolver/rocsolver.h>

#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define H(c) do { hipError_t e = (c); if (e) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)
#define B(c) do { rocblas_status e = (c); if (e) { printf("BLAS %s @%d\n", rocblas_status_to_string(e), __LINE__); exit(1); } } while (0)

__global__ void fill(double* a, long long n, int nan_upper) {
    const long long tot = n * n;
    for (long long k = blockIdx.x * (long long)blockDim.x + threadIdx.x; k < tot;
         k += (long long)gridDim.x * blockDim.x) {
        const long long col = k / n, row = k - col * n;
        double v = row == col ? 64.0 : 1.0 / (1.0 + (double)llabs(row - col));
        if (nan_upper && row < col) v = __builtin_nan("");
        a[k] = v;
    }
}
__global__ void rhs(const double* b1, double* b, long long n, int nrhs) {
    for (long long k = blockIdx.x * (long long)blockDim.x + threadIdx.x; k < n * nrhs;
         k += (long long)gridDim.x * blockDim.x)
        b[k] = b1[k % n];
}

static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

struct Ctx {
    rocblas_handle h;
    hipStream_t s;
    double* A;
    double* b;     // n × nrhs
    double* b1;    // A·1
    int64_t* info;
    long long n;
    int nrhs = 10;
};

static void setup(Ctx& c) {
    hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, c.s, c.A, c.n, 0);
    double one = 1.0, zero = 0.0;
    double* ones;
    H(hipMallocAsync(&ones, c.n * 8, c.s));
    std::vector<double> h(c.n, 1.0);
    H(hipMemcpyAsync(ones, h.data(), c.n * 8, hipMemcpyHostToDevice, c.s));
    B(rocblas_dgemv_64(c.h, rocblas_operation_none, c.n, c.n, &one, c.A, c.n, ones, 1, &zero,
                       c.b1, 1));
    H(hipFreeAsync(ones, c.s));
    hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, c.s, c.A, c.n, 1);
    hipLaunchKernelGGL(rhs, dim3(256), dim3(256), 0, c.s, c.b1, c.b, c.n, c.nrhs);
    H(hipStreamSynchronize(c.s));
}

static double check(Ctx& c) {
    std::vector<double> x(c.n * c.nrhs);
    H(hipMemcpy(x.data(), c.b, x.size() * 8, hipMemcpyDeviceToHost));
    double w = 0;
    for (double v : x) w = std::fmax(w, std::fabs(v - 1.0));
    return w;
}

static double solve_trsm(Ctx& c) {     // L y = b, Lᵀ x = y
    const double one = 1.0;
    H(hipStreamSynchronize(c.s));
    double t = now();
    B(rocblas_dtrsm_64(c.h, rocblas_side_left, rocblas_fill_lower, rocblas_operation_none,
                       rocblas_diagonal_non_unit, c.n, c.nrhs, &one, c.A, c.n, c.b, c.n));
    B(rocblas_dtrsm_64(c.h, rocblas_side_left, rocblas_fill_lower, rocblas_operation_transpose,
                       rocblas_diagonal_non_unit, c.n, c.nrhs, &one, c.A, c.n, c.b, c.n));
    H(hipStreamSynchronize(c.s));
    return now() - t;
}

static void blocked(Ctx& c, long long nb, int mode, long long panel) {
    const double one = 1.0, mone = -1.0;
    const long long n = c.n;
    for (long long k = 0; k < n; k += nb) {
        const long long kb = std::min(nb, n - k);
        double* A11 = c.A + k * n + k;
        B(rocsolver_dpotrf_64(c.h, rocblas_fill_lower, kb, A11, n, c.info));
        const long long m = n - k - kb;
        if (m <= 0) break;
        double* A21 = c.A + k * n + (k + kb);
        double* A22 = c.A + (k + kb) * n + (k + kb);
        B(rocblas_dtrsm_64(c.h, rocblas_side_right, rocblas_fill_lower, rocblas_operation_transpose,
                           rocblas_diagonal_non_unit, m, kb, &one, A11, n, A21, n));
        if (mode == 0) {
            B(rocblas_dsyrk_64(c.h, rocblas_fill_lower, rocblas_operation_none, m, kb, &mone, A21,
                               n, &one, A22, n));
        } else {
            // column panels of the trailing matrix: C[j:, j:j+w] -= A21[j:] A21[j:j+w]ᵀ
            for (long long j = 0; j < m; j += panel) {
                const long long w = std::min(panel, m - j);
                B(rocblas_dgemm_64(c.h, rocblas_operation_none, rocblas_operation_transpose,
                                   m - j, w, kb, &mone, A21 + j, n, A21 + j, n, &one,
                                   A22 + j * n + j, n));
            }
        }
    }
}

int main(int argc, char** argv) {
    Ctx c;
    c.n = argc > 1 ? atoll(argv[1]) : 60000;
    std::vector<long long> nbs;
    for (int k = 2; k < argc; ++k) nbs.push_back(atoll(argv[k]));
    if (nbs.empty()) nbs = {512, 1024, 2048};
    H(hipStreamCreate(&c.s));
    B(rocblas_create_handle(&c.h));
    B(rocblas_set_stream(c.h, c.s));
    H(hipMalloc(&c.A, c.n * c.n * 8));
    H(hipMalloc(&c.b, c.n * c.nrhs * 8));
    H(hipMalloc(&c.b1, c.n * 8));
    H(hipMalloc(&c.info, 8));
    const double fl = (double)c.n * c.n * c.n / 3.0;
    // dgemm rate reference
    {
        const long long g = 8192;
        double one = 1.0, zero = 0.0;
        for (int r = 0; r < 3; ++r) {
            H(hipStreamSynchronize(c.s));
            double t = now();
            B(rocblas_dgemm_64(c.h, rocblas_operation_none, rocblas_operation_transpose, g, g, g,
                               &one, c.A, g, c.A + g * g, g, &zero, c.A + 2 * g * g, g));
            H(hipStreamSynchronize(c.s));
            t = now() - t;
            if (r == 2) printf("dgemm %lld^3: %.2f ms %.1f TF\n", g, t * 1e3, 2.0 * g * g * g / t / 1e12);
        }
    }
    for (int rep = 0; rep < 2; ++rep) {
        setup(c);
        double t = now();
        B(rocsolver_dpotrf_64(c.h, rocblas_fill_lower, c.n, c.A, c.n, c.info));
        H(hipStreamSynchronize(c.s));
        double tf = now() - t;
        t = now();
        B(rocsolver_dpotrs_64(c.h, rocblas_fill_lower, c.n, c.nrhs, c.A, c.n, c.b, c.n));
        H(hipStreamSynchronize(c.s));
        double ts = now() - t;
        int64_t info;
        H(hipMemcpy(&info, c.info, 8, hipMemcpyDeviceToHost));
        printf("rocsolver n=%lld potrf %.3f s (%.1f TF) potrs %.4f s info %lld err %.2e\n", c.n, tf,
               fl / tf / 1e12, ts, (long long)info, check(c));
        fflush(stdout);
    }
    for (int mode = 0; mode < 2; ++mode) {
        for (long long nb : nbs) {
            for (long long panel : (mode ? std::vector<long long>{4096, 8192} : std::vector<long long>{0})) {
                setup(c);
                double t = now();
                blocked(c, nb, mode, panel);
                H(hipStreamSynchronize(c.s));
                double tf = now() - t;
                int64_t info;
                H(hipMemcpy(&info, c.info, 8, hipMemcpyDeviceToHost));
                double ts = solve_trsm(c);
                printf("blocked %s nb=%lld panel=%lld potrf %.3f s (%.1f TF) trsm-solve %.4f s info %lld err %.2e\n",
                       mode ? "gemm" : "syrk", nb, panel, tf, fl / tf / 1e12, ts, (long long)info, check(c));
                fflush(stdout);
            }
        }
    }
    return 0;
}
