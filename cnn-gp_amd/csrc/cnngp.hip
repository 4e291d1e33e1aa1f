// cnngp.hip — MI355X (gfx950) kernels for the CNN-GP Gram recursion + the C ABI of
// include/cnngp.h.  Written for CDNA4 directly: wave64, LDS-staged map chunks, one HBM
// pass per fused op.  Reference semantics are cited as /root/reference/<file>:<line>.
//
// Data layout: a tile's pair maps are one dense [nmaps][H][W] block in
// HBM (m = i·N2 + j, or m = i for diag tiles); per-image variance maps are
// [N1][H][W] / [N2][H][W].  Every kernel works on CHUNKS of whole maps per workgroup,
// so all index math inside a chunk is 32-bit and the chunk's HBM bytes are one
// contiguous, fully coalesced range.

#include <hip/hip_runtime.h>
#include <rocblas/rocblas.h>
#include <rocsolver/rocsolver.h>

#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <map>
#include <mutex>
#include <string>

#include "cnngp.h"

namespace {

// ----------------------------------------------------------------------------------
// error plumbing (no exceptions cross the ABI)
// ----------------------------------------------------------------------------------
thread_local std::string g_last_error;

int fail(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_last_error = buf;
    return code;
}

int check_launch(const char* what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(CGP_EHIP, "%s: %s", what, hipGetErrorString(e));
    return CGP_OK;
}

#define CGP_HIP(call)                                                                  \
    do {                                                                               \
        hipError_t e_ = (call);                                                        \
        if (e_ != hipSuccess)                                                          \
            return fail(CGP_EHIP, "%s: %s (%s:%d)", #call, hipGetErrorString(e_),      \
                        __FILE__, __LINE__);                                           \
    } while (0)

constexpr int kBlock = 256;          // 4 waves of 64
constexpr int kChunkElems = 2048;    // target map elements per workgroup chunk
constexpr int kMaxLds = 64 * 1024;   // bytes of LDS one conv workgroup may take

// ----------------------------------------------------------------------------------
// the ReLU covariance map (kernels.py:133-152), mirrored op by op: separate roundings
// (this file is compiled with -ffp-contract=off), torch's clamp NaN propagation,
// rsqrt as 1/sqrt (ATen's CPU rsqrt), and float constants rounded to T like torch's
// wrapped Python scalars.
// ----------------------------------------------------------------------------------
template <typename T> struct K;
template <> struct K<double> {
    static constexpr double pi = 3.141592653589793;
    static constexpr double two_pi = 6.283185307179586;
    static constexpr double tiny = 1.1754943508222875e-38;   // np.finfo(np.float32).tiny
};
template <> struct K<float> {
    static constexpr float pi = 3.14159265358979f;
    static constexpr float two_pi = 6.28318530717959f;
    static constexpr float tiny = 1.17549435e-38f;
};

__device__ __forceinline__ double sqrt_t(double x) { return __builtin_sqrt(x); }
__device__ __forceinline__ float sqrt_t(float x) { return __builtin_sqrtf(x); }
__device__ __forceinline__ double acos_t(double x) { return acos(x); }
__device__ __forceinline__ float acos_t(float x) { return acosf(x); }

template <typename T>
__device__ __forceinline__ T relu_cov(T c, T v1, T v2) {
    const T t = v1 * v2 + K<T>::tiny;                       // :146
    T cs = c * (T(1) / sqrt_t(t));                          // :149
    cs = cs < T(-1) ? T(-1) : (cs > T(1) ? T(1) : cs);      // clamp(-1, 1), NaN kept
    T d = t - c * c;                                        // :150
    d = d < T(0) ? T(0) : d;                                // clamp(min=0)
    const T s = sqrt_t(d);
    const T th = acos_t(cs);                                // :151
    return (s + (K<T>::pi - th) * c) / K<T>::two_pi;        // :152
}

// ReLU of pair map m at pixel px with the same/diag overrides of kernels.py:155-162.
template <typename T>
__device__ __forceinline__ T relu_pair(T c, const T* __restrict__ xx, const T* __restrict__ yy,
                                       unsigned i, unsigned j, int hw, int px, int same,
                                       int diag) {
    const T v1 = xx[(size_t)i * hw + px];
    if (same && (diag || i == j)) return v1 / T(2);          // xy' = xx' = xx/2
    const T v2 = yy[(size_t)j * hw + px];
    return relu_cov(c, v1, v2);
}

// pair index -> (i, j)
__device__ __forceinline__ void pair_of(unsigned m, unsigned n2, int diag, unsigned& i,
                                        unsigned& j) {
    if (diag) {
        i = j = m;
    } else {
        i = m / n2;
        j = m - i * n2;
    }
}

// ----------------------------------------------------------------------------------
// kernel parameter blocks (device side, by value)
// ----------------------------------------------------------------------------------
template <typename T>
struct ConvP {
    const T* in;
    const T* in_y;
    T* out;
    const T* addend;
    const T* pre_xx;
    const T* pre_yy;
    const T* post_xx;
    const T* post_yy;
    long long nmaps;
    unsigned n2;
    int h, w, ho, wo;
    int taps, off, stride, dil;
    int channels;
    int same, diag;
    int mpb;        // maps per block
    int hs_offset;  // element offset of the row-sum plane in LDS
    T weight, bias;
};

// ----------------------------------------------------------------------------------
// Conv2d covariance stencil, fused (kernels.py:92-98 [+ :134-165 before/after] [+ Sum]).
// One workgroup = one chunk of `mpb` whole maps:
//   stage 1  HBM -> LDS   (x the optional PRE op: ReLU or input moments)
//   stage 2  LDS -> LDS   row sums over the taps        hs[m][r][ow]
//   stage 3  LDS -> HBM   column sums, ·w + b, optional POST ReLU, optional + addend
// The constant conv weight makes the k×k stencil separable (2k LDS reads per output
// instead of k²), and the chunk's input/output are contiguous HBM ranges read and
// written exactly once.
// ----------------------------------------------------------------------------------
template <typename T, int PRE, int POST, bool ADD>
__global__ __launch_bounds__(kBlock) void conv_cov_kernel(const ConvP<T> p) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    T* tin = reinterpret_cast<T*>(smem);
    T* ths = tin + p.hs_offset;

    const int hw = p.h * p.w;
    const int howo = p.ho * p.wo;
    const long long m0 = (long long)blockIdx.x * p.mpb;
    long long rem = p.nmaps - m0;
    const int mb = rem < p.mpb ? (int)rem : p.mpb;
    const int tid = threadIdx.x;

    // ---- stage 1: stage the chunk's input maps ----
    const int nin = mb * hw;
    if constexpr (PRE == CGP_PRE_MOMENTS) {
        // division by C mirrors torch's mean (sum, then / C)
        for (int e = tid; e < nin; e += kBlock) {
            const int ml = e / hw;
            const int px = e - ml * hw;
            unsigned i, j;
            pair_of((unsigned)(m0 + ml), p.n2, p.diag, i, j);
            const T* xi = p.in + (size_t)i * p.channels * hw + px;
            const T* yj = p.in_y + (size_t)j * p.channels * hw + px;
            T acc = xi[0] * yj[0];
            for (int c = 1; c < p.channels; ++c) acc += xi[(size_t)c * hw] * yj[(size_t)c * hw];
            tin[e] = acc / T(p.channels);
        }
    } else {
        const T* src = p.in + m0 * hw;
        constexpr int U = 4;
        for (int base = tid; base < nin; base += kBlock * U) {
            T v[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int e = base + u * kBlock;
                v[u] = e < nin ? src[e] : T(0);
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int e = base + u * kBlock;
                if (e < nin) {
                    T x = v[u];
                    if constexpr (PRE == CGP_PRE_RELU) {
                        const int ml = e / hw;
                        const int px = e - ml * hw;
                        unsigned i, j;
                        pair_of((unsigned)(m0 + ml), p.n2, p.diag, i, j);
                        x = relu_pair(x, p.pre_xx, p.pre_yy, i, j, hw, px, p.same, p.diag);
                    }
                    tin[e] = x;
                }
            }
        }
    }
    __syncthreads();

    // ---- stage 2: row sums over the horizontal taps ----
    const int nhs = mb * p.h * p.wo;
    for (int e = tid; e < nhs; e += kBlock) {
        const int rr = e / p.wo;            // ml * h + r
        const int ow = e - rr * p.wo;
        const T* row = tin + rr * p.w;
        const int c0 = ow * p.stride + p.off;
        T acc = T(0);
        for (int t = 0; t < p.taps; ++t) {
            const int c = c0 + t * p.dil;
            if ((unsigned)c < (unsigned)p.w) acc += row[c];
        }
        ths[e] = acc;
    }
    __syncthreads();

    // ---- stage 3: column sums, affine, fused epilogue, store ----
    const int nout = mb * howo;
    T* dst = p.out + m0 * howo;
    const T* add = ADD ? p.addend + m0 * howo : nullptr;
    for (int e = tid; e < nout; e += kBlock) {
        const int ml = e / howo;
        const int q = e - ml * howo;
        const int oh = q / p.wo;
        const int ow = q - oh * p.wo;
        const T* col = ths + ml * p.h * p.wo + ow;
        const int r0 = oh * p.stride + p.off;
        T acc = T(0);
        for (int t = 0; t < p.taps; ++t) {
            const int r = r0 + t * p.dil;
            if ((unsigned)r < (unsigned)p.h) acc += col[r * p.wo];
        }
        T v = p.weight * acc + p.bias;
        if constexpr (POST == CGP_POST_RELU) {
            unsigned i, j;
            pair_of((unsigned)(m0 + ml), p.n2, p.diag, i, j);
            v = relu_pair(v, p.post_xx, p.post_yy, i, j, howo, q, p.same, p.diag);
        }
        if constexpr (ADD) v = v + add[e];
        dst[e] = v;
    }
}

// ----------------------------------------------------------------------------------
// standalone ReLU on pair maps (+ optional addend), chunked like the conv
// ----------------------------------------------------------------------------------
template <typename T>
struct ReluP {
    const T* xy;
    T* out;
    const T* addend;
    const T* xx;
    const T* yy;
    long long nmaps;
    unsigned n2;
    int hw, same, diag, mpb;
};

template <typename T, bool ADD>
__global__ __launch_bounds__(kBlock) void relu_pair_kernel(const ReluP<T> p) {
    const long long m0 = (long long)blockIdx.x * p.mpb;
    long long rem = p.nmaps - m0;
    const int mb = rem < p.mpb ? (int)rem : p.mpb;
    const int n = mb * p.hw;
    const T* src = p.xy + m0 * p.hw;
    T* dst = p.out + m0 * p.hw;
    const T* add = ADD ? p.addend + m0 * p.hw : nullptr;
    constexpr int U = 4;
    for (int base = threadIdx.x; base < n; base += kBlock * U) {
        T v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int e = base + u * kBlock;
            v[u] = e < n ? src[e] : T(0);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int e = base + u * kBlock;
            if (e < n) {
                const int ml = e / p.hw;
                const int px = e - ml * p.hw;
                unsigned i, j;
                pair_of((unsigned)(m0 + ml), p.n2, p.diag, i, j);
                T r = relu_pair(v[u], p.xx, p.yy, i, j, p.hw, px, p.same, p.diag);
                if constexpr (ADD) r = r + add[e];
                dst[e] = r;
            }
        }
    }
}

// ReLU on the per-image variances (kernels.py:154-164)
template <typename T>
__global__ __launch_bounds__(kBlock) void var_relu_kernel(const T* __restrict__ xx,
                                                          const T* __restrict__ yy,
                                                          long long n_xx, long long n_yy,
                                                          int same, T* xo, T* yo) {
    const long long stride = (long long)gridDim.x * kBlock;
    for (long long e = (long long)blockIdx.x * kBlock + threadIdx.x; e < n_xx + n_yy;
         e += stride) {
        if (e < n_xx) {
            xo[e] = xx[e] / T(2);
        } else {
            const long long f = e - n_xx;
            yo[f] = same ? xx[f] / T(2) : yy[f] / T(2);
        }
    }
}

// input moments, pair maps (kernels.py:44-47)
template <typename T>
__global__ __launch_bounds__(kBlock) void moments_xy_kernel(const T* __restrict__ x,
                                                            const T* __restrict__ y,
                                                            long long nmaps, unsigned n2,
                                                            int c, int hw, int diag, int mpb,
                                                            T* __restrict__ xy) {
    const long long m0 = (long long)blockIdx.x * mpb;
    long long rem = nmaps - m0;
    const int mb = rem < mpb ? (int)rem : mpb;
    const int n = mb * hw;
    T* dst = xy + m0 * hw;
    for (int e = threadIdx.x; e < n; e += kBlock) {
        const int ml = e / hw;
        const int px = e - ml * hw;
        unsigned i, j;
        pair_of((unsigned)(m0 + ml), n2, diag, i, j);
        const T* xi = x + (size_t)i * c * hw + px;
        const T* yj = y + (size_t)j * c * hw + px;
        T acc = xi[0] * yj[0];
        for (int k = 1; k < c; ++k) acc += xi[(size_t)k * hw] * yj[(size_t)k * hw];
        dst[e] = acc / T(c);
    }
}

// per-image variances (kernels.py:48-49)
template <typename T>
__global__ __launch_bounds__(kBlock) void moments_var_kernel(const T* __restrict__ x,
                                                             const T* __restrict__ y,
                                                             long long n1, long long n2, int c,
                                                             int hw, T* __restrict__ xx,
                                                             T* __restrict__ yy) {
    const long long total = (n1 + n2) * hw;
    const long long stride = (long long)gridDim.x * kBlock;
    for (long long e = (long long)blockIdx.x * kBlock + threadIdx.x; e < total; e += stride) {
        const bool is_x = e < n1 * hw;
        const long long f = is_x ? e : e - n1 * hw;
        const long long img = f / hw;
        const int px = (int)(f - img * hw);
        const T* src = (is_x ? x : y) + (size_t)img * c * hw + px;
        T acc = src[0] * src[0];
        for (int k = 1; k < c; ++k) acc += src[(size_t)k * hw] * src[(size_t)k * hw];
        (is_x ? xx : yy)[f] = acc / T(c);
    }
}

template <typename T>
__global__ __launch_bounds__(kBlock) void axpby_kernel(T alpha, const T* __restrict__ a, T beta,
                                                       const T* __restrict__ b, T* out,
                                                       long long n) {
    const long long stride = (long long)gridDim.x * kBlock;
    for (long long e = (long long)blockIdx.x * kBlock + threadIdx.x; e < n; e += stride) {
        const T pa = alpha * a[e];
        out[e] = b ? pa + beta * b[e] : pa;
    }
}

__global__ __launch_bounds__(kBlock) void cast_kernel(const float* __restrict__ in,
                                                      double* __restrict__ out, long long n) {
    const long long stride = (long long)gridDim.x * kBlock;
    for (long long e = (long long)blockIdx.x * kBlock + threadIdx.x; e < n; e += stride)
        out[e] = (double)in[e];
}

__global__ __launch_bounds__(kBlock) void transpose_kernel(const double* __restrict__ src,
                                                           long long rows, long long cols,
                                                           double* __restrict__ dst) {
    const long long n = rows * cols;
    const long long stride = (long long)gridDim.x * kBlock;
    for (long long e = (long long)blockIdx.x * kBlock + threadIdx.x; e < n; e += stride) {
        const long long r = e / cols, c = e - r * cols;
        dst[c * rows + r] = src[e];
    }
}

__global__ __launch_bounds__(kBlock) void diag_add_kernel(double* k, long long n, long long ld,
                                                          double v) {
    const long long stride = (long long)gridDim.x * kBlock;
    for (long long e = (long long)blockIdx.x * kBlock + threadIdx.x; e < n; e += stride)
        k[e * ld + e] += v;
}

__global__ __launch_bounds__(kBlock) void argmax_rows_kernel(const double* __restrict__ a,
                                                             long long rows, long long cols,
                                                             long long* __restrict__ out) {
    const long long stride = (long long)gridDim.x * kBlock;
    for (long long r = (long long)blockIdx.x * kBlock + threadIdx.x; r < rows; r += stride) {
        const double* row = a + r * cols;
        long long best = 0;
        double bv = row[0];
        for (long long c = 1; c < cols; ++c) {
            const double v = row[c];
            // torch.argmax: NaN is the maximum; otherwise first strict maximum
            if (!(bv != bv) && (v > bv || v != v)) {
                bv = v;
                best = c;
            }
        }
        out[r] = best;
    }
}

// ----------------------------------------------------------------------------------
// host helpers
// ----------------------------------------------------------------------------------
inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

inline unsigned grid_for(long long n) {
    long long g = (n + kBlock - 1) / kBlock;
    if (g > 256 * 8 * 4) g = 256 * 8 * 4;   // ≈4 rounds of 8 blocks per CU, grid-stride rest
    return (unsigned)(g < 1 ? 1 : g);
}

inline int maps_per_chunk(int hw, int requested) {
    if (requested > 0) return requested;
    int m = kChunkElems / hw;
    return m < 1 ? 1 : m;
}

int conv_out_check(const cgp_conv_args* a) {
    if (!a) return fail(CGP_EINVAL, "conv: args is NULL");
    if (!a->in || !a->out) return fail(CGP_EINVAL, "conv: in/out is NULL");
    if (a->nmaps <= 0 || a->nmaps >= (1LL << 31))
        return fail(CGP_EINVAL, "conv: nmaps=%lld out of range", (long long)a->nmaps);
    if (a->h <= 0 || a->w <= 0 || a->ho <= 0 || a->wo <= 0)
        return fail(CGP_EINVAL, "conv: bad spatial sizes %dx%d -> %dx%d", a->h, a->w, a->ho,
                    a->wo);
    if (a->taps <= 0 || a->stride <= 0 || a->dilation <= 0)
        return fail(CGP_EINVAL, "conv: taps/stride/dilation must be positive");
    // the output grid may not run past the high-side padding F.conv2d would have: its
    // padding is symmetric, -offset (+ dilation for an even "same" kernel) per side
    const long long last_r = (long long)(a->ho - 1) * a->stride + a->offset +
                             (long long)(a->taps - 1) * a->dilation;
    const long long last_c = (long long)(a->wo - 1) * a->stride + a->offset +
                             (long long)(a->taps - 1) * a->dilation;
    const long long hi_pad = -(long long)a->offset + a->dilation;
    if (a->offset > 0 || last_r > a->h - 1 + hi_pad || last_c > a->w - 1 + hi_pad)
        return fail(CGP_EINVAL, "conv: output extent %dx%d inconsistent with input %dx%d",
                    a->ho, a->wo, a->h, a->w);
    if (a->pre < CGP_PRE_NONE || a->pre > CGP_PRE_MOMENTS || a->post < 0 ||
        a->post > CGP_POST_RELU)
        return fail(CGP_EINVAL, "conv: bad pre/post op %d/%d", a->pre, a->post);
    const bool pairs = a->pre != CGP_PRE_NONE || a->post != CGP_POST_NONE;
    if (pairs) {
        if (a->n1 <= 0 || a->n2 <= 0 || a->n2 >= (1LL << 31))
            return fail(CGP_EINVAL, "conv: n1/n2 out of range");
        const long long want = a->diag ? a->n1 : a->n1 * a->n2;
        if (want != a->nmaps)
            return fail(CGP_EINVAL, "conv: nmaps=%lld but n1=%lld n2=%lld diag=%d",
                        (long long)a->nmaps, (long long)a->n1, (long long)a->n2, a->diag);
        if (a->diag && a->n1 != a->n2)
            return fail(CGP_EINVAL, "conv: diag needs n1 == n2");
    }
    if (a->pre == CGP_PRE_RELU && (!a->pre_xx || !a->pre_yy))
        return fail(CGP_EINVAL, "conv: PRE_RELU needs pre_xx/pre_yy");
    if (a->pre == CGP_PRE_MOMENTS && (!a->in_y || a->channels <= 0))
        return fail(CGP_EINVAL, "conv: PRE_MOMENTS needs in_y and channels > 0");
    if (a->post == CGP_POST_RELU && (!a->post_xx || !a->post_yy))
        return fail(CGP_EINVAL, "conv: POST_RELU needs post_xx/post_yy");
    if (a->maps_per_block < 0) return fail(CGP_EINVAL, "conv: maps_per_block < 0");
    return CGP_OK;
}

template <typename T, int PRE, int POST, bool ADD>
void launch_conv(const ConvP<T>& p, unsigned grid, size_t lds, hipStream_t s) {
    hipLaunchKernelGGL((conv_cov_kernel<T, PRE, POST, ADD>), dim3(grid), dim3(kBlock), lds, s,
                       p);
}

template <typename T, int PRE, int POST>
void launch_conv_add(const ConvP<T>& p, bool add, unsigned grid, size_t lds, hipStream_t s) {
    if (add)
        launch_conv<T, PRE, POST, true>(p, grid, lds, s);
    else
        launch_conv<T, PRE, POST, false>(p, grid, lds, s);
}

template <typename T>
int conv_impl(const cgp_conv_args* a, void* stream) {
    int rc = conv_out_check(a);
    if (rc) return rc;
    const int hw = a->h * a->w;
    int mpb = maps_per_chunk(hw, a->maps_per_block);
    auto lds_of = [&](int m) {
        const size_t in_elems = ((size_t)m * hw + 1) & ~(size_t)1;   // keep 16-B alignment
        return (in_elems + (size_t)m * a->h * a->wo) * sizeof(T);
    };
    while (mpb > 1 && lds_of(mpb) > (size_t)kMaxLds) --mpb;
    if (lds_of(mpb) > (size_t)kMaxLds)
        return fail(CGP_EINVAL, "conv: one %dx%d map does not fit the LDS budget", a->h, a->w);
    ConvP<T> p;
    p.in = static_cast<const T*>(a->in);
    p.in_y = static_cast<const T*>(a->in_y);
    p.out = static_cast<T*>(a->out);
    p.addend = static_cast<const T*>(a->addend);
    p.pre_xx = static_cast<const T*>(a->pre_xx);
    p.pre_yy = static_cast<const T*>(a->pre_yy);
    p.post_xx = static_cast<const T*>(a->post_xx);
    p.post_yy = static_cast<const T*>(a->post_yy);
    p.nmaps = a->nmaps;
    p.n2 = (unsigned)(a->n2 > 0 ? a->n2 : 1);
    p.h = a->h;
    p.w = a->w;
    p.ho = a->ho;
    p.wo = a->wo;
    p.taps = a->taps;
    p.off = a->offset;
    p.stride = a->stride;
    p.dil = a->dilation;
    p.channels = a->channels;
    p.same = a->same;
    p.diag = a->diag;
    p.mpb = mpb;
    p.hs_offset = (int)(((size_t)mpb * hw + 1) & ~(size_t)1);
    p.weight = (T)a->weight;
    p.bias = (T)a->bias;
    const long long blocks = (a->nmaps + mpb - 1) / mpb;
    if (blocks > 0x7fffffffLL) return fail(CGP_EINVAL, "conv: grid too large");
    const unsigned grid = (unsigned)blocks;
    const size_t lds = lds_of(mpb);
    const bool add = a->addend != nullptr;
    hipStream_t s = as_stream(stream);
    switch (a->pre * 2 + a->post) {
        case CGP_PRE_NONE * 2 + CGP_POST_NONE:
            launch_conv_add<T, CGP_PRE_NONE, CGP_POST_NONE>(p, add, grid, lds, s); break;
        case CGP_PRE_NONE * 2 + CGP_POST_RELU:
            launch_conv_add<T, CGP_PRE_NONE, CGP_POST_RELU>(p, add, grid, lds, s); break;
        case CGP_PRE_RELU * 2 + CGP_POST_NONE:
            launch_conv_add<T, CGP_PRE_RELU, CGP_POST_NONE>(p, add, grid, lds, s); break;
        case CGP_PRE_RELU * 2 + CGP_POST_RELU:
            launch_conv_add<T, CGP_PRE_RELU, CGP_POST_RELU>(p, add, grid, lds, s); break;
        case CGP_PRE_MOMENTS * 2 + CGP_POST_NONE:
            launch_conv_add<T, CGP_PRE_MOMENTS, CGP_POST_NONE>(p, add, grid, lds, s); break;
        case CGP_PRE_MOMENTS * 2 + CGP_POST_RELU:
            launch_conv_add<T, CGP_PRE_MOMENTS, CGP_POST_RELU>(p, add, grid, lds, s); break;
        default:
            return fail(CGP_EINVAL, "conv: bad pre/post");
    }
    return check_launch("conv_cov_kernel");
}

template <typename T>
int relu_impl(const cgp_relu_args* a, void* stream) {
    if (!a || !a->xy || !a->out || !a->xx)
        return fail(CGP_EINVAL, "relu: NULL argument");
    if (a->hw <= 0 || a->nmaps <= 0 || a->nmaps >= (1LL << 31))
        return fail(CGP_EINVAL, "relu: bad sizes");
    if (a->n1 <= 0 || a->n2 <= 0 || (a->diag ? a->n1 : a->n1 * a->n2) != a->nmaps)
        return fail(CGP_EINVAL, "relu: nmaps inconsistent with n1/n2/diag");
    if (a->diag && a->n1 != a->n2) return fail(CGP_EINVAL, "relu: diag needs n1 == n2");
    if (!(a->same && a->diag) && !a->yy) return fail(CGP_EINVAL, "relu: yy is NULL");
    ReluP<T> p;
    p.xy = static_cast<const T*>(a->xy);
    p.out = static_cast<T*>(a->out);
    p.addend = static_cast<const T*>(a->addend);
    p.xx = static_cast<const T*>(a->xx);
    p.yy = static_cast<const T*>(a->yy);
    p.nmaps = a->nmaps;
    p.n2 = (unsigned)a->n2;
    p.hw = a->hw;
    p.same = a->same;
    p.diag = a->diag;
    p.mpb = maps_per_chunk(a->hw, 0);
    const long long blocks = (a->nmaps + p.mpb - 1) / p.mpb;
    hipStream_t s = as_stream(stream);
    if (a->addend)
        hipLaunchKernelGGL((relu_pair_kernel<T, true>), dim3((unsigned)blocks), dim3(kBlock), 0,
                           s, p);
    else
        hipLaunchKernelGGL((relu_pair_kernel<T, false>), dim3((unsigned)blocks), dim3(kBlock),
                           0, s, p);
    return check_launch("relu_pair_kernel");
}

template <typename T>
int var_relu_impl(const T* xx, const T* yy, int64_t n1, int64_t n2, int32_t hw, int32_t same,
                  T* xo, T* yo, void* stream) {
    if (!xx || !yy || !xo || !yo) return fail(CGP_EINVAL, "var_relu: NULL argument");
    if (n1 <= 0 || n2 <= 0 || hw <= 0) return fail(CGP_EINVAL, "var_relu: bad sizes");
    if (same && n1 != n2) return fail(CGP_EINVAL, "var_relu: same needs n1 == n2");
    const long long nx = n1 * hw, ny = n2 * hw;
    hipLaunchKernelGGL((var_relu_kernel<T>), dim3(grid_for(nx + ny)), dim3(kBlock), 0,
                       as_stream(stream), xx, yy, nx, ny, same, xo, yo);
    return check_launch("var_relu_kernel");
}

template <typename T>
int moments_xy_impl(const T* x, const T* y, int64_t n1, int64_t n2, int32_t c, int32_t hw,
                    int32_t diag, T* xy, void* stream) {
    if (!x || !y || !xy) return fail(CGP_EINVAL, "moments_xy: NULL argument");
    if (n1 <= 0 || n2 <= 0 || c <= 0 || hw <= 0) return fail(CGP_EINVAL, "moments_xy: sizes");
    if (diag && n1 != n2) return fail(CGP_EINVAL, "moments_xy: diag needs n1 == n2");
    const long long nmaps = diag ? n1 : n1 * n2;
    if (nmaps >= (1LL << 31)) return fail(CGP_EINVAL, "moments_xy: too many maps");
    const int mpb = maps_per_chunk(hw, 0);
    const long long blocks = (nmaps + mpb - 1) / mpb;
    hipLaunchKernelGGL((moments_xy_kernel<T>), dim3((unsigned)blocks), dim3(kBlock), 0,
                       as_stream(stream), x, y, nmaps, (unsigned)n2, c, hw, diag, mpb, xy);
    return check_launch("moments_xy_kernel");
}

template <typename T>
int moments_var_impl(const T* x, const T* y, int64_t n1, int64_t n2, int32_t c, int32_t hw,
                     T* xx, T* yy, void* stream) {
    if (!x || !y || !xx || !yy) return fail(CGP_EINVAL, "moments_var: NULL argument");
    if (n1 <= 0 || n2 <= 0 || c <= 0 || hw <= 0)
        return fail(CGP_EINVAL, "moments_var: sizes");
    hipLaunchKernelGGL((moments_var_kernel<T>), dim3(grid_for((n1 + n2) * hw)), dim3(kBlock), 0,
                       as_stream(stream), x, y, (long long)n1, (long long)n2, c, hw, xx, yy);
    return check_launch("moments_var_kernel");
}

template <typename T>
int axpby_impl(double alpha, const T* a, double beta, const T* b, T* out, int64_t n,
               void* stream) {
    if (!a || !out || n < 0) return fail(CGP_EINVAL, "axpby: bad arguments");
    if (n == 0) return CGP_OK;
    hipLaunchKernelGGL((axpby_kernel<T>), dim3(grid_for(n)), dim3(kBlock), 0, as_stream(stream),
                       (T)alpha, a, (T)beta, b, out, (long long)n);
    return check_launch("axpby_kernel");
}

// rocBLAS handle per device, created on first use and kept for the process lifetime
std::mutex g_blas_mu;
std::map<int, rocblas_handle> g_blas;

int blas_handle(rocblas_handle* h) {
    int dev = 0;
    CGP_HIP(hipGetDevice(&dev));
    std::lock_guard<std::mutex> lk(g_blas_mu);
    auto it = g_blas.find(dev);
    if (it == g_blas.end()) {
        rocblas_handle nh;
        rocblas_status st = rocblas_create_handle(&nh);
        if (st != rocblas_status_success)
            return fail(CGP_EBLAS, "rocblas_create_handle: %s", rocblas_status_to_string(st));
        it = g_blas.emplace(dev, nh).first;
    }
    *h = it->second;
    return CGP_OK;
}

#define CGP_BLAS(call)                                                                 \
    do {                                                                               \
        rocblas_status st_ = (call);                                                   \
        if (st_ != rocblas_status_success)                                             \
            return fail(CGP_EBLAS, "%s: %s", #call, rocblas_status_to_string(st_));    \
    } while (0)

}  // namespace

// ==================================================================================
// C ABI
// ==================================================================================
extern "C" {

int cgp_abi_version(void) { return CGP_ABI_VERSION; }
const char* cgp_last_error(void) { return g_last_error.c_str(); }
size_t cgp_conv_args_size(void) { return sizeof(cgp_conv_args); }
size_t cgp_relu_args_size(void) { return sizeof(cgp_relu_args); }

int cgp_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) {
        (void)hipGetLastError();
        return 0;
    }
    return n;
}

int cgp_moments_xy_f64(const double* x, const double* y, int64_t n1, int64_t n2, int32_t c,
                       int32_t hw, int32_t diag, double* xy, void* stream) {
    return moments_xy_impl<double>(x, y, n1, n2, c, hw, diag, xy, stream);
}
int cgp_moments_xy_f32(const float* x, const float* y, int64_t n1, int64_t n2, int32_t c,
                       int32_t hw, int32_t diag, float* xy, void* stream) {
    return moments_xy_impl<float>(x, y, n1, n2, c, hw, diag, xy, stream);
}
int cgp_moments_var_f64(const double* x, const double* y, int64_t n1, int64_t n2, int32_t c,
                        int32_t hw, double* xx, double* yy, void* stream) {
    return moments_var_impl<double>(x, y, n1, n2, c, hw, xx, yy, stream);
}
int cgp_moments_var_f32(const float* x, const float* y, int64_t n1, int64_t n2, int32_t c,
                        int32_t hw, float* xx, float* yy, void* stream) {
    return moments_var_impl<float>(x, y, n1, n2, c, hw, xx, yy, stream);
}
int cgp_conv_f64(const cgp_conv_args* args, void* stream) {
    return conv_impl<double>(args, stream);
}
int cgp_conv_f32(const cgp_conv_args* args, void* stream) {
    return conv_impl<float>(args, stream);
}
int cgp_relu_f64(const cgp_relu_args* args, void* stream) {
    return relu_impl<double>(args, stream);
}
int cgp_relu_f32(const cgp_relu_args* args, void* stream) {
    return relu_impl<float>(args, stream);
}
int cgp_var_relu_f64(const double* xx, const double* yy, int64_t n1, int64_t n2, int32_t hw,
                     int32_t same, double* xo, double* yo, void* stream) {
    return var_relu_impl<double>(xx, yy, n1, n2, hw, same, xo, yo, stream);
}
int cgp_var_relu_f32(const float* xx, const float* yy, int64_t n1, int64_t n2, int32_t hw,
                     int32_t same, float* xo, float* yo, void* stream) {
    return var_relu_impl<float>(xx, yy, n1, n2, hw, same, xo, yo, stream);
}
int cgp_axpby_f64(double alpha, const double* a, double beta, const double* b, double* out,
                  int64_t n, void* stream) {
    return axpby_impl<double>(alpha, a, beta, b, out, n, stream);
}
int cgp_axpby_f32(double alpha, const float* a, double beta, const float* b, float* out,
                  int64_t n, void* stream) {
    return axpby_impl<float>(alpha, a, beta, b, out, n, stream);
}

int cgp_cast_f32_f64(const float* in, double* out, int64_t n, void* stream) {
    if (!in || !out || n < 0) return fail(CGP_EINVAL, "cast: bad arguments");
    if (n == 0) return CGP_OK;
    hipLaunchKernelGGL(cast_kernel, dim3(grid_for(n)), dim3(kBlock), 0, as_stream(stream), in,
                       out, (long long)n);
    return check_launch("cast_kernel");
}

int cgp_transpose_f64(const double* src, int64_t rows, int64_t cols, double* dst,
                      void* stream) {
    if (!src || !dst || rows < 0 || cols < 0) return fail(CGP_EINVAL, "transpose: bad args");
    if (rows * cols == 0) return CGP_OK;
    hipLaunchKernelGGL(transpose_kernel, dim3(grid_for(rows * cols)), dim3(kBlock), 0,
                       as_stream(stream), src, (long long)rows, (long long)cols, dst);
    return check_launch("transpose_kernel");
}

int cgp_chol_solve_f64(double* k, int64_t n, int64_t ldk, double* bt, int64_t nrhs,
                       int64_t ldb, double jitter, int64_t* info, void* stream) {
    if (!k || !bt || !info) return fail(CGP_EINVAL, "chol_solve: NULL argument");
    if (n <= 0 || ldk < n || nrhs <= 0 || ldb < n)
        return fail(CGP_EINVAL, "chol_solve: bad sizes n=%lld ldk=%lld nrhs=%lld ldb=%lld",
                    (long long)n, (long long)ldk, (long long)nrhs, (long long)ldb);
    hipStream_t s = as_stream(stream);
    rocblas_handle h;
    int rc = blas_handle(&h);
    if (rc) return rc;
    std::lock_guard<std::mutex> lk(g_blas_mu);
    CGP_BLAS(rocblas_set_stream(h, s));
    if (jitter != 0.0) {
        hipLaunchKernelGGL(diag_add_kernel, dim3(grid_for(n)), dim3(kBlock), 0, s, k,
                           (long long)n, (long long)ldk, jitter);
        rc = check_launch("diag_add_kernel");
        if (rc) return rc;
    }
    int64_t* dinfo = nullptr;
    CGP_HIP(hipMallocAsync(reinterpret_cast<void**>(&dinfo), sizeof(int64_t), s));
    // row-major upper triangle == column-major lower triangle
    rocblas_status st = rocsolver_dpotrf_64(h, rocblas_fill_lower, n, k, ldk, dinfo);
    int64_t hinfo = -1;
    if (st == rocblas_status_success) {
        hipError_t e = hipMemcpyAsync(&hinfo, dinfo, sizeof(int64_t), hipMemcpyDeviceToHost, s);
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        if (e != hipSuccess) {
            (void)hipFreeAsync(dinfo, s);
            return fail(CGP_EHIP, "chol_solve: info readback: %s", hipGetErrorString(e));
        }
    }
    if (st != rocblas_status_success) {
        (void)hipFreeAsync(dinfo, s);
        return fail(CGP_EBLAS, "rocsolver_dpotrf_64: %s", rocblas_status_to_string(st));
    }
    *info = hinfo;
    if (hinfo == 0) {
        st = rocsolver_dpotrs_64(h, rocblas_fill_lower, n, nrhs, k, ldk, bt, ldb);
        if (st != rocblas_status_success) {
            (void)hipFreeAsync(dinfo, s);
            return fail(CGP_EBLAS, "rocsolver_dpotrs_64: %s", rocblas_status_to_string(st));
        }
    }
    CGP_HIP(hipFreeAsync(dinfo, s));
    CGP_HIP(hipStreamSynchronize(s));
    return CGP_OK;
}

int cgp_gemm_f64(const double* a, const double* b, double* c, int64_t m, int64_t n,
                 int64_t kdim, void* stream) {
    if (!a || !b || !c || m <= 0 || n <= 0 || kdim <= 0)
        return fail(CGP_EINVAL, "gemm: bad arguments");
    rocblas_handle h;
    int rc = blas_handle(&h);
    if (rc) return rc;
    std::lock_guard<std::mutex> lk(g_blas_mu);
    CGP_BLAS(rocblas_set_stream(h, as_stream(stream)));
    const double one = 1.0, zero = 0.0;
    CGP_BLAS(rocblas_set_pointer_mode(h, rocblas_pointer_mode_host));
    // row-major C = A·B  <=>  column-major Cᵀ = Bᵀ·Aᵀ
    CGP_BLAS(rocblas_dgemm_64(h, rocblas_operation_none, rocblas_operation_none, n, m, kdim,
                              &one, b, n, a, kdim, &zero, c, n));
    return CGP_OK;
}

int cgp_argmax_rows_f64(const double* a, int64_t rows, int64_t cols, int64_t* out,
                        void* stream) {
    if (!a || !out || rows < 0 || cols <= 0) return fail(CGP_EINVAL, "argmax: bad arguments");
    if (rows == 0) return CGP_OK;
    hipLaunchKernelGGL(argmax_rows_kernel, dim3(grid_for(rows)), dim3(kBlock), 0,
                       as_stream(stream), a, (long long)rows, (long long)cols,
                       reinterpret_cast<long long*>(out));
    return check_launch("argmax_rows_kernel");
}

}  // extern "C"
