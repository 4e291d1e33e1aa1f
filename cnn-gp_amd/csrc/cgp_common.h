// cgp_common.h — device math and host plumbing shared by the libcnngp translation
// units (cnngp.hip: layer-by-layer kernels + C ABI; netfuse.hip: whole-network kernel).
#pragma once

#include <hip/hip_runtime.h>

#include <string>

#include "cnngp.h"
#include "relu_poly.h"

namespace cgp {

// error plumbing (no exceptions cross the ABI); defined in cnngp.hip
int fail(int code, const char* fmt, ...);
int check_launch(const char* what);
// compute units of the current device (cached; launch geometry of persistent kernels)
int device_cus();
inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }
// the device that owns stream s (the current device for the null stream)
inline hipError_t stream_device(hipStream_t s, int* dev) {
    if (s == nullptr) return hipGetDevice(dev);
    hipDevice_t d = 0;
    const hipError_t e = hipStreamGetDevice(s, &d);
    if (e == hipSuccess) *dev = (int)d;
    return e;
}

#define CGP_HIP(call)                                                                  \
    do {                                                                               \
        hipError_t e_ = (call);                                                        \
        if (e_ != hipSuccess)                                                          \
            return fail(CGP_EHIP, "%s: %s (%s:%d)", #call, hipGetErrorString(e_),      \
                        __FILE__, __LINE__);                                           \
    } while (0)


// ----------------------------------------------------------------------------------
// n / d for 0 <= n < 2^31 by multiply-high ("division by invariant integers"):
// q = (umulhi(n, m) + n) >> s with s = ceil(log2 d), m = floor(2^32 (2^s - d) / d) + 1.
// ----------------------------------------------------------------------------------
struct FastDiv {
    unsigned m, s, d;
};
__host__ __device__ inline FastDiv make_fastdiv(unsigned d) {
    FastDiv f;
    f.d = d;
    f.s = 0;
    while ((1ull << f.s) < d) ++f.s;
    f.m = (unsigned)(((1ull << 32) * ((1ull << f.s) - d)) / d + 1);
    return f;
}
__host__ __device__ __forceinline__ unsigned umulhi32(unsigned a, unsigned b) {
#ifdef __HIP_DEVICE_COMPILE__
    return __umulhi(a, b);
#else
    return (unsigned)(((unsigned long long)a * b) >> 32);
#endif
}
__host__ __device__ __forceinline__ unsigned fdiv(unsigned n, const FastDiv& f) {
    return (umulhi32(n, f.m) + n) >> f.s;
}

// ----------------------------------------------------------------------------------
// The ReLU covariance map (kernels.py:133-152).
//
// relu_exact mirrors the reference op by op: separate roundings (this file is compiled
// with -ffp-contract=off), torch's clamp NaN propagation, rsqrt as 1/sqrt (ATen's CPU
// rsqrt), acos, and float constants rounded to T like torch's wrapped Python scalars.
//
// relu_fast is the same map in closed form.  With a = |rho| = |c|/sqrt(t) (clamped) and
// x = (1 - a)/2, acos a = 2 asin sqrt(x) turns (sqrt(t - c²) + (π - acos rho)·c)/2π into
//     max(c, 0)/2 + sqrt(t) · x · sqrt(x) · P(x)
// with P analytic on [0, 1/2] (tools/fit_relu_poly.py; relu_poly.h: monomials in x,
// degree 13, 1.6e-14 relative).
// One branch-free polynomial, two hardware rsq's refined by Newton steps, no division:
// ~35 double ops instead of ~190 slots for correctly rounded div/sqrt/acos.  Near
// |rho| = 1 the reference's own acos(rho) is ill-conditioned (~1e-8 relative noise from
// the last bit of rho); relu_fast evaluates the smooth map there.
// ----------------------------------------------------------------------------------
template <typename T> struct K;
template <> struct K<double> {
    static constexpr double pi = 3.141592653589793;
    static constexpr double two_pi = 6.283185307179586;
    static constexpr double tiny = 1.1754943508222875e-38;   // np.finfo(np.float32).tiny
    static constexpr double xfloor = 1e-300;
};
// (fast path) floors keep rsq finite at x = 0; the product is multiplied by x = 0 anyway
template <> struct K<float> {
    static constexpr float pi = 3.14159265358979f;
    static constexpr float two_pi = 6.28318530717959f;
    static constexpr float tiny = 1.17549435e-38f;
    static constexpr float xfloor = 1e-30f;
};

__device__ __forceinline__ double sqrt_t(double x) { return __builtin_sqrt(x); }
__device__ __forceinline__ float sqrt_t(float x) { return __builtin_sqrtf(x); }
__device__ __forceinline__ double acos_t(double x) { return acos(x); }
__device__ __forceinline__ float acos_t(float x) { return acosf(x); }

template <typename T>
__device__ __forceinline__ T relu_exact_inl(T c, T v1, T v2) {
    const T t = v1 * v2 + K<T>::tiny;                       // :146
    T cs = c * (T(1) / sqrt_t(t));                          // :149
    cs = cs < T(-1) ? T(-1) : (cs > T(1) ? T(1) : cs);      // clamp(-1, 1), NaN kept
    T d = t - c * c;                                        // :150
    d = d < T(0) ? T(0) : d;                                // clamp(min=0)
    const T s = sqrt_t(d);
    const T th = acos_t(cs);                                // :151
    return (s + (K<T>::pi - th) * c) / K<T>::two_pi;        // :152
}
template <typename T>
__device__ __noinline__ T relu_exact(T c, T v1, T v2) {
    return relu_exact_inl(c, v1, v2);
}

// rsqrt(t): hardware estimate refined by one Newton step y += y(1 - t y²)/2.  Measured on
// MI355X (tools/probes/rsq_probe.hip): v_rsq_f64 5.2e-8 -> 4.2e-15 after one step;
// v_rsq_f32 is 9.4e-8 raw (float rounding level), used as is.
__device__ __forceinline__ double rsqrt_fast(double t) {
    const double y = __builtin_amdgcn_rsq(t);
    const double e = __builtin_fma(-t * y, y, 1.0);
    return __builtin_fma(0.5 * y, e, y);
}
__device__ __forceinline__ float rsqrt_fast(float t) { return __builtin_amdgcn_rsqf(t); }
// sqrt(x) from the hardware rsqrt estimate r: s0 = x·r, then one Newton step for the
// root itself, s = s0 + (r/2)(x - s0²) — 4 ops after the rsq instead of 5 for refining
// r and multiplying; same accuracy (the estimate's 5e-8 squares away)
__device__ __forceinline__ double sqrt_fast(double x) {
    const double r = __builtin_amdgcn_rsq(x);
    const double s0 = x * r;
    return __builtin_fma(0.5 * r, __builtin_fma(-s0, s0, x), s0);
}
__device__ __forceinline__ float sqrt_fast(float x) { return x * __builtin_amdgcn_rsqf(x); }
__device__ __forceinline__ double relu_poly(double x) {
    double r = kReluPolyD[kReluPolyDegD];
#pragma unroll
    for (int k = kReluPolyDegD - 1; k >= 0; --k) r = __builtin_fma(r, x, kReluPolyD[k]);
    return r;
}
__device__ __forceinline__ float relu_poly(float x) {
    float r = kReluPolyF[kReluPolyDegF];
#pragma unroll
    for (int k = kReluPolyDegF - 1; k >= 0; --k) r = __builtin_fmaf(r, x, kReluPolyF[k]);
    return r;
}
__device__ __forceinline__ double fmin_t(double a, double b) { return __builtin_fmin(a, b); }
__device__ __forceinline__ float fmin_t(float a, float b) { return __builtin_fminf(a, b); }
__device__ __forceinline__ double fmax_t(double a, double b) { return __builtin_fmax(a, b); }
__device__ __forceinline__ float fmax_t(float a, float b) { return __builtin_fmaxf(a, b); }
__device__ __forceinline__ double fabs_t(double a) { return __builtin_fabs(a); }
__device__ __forceinline__ float fabs_t(float a) { return __builtin_fabsf(a); }
__device__ __forceinline__ double fma_t(double a, double b, double c) {
    return __builtin_fma(a, b, c);
}
__device__ __forceinline__ float fma_t(float a, float b, float c) {
    return __builtin_fmaf(a, b, c);
}

// Polynomial coefficients as SGPR operands.  With compile-time constants the compiler
// pins them in VGPRs and turns every Horner step into v_mov_b64 + v_fmac_f64; read from
// a __constant__ table through a pointer it cannot hoist (poly_table()), each step is one
// v_fma_f64 with an SGPR-pair operand and the table lives in SGPRs only while in use.
// P̃(x4) = P(x4/4)/16: coefficient k scaled by 1/(16·4^k), exact powers of two, so Horner in
// x4 = 4x rounds exactly like Horner in x (relu_q_n)
// x-side variance maps the fp64 closed form reads: v/16 (exact; ABI 9, cgp_net_xvar_scale).
// Its Newton step then yields y = 8/sqrt(t), so u = 4x = 2 - |c/4|·y is one fma with source
// modifiers, sqrt(t)/2 comes out of the same step and the polynomial's coefficients carry
// the factor 2 back (exact).  Rounds 2-3 read v/4 and needed a multiply and a min for u:
// one op more per pixel, measured 0.9-1.4% slower on all three configs
// (profiles/r4/ab_r4m_xvar_scale.log)
constexpr double kXVarScale = 0.0625;
constexpr double kPolyQ = 0.125;   // P̃(x4) = P(x4/4)·kPolyQ·4^-k per coefficient
constexpr double poly_q(int k) {
    double v = kReluPolyD[k] * kPolyQ;
    for (int n = 0; n < k; ++n) v *= 0.25;
    return v;
}
struct PolyCoef {
    double c[kReluPolyDegD + 1];
};
constexpr PolyCoef poly_coef(bool quartered) {
    PolyCoef t{};
    for (int k = 0; k <= kReluPolyDegD; ++k) t.c[k] = quartered ? poly_q(k) : kReluPolyD[k];
    return t;
}
static __constant__ PolyCoef kReluPolyTabD = poly_coef(false);
static __constant__ PolyCoef kReluPolyTabDq = poly_coef(true);

// Range-adaptive ReLU: lower-degree fits of P on x in [0, kReluAdaptX0/1/2] = [0, 1/8],
// [0, 1/4], [0, 3/8], quartered like kReluPolyTabDq.  Default (CGP_RELU_TOL=1, round 5):
// degrees 6, 8, 9 and 11 on [0, 1/2], every fit within 1e-12 of the exact map (2.2e-13 /
// 1.3e-13 / 9.2e-13 / 7.6e-13; ConvNet +2%, mnist_as_tf +1-2.5%, cifar10 +2%,
// profiles/r5/ab_r5d_relu_tol.log); CGP_RELU_TOL=0: degrees 7, 9, 11, 13 at 1.6e-14
// (tools/fit_relu_poly.py ADAPT / ADAPT_TOL).  relu_q_n takes the shortest one whose interval holds every pixel of its
// vote group (a uniform branch).  Deep layers have |rho| near 1 (x small): on MNIST-like
// pairs the ConvNet's ReLUs 2-7 have x <= 0.24 and its last four x <= 0.125.
// Measured and not kept: every degree 6-13 by a binary search of votes, one
// unrolled degree-13 chain entered at the wave's degree, Horner chains as asm blocks.
template <int D>
struct AdaptCoef {
    double c[D + 1];
};
template <int D>
constexpr AdaptCoef<D> adapt_coef(const double (&p)[D + 1]) {
    AdaptCoef<D> t{};
    for (int k = 0; k <= D; ++k) {
        double v = p[k] * kPolyQ;
        for (int n = 0; n < k; ++n) v *= 0.25;
        t.c[k] = v;
    }
    return t;
}
static __constant__ AdaptCoef<kReluAdaptDeg0> kReluAdaptTab0 = adapt_coef<kReluAdaptDeg0>(kReluAdaptP0);
static __constant__ AdaptCoef<kReluAdaptDeg1> kReluAdaptTab1 = adapt_coef<kReluAdaptDeg1>(kReluAdaptP1);
static __constant__ AdaptCoef<kReluAdaptDeg2> kReluAdaptTab2 = adapt_coef<kReluAdaptDeg2>(kReluAdaptP2);

typedef const __attribute__((address_space(4))) double* ConstD;   // scalar-loadable
struct PolyTab {
    ConstD d, dq;
    ConstD a0, a1, a2;
};
__device__ __forceinline__ PolyTab poly_table() {
    ConstD p = (ConstD)kReluPolyTabD.c;
    ConstD q = (ConstD)kReluPolyTabDq.c;
    asm volatile("" : "+s"(p), "+s"(q));
    ConstD a0 = (ConstD)kReluAdaptTab0.c;
    ConstD a1 = (ConstD)kReluAdaptTab1.c;
    ConstD a2 = (ConstD)kReluAdaptTab2.c;
    asm volatile("" : "+s"(a0), "+s"(a1), "+s"(a2));
    return PolyTab{p, q, a0, a1, a2};
}
// r·u + c with c in an SGPR pair: the VOP3 form (the compiler would copy c to VGPRs
// for v_fmac_f64 instead)
__device__ __forceinline__ double fma_sc(double r, double u, double c) {
    double o;
    asm("v_fma_f64 %0, %1, %2, %3" : "=v"(o) : "v"(r), "v"(u), "s"(c));
    return o;
}
__device__ __forceinline__ double relu_poly(double x, const PolyTab& t) {
    double r = fma_sc(t.d[kReluPolyDegD], x, t.d[kReluPolyDegD - 1]);
#pragma unroll
    for (int k = kReluPolyDegD - 2; k >= 0; --k) r = fma_sc(r, x, t.d[k]);
    return r;
}
__device__ __forceinline__ float relu_poly(float x, const PolyTab&) { return relu_poly(x); }

// The same map, trimmed for the whole-network kernel (39 instead of 45 VALU ops):
// t in one rounding (fma), 0.5·max(c, 0) as 0.25·(c + |c|) — exact, and NaN in c
// propagates through the add, so the (c - c) term is not needed.
template <typename T>
__device__ __forceinline__ T relu_fast(T c, T v1, T v2, const PolyTab& tab) {
    const T t = fma_t(v1, v2, K<T>::tiny);
    const T y = rsqrt_fast(t);
    const T st = t * y;                                     // sqrt(t)
    const T a = fmin_t(fabs_t(c * y), T(1));                // |rho| clamped
    const T x = fma_t(T(-0.5), a, T(0.5));                  // (1 - a)/2
    const T sx = sqrt_fast(fmax_t(x, K<T>::xfloor));        // sqrt(x)
    const T p = relu_poly(x, tab);                          // P(x)
    const T hpos = (c + fabs_t(c)) * T(0.25);               // max(c, 0) / 2
    return fma_t((st * x) * sx, p, hpos);
}

// R independent ReLUs evaluated stage by stage (stage-major source order).  The SGPR
// Horner steps are inline asm, which the scheduler keeps in source order, so a per-pixel
// loop would run R dependent 16-step chains back to back; interleaved here, every step
// has R independent FMAs in flight.  Same arithmetic as relu_fast(c, v1, v2, tab).
// |rho| clamped to 1 - 2^-52 (not 1) keeps x = (1 - |rho|)/2 >= 2^-53, so rsq(x) is
// finite without a floor on x: one op less per pixel; where |rho| >= 1 - 2^-52 the x^1.5
// term is below 1e-23 of sqrt(t)
constexpr double kRhoMax = 1.0 - 0x1p-52;
template <int R>
__device__ __forceinline__ void relu_fast_n(double (&c)[R], const double (&v1)[R],
                                            const double (&v2)[R], const PolyTab& tab) {
    double y[R], st[R], a[R], sx[R], u[R], p[R];   // u: x
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const double t = __builtin_fma(v1[r], v2[r], K<double>::tiny);
        y[r] = rsqrt_fast(t);
        st[r] = t * y[r];
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
        a[r] = __builtin_fmin(__builtin_fabs(c[r] * y[r]), kRhoMax);
        u[r] = __builtin_fma(-0.5, a[r], 0.5);
        sx[r] = (st[r] * u[r]) * sqrt_fast(u[r]);
    }
#pragma unroll
    for (int r = 0; r < R; ++r) p[r] = fma_sc(tab.d[kReluPolyDegD], u[r], tab.d[kReluPolyDegD - 1]);
#pragma unroll
    for (int k = kReluPolyDegD - 2; k >= 0; --k) {
        const double ck = tab.d[k];
#pragma unroll
        for (int r = 0; r < R; ++r) p[r] = fma_sc(p[r], u[r], ck);
    }
#pragma unroll
    for (int r = 0; r < R; ++r)
        c[r] = __builtin_fma(sx[r], p[r], (c[r] + __builtin_fabs(c[r])) * 0.25);
}
// The map of relu_fast_n in the form the whole-network kernel runs (28 VALU ops + 2 rsq
// per pixel instead of 31): every 1/2 of the two Newton steps and the output's 1/4 is
// folded into a power-of-two scaling of an input or a coefficient, so each Newton step
// costs 4 ops.  A refinement y = y0(1 + e/2), e = 1 - A·y0², of y0 ≈ rsq(A) is
// y = r·(3 − m·r) with r = rsq(4A) ≈ y0/2 and m = 4A·r — and 4A·r·(3 − m·r) = 4·sqrt(A).
// Inputs, all exact scalings of relu_fast's:
//   v1q = v1/16 (the x-side variance map, scaled by the host: cgp_net_xvar_scale),
//   cq  = c/4   (QIN: the producing conv already applied w/4 and b/4; else one multiply),
// then T = v1q·v2 + tiny/16 = t/16 gives r = rsq(T) ≈ 4/sqrt(t): Y = r·(3 − T·r·r) =
// 8/sqrt(t), T·r·(3 − T·r·r) = sqrt(t)/2, and x4 = 4x = 2 − 2|rho| = 2 − |cq|·Y in one fma
// (round 3 read v/4, got Y = 4/sqrt(t) and spent a multiply and a min on |rho|).  With
// 4·sqrt(x) = x4·h·(3 − x4·h·h), h = rsq(x4), the polynomial term is
// (sqrt(t)/2)·x4·(4 sqrt x)·P̃(x4) with P̃ = P/8 at x4/4, and max(c, 0)/2 = cq + |cq|.
// R interleaved Horner chains of degree D with SGPR coefficients t[0..D]
template <int R, int D>
__device__ __forceinline__ void horner_q(double (&p)[R], const double (&u)[R], ConstD t) {
#pragma unroll
    for (int r = 0; r < R; ++r) p[r] = fma_sc(t[D], u[r], t[D - 1]);
#pragma unroll
    for (int k = D - 2; k >= 0; --k) {
        const double ck = t[k];
#pragma unroll
        for (int r = 0; r < R; ++r) p[r] = fma_sc(p[r], u[r], ck);
    }
}
// AD: 0 the full polynomial; 1 the range-adaptive choice, uniform over the wave (its lanes
// hold the same items of one pair in every workgroup); 2 the choice per vote group: `seg` is
// the mask of this wave's lanes in this lane's vote group (multi-pair stages: a fixed set
// of the pair's items, netfuse.hip vote_lanes), so a pair's polynomial depends on its own
// pixels only and a wave whose groups disagree runs each chosen polynomial under its lanes'
// exec mask
// The vote's interval test on the high 32 bits of u = x4 (u > 0: floored at 2^-51, or NaN):
// for positive doubles the high word is monotone in the value, and the thresholds 0.5 / 1 /
// 1.5 have zero low words, so hi(u) < hi(thr) implies u < thr — conservative (u within
// 2^-20 relative below a threshold, or equal to it, takes the next longer polynomial,
// whose interval also holds it); NaN pixels (high word 0x7ff8…) take the longest one.
// The max over a lane's R pixels is then 32-bit (v_max3_u32: two pixels per instruction)
// instead of R − 1 v_max_f64.  CGP_RELU_VOTE_HI=0 restores the fp64 max.
#ifndef CGP_RELU_VOTE_HI
#define CGP_RELU_VOTE_HI 1
#endif
__device__ __forceinline__ unsigned vote_hi(double v) {
    return (unsigned)(__builtin_bit_cast(unsigned long long, v) >> 32);
}
template <int R>
__device__ __forceinline__ unsigned vote_hi_max(const double (&u)[R]) {
    unsigned m = vote_hi(u[0]);
#pragma unroll
    for (int r = 1; r < R; ++r) m = m > vote_hi(u[r]) ? m : vote_hi(u[r]);
    return m;
}
template <int R, bool QIN, int AD = 0>
__device__ __forceinline__ void relu_q_n(double (&c)[R], const double (&v1q)[R],
                                         const double (&v2)[R], const PolyTab& tab,
                                         unsigned long long seg = ~0ull) {
    double y[R], st[R], sx[R], u[R], p[R];   // u: x4
#pragma unroll
    for (int r = 0; r < R; ++r) {
        if constexpr (!QIN) c[r] *= 0.25;
        const double T = __builtin_fma(v1q[r], v2[r], kXVarScale * K<double>::tiny);
        const double r0 = __builtin_amdgcn_rsq(T);
        const double m = T * r0;
        const double k = __builtin_fma(-m, r0, 3.0);
        y[r] = r0 * k;      // 8/sqrt(t)
        st[r] = m * k;      // sqrt(t)/2
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
        // u = 2 - 2|rho| in one rounding, floored at 2^-51 (|rho| <= 1 - 2^-52, above)
        u[r] = __builtin_fmax(__builtin_fma(-__builtin_fabs(c[r]), y[r], 2.0), 2.0 - 2.0 * kRhoMax);
        const double h = __builtin_amdgcn_rsq(u[r]);
        const double m = u[r] * h;
        const double sq4 = m * __builtin_fma(-m, h, 3.0);
        sx[r] = (st[r] * u[r]) * sq4;
    }
    if constexpr (AD == 2) {
        const unsigned long long ex = __builtin_amdgcn_read_exec() & seg;
        auto all_seg = [&](bool pred) { return (__ballot(pred) & seg) == ex; };
#if CGP_RELU_VOTE_HI
        const unsigned hm = vote_hi_max<R>(u);
        if (all_seg(hm < vote_hi(4.0 * kReluAdaptX0))) {
            horner_q<R, kReluAdaptDeg0>(p, u, tab.a0);
        } else if (all_seg(hm < vote_hi(4.0 * kReluAdaptX1))) {
            horner_q<R, kReluAdaptDeg1>(p, u, tab.a1);
        } else if (all_seg(hm < vote_hi(4.0 * kReluAdaptX2))) {
#else
        double um = u[0];
#pragma unroll
        for (int r = 1; r < R; ++r) um = __builtin_fmax(um, u[r]);
        if (all_seg(um <= 4.0 * kReluAdaptX0)) {
            horner_q<R, kReluAdaptDeg0>(p, u, tab.a0);
        } else if (all_seg(um <= 4.0 * kReluAdaptX1)) {
            horner_q<R, kReluAdaptDeg1>(p, u, tab.a1);
        } else if (all_seg(um <= 4.0 * kReluAdaptX2)) {
#endif
            horner_q<R, kReluAdaptDeg2>(p, u, tab.a2);
        } else {
            horner_q<R, kReluPolyDegD>(p, u, tab.dq);
        }
    } else if constexpr (AD == 1) {
        // the largest x4 = 4x of the lane's pixels; the wave takes the shortest polynomial
        // whose interval holds every active lane's pixels (x4 <= 4·kReluAdaptX)
#if CGP_RELU_VOTE_HI
        const unsigned hm = vote_hi_max<R>(u);
        if (__all(hm < vote_hi(4.0 * kReluAdaptX0))) {
            horner_q<R, kReluAdaptDeg0>(p, u, tab.a0);
        } else if (__all(hm < vote_hi(4.0 * kReluAdaptX1))) {
            horner_q<R, kReluAdaptDeg1>(p, u, tab.a1);
        } else if (__all(hm < vote_hi(4.0 * kReluAdaptX2))) {
#else
        double um = u[0];
#pragma unroll
        for (int r = 1; r < R; ++r) um = __builtin_fmax(um, u[r]);
        if (__all(um <= 4.0 * kReluAdaptX0)) {
            horner_q<R, kReluAdaptDeg0>(p, u, tab.a0);
        } else if (__all(um <= 4.0 * kReluAdaptX1)) {
            horner_q<R, kReluAdaptDeg1>(p, u, tab.a1);
        } else if (__all(um <= 4.0 * kReluAdaptX2)) {
#endif
            horner_q<R, kReluAdaptDeg2>(p, u, tab.a2);
        } else {
            horner_q<R, kReluPolyDegD>(p, u, tab.dq);
        }
    } else {
        horner_q<R, kReluPolyDegD>(p, u, tab.dq);
    }
#pragma unroll
    for (int r = 0; r < R; ++r) c[r] = __builtin_fma(sx[r], p[r], c[r] + __builtin_fabs(c[r]));
}
// fp32: pixels in pairs on the packed-fp32 VALU (v_pk_fma_f32 / v_pk_mul_f32 /
// v_pk_add_f32 do two fp32 lanes per instruction at the rate of one).  Each element sees
// exactly relu_fast's IEEE operations in the same order, so the packed form is
// bit-identical to the scalar one; only min/max/abs and the rsq estimates stay scalar (no
// packed form).  An odd R leaves one pixel on the scalar path.
typedef float cgp_f2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ cgp_f2 relu_fast2(cgp_f2 c, cgp_f2 v1, cgp_f2 v2) {
    const cgp_f2 t = __builtin_elementwise_fma(v1, v2, cgp_f2(K<float>::tiny));
    const cgp_f2 y = {__builtin_amdgcn_rsqf(t.x), __builtin_amdgcn_rsqf(t.y)};
    const cgp_f2 st = t * y;                                   // sqrt(t)
    const cgp_f2 cy = c * y;
    const cgp_f2 a = {__builtin_fminf(__builtin_fabsf(cy.x), 1.0f),
                      __builtin_fminf(__builtin_fabsf(cy.y), 1.0f)};   // |rho| clamped
    const cgp_f2 x = __builtin_elementwise_fma(cgp_f2(-0.5f), a, cgp_f2(0.5f));
    const cgp_f2 xm = {__builtin_fmaxf(x.x, K<float>::xfloor), __builtin_fmaxf(x.y, K<float>::xfloor)};
    const cgp_f2 h = {__builtin_amdgcn_rsqf(xm.x), __builtin_amdgcn_rsqf(xm.y)};
    const cgp_f2 sx = xm * h;                                  // sqrt(x)
    cgp_f2 p = cgp_f2(kReluPolyF[kReluPolyDegF]);
#pragma unroll
    for (int k = kReluPolyDegF - 1; k >= 0; --k)
        p = __builtin_elementwise_fma(p, x, cgp_f2(kReluPolyF[k]));
    const cgp_f2 ac = {__builtin_fabsf(c.x), __builtin_fabsf(c.y)};
    const cgp_f2 hpos = (c + ac) * cgp_f2(0.25f);              // max(c, 0) / 2
    return __builtin_elementwise_fma((st * x) * sx, p, hpos);
}
// relu_fast's steps before / after the polynomial, packed (two pixels) and scalar: x, the
// factor m = (sqrt(t)·x)·sqrt(x) and max(c, 0)/2, then out = m·P(x) + max(c, 0)/2 — the
// same IEEE operations in the same order as relu_fast2 / relu_fast
__device__ __forceinline__ void relu_prep2(cgp_f2 c, cgp_f2 v1, cgp_f2 v2, cgp_f2& x, cgp_f2& m,
                                           cgp_f2& hpos) {
    const cgp_f2 t = __builtin_elementwise_fma(v1, v2, cgp_f2(K<float>::tiny));
    const cgp_f2 y = {__builtin_amdgcn_rsqf(t.x), __builtin_amdgcn_rsqf(t.y)};
    const cgp_f2 st = t * y;
    const cgp_f2 cy = c * y;
    const cgp_f2 a = {__builtin_fminf(__builtin_fabsf(cy.x), 1.0f),
                      __builtin_fminf(__builtin_fabsf(cy.y), 1.0f)};
    x = __builtin_elementwise_fma(cgp_f2(-0.5f), a, cgp_f2(0.5f));
    const cgp_f2 xm = {__builtin_fmaxf(x.x, K<float>::xfloor), __builtin_fmaxf(x.y, K<float>::xfloor)};
    const cgp_f2 h = {__builtin_amdgcn_rsqf(xm.x), __builtin_amdgcn_rsqf(xm.y)};
    m = (st * x) * (xm * h);
    const cgp_f2 ac = {__builtin_fabsf(c.x), __builtin_fabsf(c.y)};
    hpos = (c + ac) * cgp_f2(0.25f);
}
__device__ __forceinline__ void relu_prep1(float c, float v1, float v2, float& x, float& m,
                                           float& hpos) {
    const float t = __builtin_fmaf(v1, v2, K<float>::tiny);
    const float y = __builtin_amdgcn_rsqf(t);
    const float st = t * y;
    const float a = __builtin_fminf(__builtin_fabsf(c * y), 1.0f);
    x = __builtin_fmaf(-0.5f, a, 0.5f);
    const float xm = __builtin_fmaxf(x, K<float>::xfloor);
    m = (st * x) * (xm * __builtin_amdgcn_rsqf(xm));
    hpos = (c + __builtin_fabsf(c)) * 0.25f;
}
// R pixels (packed pairs + an odd scalar one) through the degree-D Horner of P
template <int R, int D>
__device__ __forceinline__ void relu_poly_f(const float (&P)[D + 1], float (&c)[R],
                                            const cgp_f2 (&x2)[R / 2 + 1],
                                            const cgp_f2 (&m2)[R / 2 + 1],
                                            const cgp_f2 (&h2)[R / 2 + 1], float xs, float ms,
                                            float hs) {
#pragma unroll
    for (int q = 0; q < R / 2; ++q) {
        cgp_f2 p = cgp_f2(P[D]);
#pragma unroll
        for (int k = D - 1; k >= 0; --k) p = __builtin_elementwise_fma(p, x2[q], cgp_f2(P[k]));
        const cgp_f2 o = __builtin_elementwise_fma(m2[q], p, h2[q]);
        c[2 * q] = o.x;
        c[2 * q + 1] = o.y;
    }
    if constexpr (R % 2) {
        float p = P[D];
#pragma unroll
        for (int k = D - 1; k >= 0; --k) p = __builtin_fmaf(p, xs, P[k]);
        c[R - 1] = __builtin_fmaf(ms, p, hs);
    }
}
// R fp32 ReLUs: packed pairs + an odd scalar pixel through the degree-6 polynomial (its
// range-adaptive form measured neutral: the fp32 kernel is latency bound)
template <int R>
__device__ __forceinline__ void relu_fast_n(float (&c)[R], const float (&v1)[R],
                                            const float (&v2)[R], const PolyTab&) {
    cgp_f2 x2[R / 2 + 1], m2[R / 2 + 1], h2[R / 2 + 1];
    float xs = 0.0f, ms = 0.0f, hs = 0.0f;
#pragma unroll
    for (int q = 0; q < R / 2; ++q)
        relu_prep2(cgp_f2{c[2 * q], c[2 * q + 1]}, cgp_f2{v1[2 * q], v1[2 * q + 1]},
                   cgp_f2{v2[2 * q], v2[2 * q + 1]}, x2[q], m2[q], h2[q]);
    if constexpr (R % 2) relu_prep1(c[R - 1], v1[R - 1], v2[R - 1], xs, ms, hs);
    relu_poly_f<R, kReluPolyDegF>(kReluPolyF, c, x2, m2, h2, xs, ms, hs);
}

template <typename T>
__device__ __forceinline__ T relu_fast(T c, T v1, T v2) {
    const T t = v1 * v2 + K<T>::tiny;
    const T y = rsqrt_fast(t);
    const T st = t * y;                                     // sqrt(t)
    const T a = fmin_t(fabs_t(c * y), T(1));                // |rho| clamped
    const T x = fma_t(T(-0.5), a, T(0.5));                  // (1 - a)/2
    const T sx = sqrt_fast(fmax_t(x, K<T>::xfloor));        // sqrt(x)
    const T p = relu_poly(x);
    const T pos = fmax_t(c, T(0));
    // (c - c): 0 for finite c, NaN for NaN c — keeps the reference's NaN propagation
    return fma_t((st * x) * sx, p, T(0.5) * pos) + (c - c);
}

// ReLU of pair map m at pixel px with the same/diag overrides of kernels.py:155-162.
template <typename T>
__device__ __forceinline__ T relu_pair(T c, const T* __restrict__ xx, const T* __restrict__ yy,
                                       unsigned i, unsigned j, int hw, int px, int same,
                                       int diag, int exact) {
    const T v1 = xx[(size_t)i * hw + px];
    if (same && (diag || i == j)) return v1 / T(2);          // xy' = xx' = xx/2
    const T v2 = yy[(size_t)j * hw + px];
    return exact ? relu_exact(c, v1, v2) : relu_fast(c, v1, v2);
}

// pair index -> (i, j)
__device__ __forceinline__ void pair_of(unsigned m, const FastDiv& n2, int diag, unsigned& i,
                                        unsigned& j) {
    if (diag) {
        i = j = m;
    } else {
        i = fdiv(m, n2);
        j = m - i * n2.d;
    }
}

// LDS-only barrier: waits for this wave's LDS traffic, not for its global loads, so the
// next chunk's prefetch stays in flight across it (cdna_hip_programming.md §5).
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

}  // namespace cgp
