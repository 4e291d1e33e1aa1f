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
#include <algorithm>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "cnngp.h"
#include "cgp_common.h"

namespace cgp {


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


// compute units of the current device (cached; launch geometry of persistent kernels)
int device_cus() {
    static std::mutex mu;
    static std::map<int, int> cache;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 256;
    std::lock_guard<std::mutex> lk(mu);
    auto it = cache.find(dev);
    if (it != cache.end()) return it->second;
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        n <= 0)
        n = 256;
    cache[dev] = n;
    return n;
}

}  // namespace cgp

using namespace cgp;

namespace {

constexpr int kBlock = 256;          // 4 waves of 64
constexpr int kChunkElems = 2048;    // map elements one workgroup stages per chunk
constexpr int kEMax = kChunkElems / kBlock;   // prefetch registers per thread (8)
constexpr int kMaxLds = 64 * 1024;   // bytes of LDS one conv workgroup may take


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
    long long nchunks;
    FastDiv n2;       // pair index -> (i, j)
    FastDiv dw;       // in-map element -> row
    FastDiv dhw;      // chunk element -> map
    FastDiv dwo;      // output row
    FastDiv dhowo;    // output map
    int h, w, ho, wo;
    int hp, wp;       // padded LDS plane (zero halo)
    int plo_r, plo_c; // halo before row/col 0
    int c0, r0;       // first tap column / row in the padded plane for output 0
    int taps, stride, dil;
    int channels;
    int pre, post, add, same, diag, exact;
    int mpb;          // maps per chunk
    int hs_offset;    // element offset of the row-sum plane in LDS
    T weight, bias;
};

// ----------------------------------------------------------------------------------
// Conv2d covariance stencil, fused (kernels.py:92-98 [+ :134-165 before/after] [+ Sum]).
//
// Persistent workgroups walk chunks of `mpb` whole maps.  Per chunk:
//   load     HBM -> registers (issued one chunk ahead, in flight during the compute)
//   stage 1  registers -> LDS, into zero-haloed padded planes (x the PRE op)
//   stage 2  LDS -> LDS   row sums over the taps, no bounds checks   hs[m][r][ow]
//   stage 3  LDS -> HBM   column sums, ·w + b, POST ReLU, + addend
// The constant conv weight makes the k×k stencil separable (2k LDS reads per output
// instead of k²); TAPS > 0 unrolls the tap loops.  Every HBM byte is read or written
// once, with whole-chunk contiguous (coalesced) ranges.
// ----------------------------------------------------------------------------------
template <typename T, int TAPS>
__global__ __launch_bounds__(kBlock, 4) void conv_cov_kernel(const ConvP<T> p) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    T* tin = reinterpret_cast<T*>(smem);
    T* ths = tin + p.hs_offset;
    const int tid = threadIdx.x;
    const int hw = p.h * p.w;
    const int howo = p.ho * p.wo;
    const int plane = p.hp * p.wp;
    const int taps = TAPS > 0 ? TAPS : p.taps;

    // zero the padded planes once: the halo is never written afterwards
    for (int e = tid; e < p.mpb * plane; e += kBlock) tin[e] = T(0);

    T v[kEMax];
    // plain map loads go through the prefetch registers; the input moments (first layer
    // only, small cached image reads) are computed in stage 1 instead
    const bool prefetch = p.pre != CGP_PRE_MOMENTS;
    auto load_chunk = [&](long long chunk) {
        const long long m0 = chunk * p.mpb;
        const long long rem = p.nmaps - m0;
        const int nin = (rem < p.mpb ? (int)rem : p.mpb) * hw;
        const T* src = p.in + m0 * hw;
#pragma unroll
        for (int k = 0; k < kEMax; ++k) {
            const int e = tid + k * kBlock;
            v[k] = e < nin ? src[e] : T(0);
        }
    };

    long long chunk = blockIdx.x;
    if (prefetch && chunk < p.nchunks) load_chunk(chunk);
    __syncthreads();   // halo zeroing complete
    for (; chunk < p.nchunks; chunk += gridDim.x) {
        const long long m0 = chunk * p.mpb;
        const long long rem = p.nmaps - m0;
        const int mb = rem < p.mpb ? (int)rem : p.mpb;
        const int nin = mb * hw;

        // ---- stage 1: registers -> padded LDS planes ----
#pragma unroll
        for (int k = 0; k < kEMax; ++k) {
            const int e = tid + k * kBlock;
            if (prefetch && e < nin) {
                const unsigned ml = fdiv((unsigned)e, p.dhw);
                const int px = e - (int)ml * hw;
                const unsigned r = fdiv((unsigned)px, p.dw);
                const int c = px - (int)r * p.w;
                tin[(int)ml * plane + ((int)r + p.plo_r) * p.wp + c + p.plo_c] = v[k];
            }
        }
        // moments, and chunks larger than the prefetch window: direct path
        for (int e = tid + (prefetch ? kEMax * kBlock : 0); e < nin; e += kBlock) {
            const unsigned ml = fdiv((unsigned)e, p.dhw);
            const int px = e - (int)ml * hw;
            const unsigned r = fdiv((unsigned)px, p.dw);
            const int c = px - (int)r * p.w;
            T x;
            if (p.pre == CGP_PRE_MOMENTS) {
                unsigned i, j;
                pair_of((unsigned)(m0 + ml), p.n2, p.diag, i, j);
                const T* xi = p.in + (size_t)i * p.channels * hw + px;
                const T* yj = p.in_y + (size_t)j * p.channels * hw + px;
                x = xi[0] * yj[0];
                for (int cc = 1; cc < p.channels; ++cc)
                    x += xi[(size_t)cc * hw] * yj[(size_t)cc * hw];
                x = x / T(p.channels);
            } else {
                x = p.in[m0 * hw + e];
            }
            tin[(int)ml * plane + ((int)r + p.plo_r) * p.wp + c + p.plo_c] = x;
        }
        // PRE ReLU in place on the staged interior (each thread revisits its own writes,
        // so no barrier is needed before it)
        if (p.pre == CGP_PRE_RELU) {
            for (int e = tid; e < nin; e += kBlock) {
                const unsigned ml = fdiv((unsigned)e, p.dhw);
                const int px = e - (int)ml * hw;
                const unsigned r = fdiv((unsigned)px, p.dw);
                const int c = px - (int)r * p.w;
                unsigned i, j;
                pair_of((unsigned)(m0 + ml), p.n2, p.diag, i, j);
                T* slot = tin + (int)ml * plane + ((int)r + p.plo_r) * p.wp + c + p.plo_c;
                *slot = relu_pair(*slot, p.pre_xx, p.pre_yy, i, j, hw, px, p.same, p.diag,
                                  p.exact);
            }
        }
        lds_barrier();

        // the next chunk's HBM reads fly while this one is computed
        if (prefetch && chunk + gridDim.x < p.nchunks) load_chunk(chunk + gridDim.x);

        // ---- stage 2: row sums over the horizontal taps (every padded row) ----
        const int nhs = mb * p.hp * p.wo;
        for (int e = tid; e < nhs; e += kBlock) {
            const unsigned rowi = fdiv((unsigned)e, p.dwo);        // ml * hp + rp
            const int ow = e - (int)rowi * p.wo;
            const T* src = tin + (int)rowi * p.wp + ow * p.stride + p.c0;
            T acc = src[0];
#pragma unroll
            for (int t = 1; t < (TAPS > 0 ? TAPS : 1); ++t) acc += src[t * p.dil];
            if (TAPS == 0)
                for (int t = 1; t < taps; ++t) acc += src[t * p.dil];
            ths[e] = acc;
        }
        lds_barrier();

        // ---- stage 3: column sums, affine, fused epilogue, store ----
        const int nout = mb * howo;
        T* dst = p.out + m0 * howo;
        const T* add = p.add ? p.addend + m0 * howo : nullptr;
        for (int e = tid; e < nout; e += kBlock) {
            const unsigned ml = fdiv((unsigned)e, p.dhowo);
            const int q = e - (int)ml * howo;
            const unsigned oh = fdiv((unsigned)q, p.dwo);
            const int ow = q - (int)oh * p.wo;
            const T* col = ths + ((int)ml * p.hp + (int)oh * p.stride + p.r0) * p.wo + ow;
            const int cs = p.dil * p.wo;
            T acc = col[0];
#pragma unroll
            for (int t = 1; t < (TAPS > 0 ? TAPS : 1); ++t) acc += col[t * cs];
            if (TAPS == 0)
                for (int t = 1; t < taps; ++t) acc += col[t * cs];
            T val = p.weight * acc + p.bias;
            if (p.post == CGP_POST_RELU) {
                unsigned i, j;
                pair_of((unsigned)(m0 + ml), p.n2, p.diag, i, j);
                val = relu_pair(val, p.post_xx, p.post_yy, i, j, howo, q, p.same, p.diag,
                                p.exact);
            }
            if (p.add) val = val + add[e];
            dst[e] = val;
        }
    }
}

// ----------------------------------------------------------------------------------
// Conv2d covariance stencil for the geometries the configs use (compile-time shapes).
//
// Same chunked algorithm as conv_cov_kernel, with every map dimension a compile-time
// constant, so index math folds to shifts/multiply-highs, the tap loops unroll into
// ds_read_b64 with immediate offsets, and the parameter block stays small (no SGPR
// spills).  Memory pipeline per chunk (one chunk = MB whole maps):
//   top      wait for this chunk's input DMA; issue its variance/addend loads (registers)
//   stage 1  input staging -> zero-haloed padded planes (+ PRE ReLU / input moments)
//   DMA      next chunk's input maps HBM -> LDS staging (global_load_lds, fixed count
//            per wave, branch-free), in flight during stages 2-3
//   stage 2  row sums, one output per item
//   stage 3  column sums, R3 output rows per item; ·w + b, POST ReLU, + addend, store
// ----------------------------------------------------------------------------------
template <int H_, int W_, int HO_, int WO_, int TAPS_, int S_, int OFF_>
struct Geo {
    static constexpr int H = H_, W = W_, HO = HO_, WO = WO_, TAPS = TAPS_, S = S_, OFF = OFF_;
    static constexpr int HW = H * W, HOWO = HO * WO;
    static constexpr int PLO = OFF < 0 ? -OFF : 0;
    static constexpr int R3 = HO >= 8 ? 4 : (HO >= 2 ? 2 : 1);   // rows per stage-3 item
    static constexpr int R2 = WO % 4 == 0 ? 4 : (WO % 2 == 0 ? 2 : 1);   // cols per stage-2 item
    static constexpr int HOS = (HO + R3 - 1) / R3 * R3;
    static constexpr int LASTC = (WO - 1) * S + OFF + TAPS - 1;
    static constexpr int LASTR = (HOS - 1) * S + OFF + TAPS - 1;
    static constexpr int WP = W + PLO + (LASTC > W - 1 ? LASTC - (W - 1) : 0);
    static constexpr int HP = H + PLO + (LASTR > H - 1 ? LASTR - (H - 1) : 0);
    static constexpr int C0 = OFF + PLO, R0 = OFF + PLO;
    static constexpr int PL = HP * WP;
    static constexpr int WIN = (R3 - 1) * S + TAPS;               // stage-3 register window
    static constexpr int WIN2 = (R2 - 1) * S + TAPS;              // stage-2 register window
};

// out[o] = sum_{t<TAPS} w[o*S + t] for o < R, sharing partial sums between the R
// overlapping windows (stride 1): the core w[R-1 .. TAPS-1] is common to every output,
// so R outputs cost (TAPS - R) + R(R - 1) adds instead of R(TAPS - 1).
template <typename T, int TAPS, int S, int R>
__device__ __forceinline__ void window_sums(const T (&w)[(R - 1) * S + TAPS], T (&out)[R]) {
    if constexpr (S == 1 && TAPS > R && R > 1) {
        T core = w[R - 1];
#pragma unroll
        for (int t = R; t < TAPS; ++t) core += w[t];
#pragma unroll
        for (int o = 0; o < R; ++o) {
            T acc;
            if (o < R - 1) {
                acc = w[o];
#pragma unroll
                for (int t = o + 1; t < R - 1; ++t) acc += w[t];
                acc += core;
            } else {
                acc = core;
            }
#pragma unroll
            for (int t = TAPS; t < TAPS + o; ++t) acc += w[t];
            out[o] = acc;
        }
    } else {
#pragma unroll
        for (int o = 0; o < R; ++o) {
            T acc = w[o * S];
#pragma unroll
            for (int t = 1; t < TAPS; ++t) acc += w[o * S + t];
            out[o] = acc;
        }
    }
}

constexpr int cround(int n, int a) { return (n + a - 1) / a * a; }

template <typename T, class G>
struct GeoLayout {
    static constexpr int al = 16 / (int)sizeof(T);
    static constexpr int PAD = 1024 / (int)sizeof(T);   // DMA tail slack after a staging buffer
    static constexpr int lds_elems(int mb) {
        return 2 * (cround(mb * G::HW, al) + PAD) + cround(mb * G::PL, al) +
               cround(mb * G::HP * G::WO, al);
    }
    static constexpr int pick_mb() {
        int mb = kChunkElems / G::HW;
        if (mb < 1) mb = 1;
        if (mb > 16) mb = 16;
        while (mb > 1 && lds_elems(mb) * (int)sizeof(T) > 32 * 1024) --mb;
        return mb;
    }
    static constexpr int MB = pick_mb();
    static constexpr int IN_STRIDE = cround(MB * G::HW, al) + PAD;   // two input buffers
    static constexpr int L_PLANE = 2 * IN_STRIDE;
    static constexpr int L_HS = L_PLANE + cround(MB * G::PL, al);
    static constexpr int ELEMS = L_HS + cround(MB * G::HP * G::WO, al);
    static constexpr int IN_BYTES = MB * G::HW * (int)sizeof(T);
    static constexpr int DMA16 = (IN_BYTES % 16) == 0 && (G::HW * (int)sizeof(T)) % 16 == 0;
    static constexpr int PIECE = DMA16 ? 1024 : 256;
    static constexpr int PIECES = (IN_BYTES + PIECE - 1) / PIECE;
    static constexpr int PW = (PIECES + kBlock / 64 - 1) / (kBlock / 64);   // per wave
    static constexpr int N3 = MB * (G::HOS / G::R3) * G::WO;
    static constexpr int I3 = (N3 + kBlock - 1) / kBlock;
};

template <typename T>
struct GeoP {
    const T* in;
    const T* in_y;
    T* out;
    const T* addend;
    const T* pre_xx;
    const T* pre_yy;
    const T* post_xx;
    const T* post_yy;
    long long nmaps, nchunks;
    FastDiv n2;
    int channels, pre, post, add, same, diag;
    T weight, bias;
};

typedef __attribute__((address_space(1))) void* gptr_t;
typedef __attribute__((address_space(3))) void* lptr_t;

// The chunk's input maps -> LDS staging by LDS-DMA: exactly PW instructions per wave with
// all 64 lanes active (sources clamped into the chunk, tails land in the pad), so the
// compiler's vmcnt bookkeeping for loads issued before it stays exact.
template <typename T, class G>
__device__ __forceinline__ void geo_dma_input(const GeoP<T>& p, long long chunk,
                                              unsigned char* smem, int wave, int lane) {
    // smem: this buffer's base
    using L = GeoLayout<T, G>;
    const long long m0 = chunk * L::MB;
    const long long rem = p.nmaps - m0;
    const int nbytes = (rem < L::MB ? (int)rem : L::MB) * G::HW * (int)sizeof(T);
    const char* src = reinterpret_cast<const char*>(p.in + m0 * G::HW);
#pragma unroll
    for (int k = 0; k < L::PW; ++k) {
        int pc = wave * L::PW + k;
        if (pc >= L::PIECES) pc = L::PIECES - 1;                   // duplicate, harmless
        int o = pc * L::PIECE + lane * (L::PIECE / 64);
        if (o > nbytes - L::PIECE / 64) o = nbytes - L::PIECE / 64;   // clamp the tail
        unsigned char* dst = smem + (size_t)pc * L::PIECE;
        if constexpr (L::DMA16)
            __builtin_amdgcn_global_load_lds((gptr_t)(src + o), (lptr_t)dst, 16, 0, 0);
        else
            __builtin_amdgcn_global_load_lds((gptr_t)(src + o), (lptr_t)dst, 4, 0, 0);
    }
}

template <typename T, class G, int PRE, bool POST, bool ADD>
__global__ __launch_bounds__(kBlock) void conv_geo_kernel(const GeoP<T> p) {
    using L = GeoLayout<T, G>;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    T* lds = reinterpret_cast<T*>(smem);
    T* plane = lds + L::L_PLANE;
    T* hs = lds + L::L_HS;
    const int tid = threadIdx.x;
    const int wave = tid >> 6, lane = tid & 63;
    constexpr bool moments = PRE == CGP_PRE_MOMENTS;
    auto inbuf = [&](int b) { return smem + (size_t)b * L::IN_STRIDE * sizeof(T); };

    for (int e = tid; e < L::MB * G::PL; e += kBlock) plane[e] = T(0);   // halo: zero forever
    // input DMA runs two chunks ahead: chunk k's maps land in buffer k & 1
    long long chunk = blockIdx.x;
    if constexpr (!moments) {
        if (chunk < p.nchunks) {
            const long long c1 = chunk + gridDim.x;
            geo_dma_input<T, G>(p, chunk, inbuf(0), wave, lane);
            geo_dma_input<T, G>(p, c1 < p.nchunks ? c1 : chunk, inbuf(1), wave, lane);
        }
    }

    for (int buf = 0; chunk < p.nchunks; chunk += gridDim.x, buf ^= 1) {
        const long long m0 = chunk * L::MB;
        const long long rem = p.nmaps - m0;
        const int mb = rem < L::MB ? (int)rem : L::MB;
        const T* sin = reinterpret_cast<const T*>(inbuf(buf));
        // this chunk's DMA is older than the last PW VM ops (the next chunk's DMA)
        if constexpr (moments)
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        else
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(L::PW) : "memory");
        lds_barrier();

        const T* addend_c = ADD ? p.addend + m0 * G::HOWO : nullptr;
        // variance / addend values this thread's stage-3 outputs need (loaded now, used
        // after stage 2)
        T vx[L::I3][G::R3], vy[L::I3][G::R3], ad[L::I3][G::R3];
        unsigned pi[L::I3], pj[L::I3];
#pragma unroll
        for (int k = 0; k < L::I3; ++k) {
            int e = tid + k * kBlock;
            if (e >= mb * (G::HOS / G::R3) * G::WO) e = 0;             // clamp: valid address
            const int ow = e % G::WO;
            const int rr = e / G::WO;
            const int ml = rr / (G::HOS / G::R3);
            const int oh0 = (rr - ml * (G::HOS / G::R3)) * G::R3;
            unsigned i = 0, j = 0;
            pair_of((unsigned)(m0 + ml), p.n2, p.diag, i, j);
            pi[k] = i;
            pj[k] = j;
            // 32-bit element offsets from scalar bases (saddr + voffset addressing)
            const unsigned xo = i * (unsigned)G::HOWO, yo = j * (unsigned)G::HOWO;
            const unsigned ao = (unsigned)(ml * G::HOWO);
#pragma unroll
            for (int o = 0; o < G::R3; ++o) {
                const int oh = oh0 + o < G::HO ? oh0 + o : G::HO - 1;
                const unsigned q = (unsigned)(oh * G::WO + ow);
                if constexpr (POST) {
                    vx[k][o] = p.post_xx[xo + q];
                    vy[k][o] = p.post_yy[yo + q];
                }
                if constexpr (ADD) ad[k][o] = addend_c[ao + q];
            }
        }

        // ---- stage 1: staging -> padded planes (+ PRE ReLU, or the input moments) ----
        for (int e = tid; e < mb * G::HW; e += kBlock) {
            const int ml = e / G::HW;
            const int px = e - ml * G::HW;
            const int r = px / G::W;
            const int c = px - r * G::W;
            T x;
            if constexpr (moments) {
                unsigned i, j;
                pair_of((unsigned)(m0 + ml), p.n2, p.diag, i, j);
                const T* xi = p.in + (size_t)i * p.channels * G::HW + px;
                const T* yj = p.in_y + (size_t)j * p.channels * G::HW + px;
                x = xi[0] * yj[0];
                for (int cc = 1; cc < p.channels; ++cc)
                    x += xi[(size_t)cc * G::HW] * yj[(size_t)cc * G::HW];
                x = x / T(p.channels);
            } else {
                x = sin[e];
                if constexpr (PRE == CGP_PRE_RELU) {
                    unsigned i, j;
                    pair_of((unsigned)(m0 + ml), p.n2, p.diag, i, j);
                    x = relu_pair(x, p.pre_xx, p.pre_yy, i, j, G::HW, px, p.same, p.diag, 0);
                }
            }
            plane[ml * G::PL + (r + G::PLO) * G::WP + c + G::PLO] = x;
        }
        lds_barrier();

        // ---- stage 2: row sums (every padded row), R2 outputs per item ----
        constexpr int NSEG2 = G::WO / G::R2;
        for (int e = tid; e < mb * G::HP * NSEG2; e += kBlock) {
            const int rowi = e / NSEG2;                           // ml * HP + rp
            const int seg = e - rowi * NSEG2;
            const T* src = plane + rowi * G::WP + seg * (G::R2 * G::S) + G::C0;
            T win[G::WIN2];
#pragma unroll
            for (int t = 0; t < G::WIN2; ++t) win[t] = src[t];
            T res[G::R2];
            window_sums<T, G::TAPS, G::S, G::R2>(win, res);
#pragma unroll
            for (int o = 0; o < G::R2; ++o) hs[rowi * G::WO + seg * G::R2 + o] = res[o];
        }
        lds_barrier();

        // ---- stage 3: column sums over R3 rows per item, epilogue, store ----
        T* out = p.out + m0 * G::HOWO;
#pragma unroll
        for (int k = 0; k < L::I3; ++k) {
            const int e = tid + k * kBlock;
            if (e < mb * (G::HOS / G::R3) * G::WO) {
                const int ow = e % G::WO;
                const int rr = e / G::WO;
                const int ml = rr / (G::HOS / G::R3);
                const int oh0 = (rr - ml * (G::HOS / G::R3)) * G::R3;
                const T* src = hs + (ml * G::HP + oh0 * G::S + G::R0) * G::WO + ow;
                T win[G::WIN];
#pragma unroll
                for (int t = 0; t < G::WIN; ++t) win[t] = src[t * G::WO];
                T res[G::R3];
                window_sums<T, G::TAPS, G::S, G::R3>(win, res);
#pragma unroll
                for (int o = 0; o < G::R3; ++o) res[o] = p.weight * res[o] + p.bias;
                if constexpr (POST) {
                    const bool ovr = p.same && (p.diag || pi[k] == pj[k]);
#pragma unroll
                    for (int o = 0; o < G::R3; ++o) {
                        const T r = relu_fast(res[o], vx[k][o], vy[k][o]);
                        res[o] = ovr ? vx[k][o] / T(2) : r;
                    }
                }
                // materialise every result before the first (predicated) store: otherwise
                // hipcc sinks each output's math into its store block and re-waits vmcnt(0)
                // per block, serialising on the stores just issued
#pragma unroll
                for (int o = 0; o < G::R3; ++o) {
                    if constexpr (ADD) res[o] = res[o] + ad[k][o];
                    asm volatile("" ::"v"(res[o]));
                }
#pragma unroll
                for (int o = 0; o < G::R3; ++o) {
                    // (non-temporal stores measured -5%: profiles/r4/ab_r4f_stencil_nt_store.log)
                    if (oh0 + o < G::HO)
                        out[(unsigned)(ml * G::HOWO + (oh0 + o) * G::WO + ow)] = res[o];
                }
            }
        }
        // buffer `buf` was consumed in stage 1: fetch chunk k+2 into it (unconditional —
        // past the end it re-fetches this chunk — so every path issues exactly PW ops)
        if constexpr (!moments) {
            const long long nxt = chunk + 2 * (long long)gridDim.x;
            geo_dma_input<T, G>(p, nxt < p.nchunks ? nxt : chunk, inbuf(buf), wave, lane);
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// the geometries of configs/*.py (taps, stride, offset as Conv2d lowers them)
#define CGP_GEOMETRIES(X)            \
    X(28, 28, 28, 28, 7, 1, -3)      \
    X(28, 28, 28, 28, 1, 1, 0)       \
    X(32, 32, 32, 32, 1, 1, 0)       \
    X(28, 28, 28, 28, 4, 1, -1)      \
    X(28, 28, 28, 28, 3, 1, -1)      \
    X(28, 28, 14, 14, 3, 2, -1)      \
    X(28, 28, 14, 14, 1, 2, 0)       \
    X(14, 14, 14, 14, 3, 1, -1)      \
    X(14, 14, 7, 7, 3, 2, -1)        \
    X(14, 14, 7, 7, 1, 2, 0)         \
    X(7, 7, 7, 7, 3, 1, -1)          \
    X(32, 32, 32, 32, 3, 1, -1)      \
    X(32, 32, 16, 16, 3, 2, -1)      \
    X(32, 32, 16, 16, 1, 2, 0)       \
    X(16, 16, 16, 16, 3, 1, -1)      \
    X(16, 16, 8, 8, 3, 2, -1)        \
    X(16, 16, 8, 8, 1, 2, 0)         \
    X(8, 8, 8, 8, 3, 1, -1)

// ----------------------------------------------------------------------------------
// standalone ReLU on pair maps (+ optional addend), one chunk of maps per workgroup
// ----------------------------------------------------------------------------------
template <typename T>
struct ReluP {
    const T* xy;
    T* out;
    const T* addend;
    const T* xx;
    const T* yy;
    long long nmaps;
    FastDiv n2, dhw;
    int hw, same, diag, exact, mpb;
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
    T v[kEMax];
#pragma unroll
    for (int k = 0; k < kEMax; ++k) {
        const int e = threadIdx.x + k * kBlock;
        v[k] = e < n ? src[e] : T(0);
    }
#pragma unroll
    for (int k = 0; k < kEMax; ++k) {
        const int e = threadIdx.x + k * kBlock;
        if (e < n) {
            const unsigned ml = fdiv((unsigned)e, p.dhw);
            const int px = e - (int)ml * p.hw;
            unsigned i, j;
            pair_of((unsigned)(m0 + ml), p.n2, p.diag, i, j);
            T r = relu_pair(v[k], p.xx, p.yy, i, j, p.hw, px, p.same, p.diag, p.exact);
            if constexpr (ADD) r = r + add[e];
            dst[e] = r;
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
                                                            long long nmaps, FastDiv n2,
                                                            FastDiv dhw, int c, int hw,
                                                            int diag, int mpb,
                                                            T* __restrict__ xy) {
    const long long m0 = (long long)blockIdx.x * mpb;
    long long rem = nmaps - m0;
    const int mb = rem < mpb ? (int)rem : mpb;
    const int n = mb * hw;
    T* dst = xy + m0 * hw;
    for (int e = threadIdx.x; e < n; e += kBlock) {
        const unsigned ml = fdiv((unsigned)e, dhw);
        const int px = e - (int)ml * hw;
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

// dst_k = alpha·src_k for up to kScaleBatch buffers in one launch (blockIdx.y = buffer):
// the fp64 whole-network kernel's quartered x-side variance maps, one launch per tile
// instead of one per map
constexpr int kScaleBatch = 32;
struct ScaleBatch {
    const double* src[kScaleBatch];
    double* dst[kScaleBatch];
    long long n[kScaleBatch];
};
__global__ __launch_bounds__(kBlock) void scale_batch_kernel(ScaleBatch b, double alpha) {
    const int k = blockIdx.y;
    const double* __restrict__ src = b.src[k];
    double* __restrict__ dst = b.dst[k];
    const long long n = b.n[k];
    const long long stride = (long long)gridDim.x * kBlock;
    for (long long e = (long long)blockIdx.x * kBlock + threadIdx.x; e < n; e += stride)
        dst[e] = alpha * src[e];
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

// var[r] = d[r] − Σ_c v[r][c]² — one workgroup per row (grid-stride over rows), each
// thread a strided partial sum, then a fixed-order LDS tree: deterministic, coalesced.
__global__ __launch_bounds__(kBlock) void row_sumsq_sub_kernel(const double* __restrict__ v,
                                                               long long rows, long long cols,
                                                               long long ld,
                                                               const double* d, double* out) {
    __shared__ double part[kBlock];
    for (long long r = blockIdx.x; r < rows; r += gridDim.x) {
        const double* row = v + r * ld;
        double acc = 0.0;
        for (long long c = threadIdx.x; c < cols; c += kBlock) acc = __builtin_fma(row[c], row[c], acc);
        part[threadIdx.x] = acc;
        __syncthreads();
        for (int w = kBlock / 2; w > 0; w >>= 1) {
            if ((int)threadIdx.x < w) part[threadIdx.x] += part[threadIdx.x + w];
            __syncthreads();
        }
        if (threadIdx.x == 0) out[r] = d[r] - part[0];
        __syncthreads();
    }
}

// ---- the solution check (cgp_sym_mirror_f64 / cgp_sym_residual_f64) ------------------
// The solve reads only the row-major upper triangle of K and overwrites it with the
// factor; the strictly-lower triangle is free (NaN tiles in the reference's files).  The
// mirror copies the system there before the factorisation, so after the solve the whole
// residual Y − K·X can be formed in one pass over the lower triangle: every row of the
// system is checked, not a sample (a wrong factor can be wrong in a few rows only).
constexpr int kSymT = 64;                 // tile edge
constexpr int kSymLd = kSymT + 1;         // LDS pitch (doubles)
constexpr int kSymRhs = 16;               // right-hand sides per residual launch
constexpr int kSymChunk = 8;              // tiles of one row panel per residual workgroup

// workgroup (I, J), J <= I: the upper block (J, I) read row by row into LDS, written
// transposed as the lower block (I, J) row by row (both coalesced); a diagonal tile
// copies its own upper part down and stores the diagonal.  Reads (upper, incl. the
// diagonal) and writes (strictly lower) never meet across workgroups.
__global__ __launch_bounds__(kBlock) void sym_mirror_kernel(double* __restrict__ k, long long n,
                                                           long long ld,
                                                           double* __restrict__ diag) {
    const int I = blockIdx.x, J = blockIdx.y;
    if (J > I) return;
    __shared__ double t[kSymT * kSymLd];
    const long long r0 = (long long)J * kSymT, c0 = (long long)I * kSymT;
    for (int e = threadIdx.x; e < kSymT * kSymT; e += kBlock) {
        const int r = e >> 6, c = e & 63;
        const long long gr = r0 + r, gc = c0 + c;
        t[r * kSymLd + c] = (gr < n && gc < n && gc >= gr) ? k[gr * ld + gc] : 0.0;
    }
    __syncthreads();
    for (int e = threadIdx.x; e < kSymT * kSymT; e += kBlock) {
        const int rr = e >> 6, cc = e & 63;          // destination (c0 + rr, r0 + cc)
        const long long gr = c0 + rr, gc = r0 + cc;
        if (gr < n && gc < n) {
            if (gc < gr)
                k[gr * ld + gc] = t[cc * kSymLd + rr];
            else if (gc == gr)
                diag[gr] = t[cc * kSymLd + rr];
        }
    }
}

// r[q][i] −= Σ_j (L + Lᵀ + diag(d))[i][j]·x[q][j], L = the strictly-lower triangle of K;
// sumsq[0] += Σ L[i][j]² over the tiles read.  Workgroup (I, c): row panel I, tiles
// J in [c·kSymChunk, min((c+1)·kSymChunk, I + 1)).  Per tile (staged in LDS): the rows of
// panel I gain L_IJ·x_J (registers, over the chunk), the columns of J gain L_IJᵀ·x_I (one
// atomic add per column and right-hand side).  Wave g handles right-hand sides g, g+4, …
// (uniform per wave: the x reads are LDS broadcasts).
__global__ __launch_bounds__(kBlock) void sym_residual_kernel(const double* __restrict__ k,
                                                             long long n, long long ld,
                                                             const double* __restrict__ diag,
                                                             const double* __restrict__ x,
                                                             double* r, int nrhs, long long ldx,
                                                             double* sumsq) {
    const int I = blockIdx.x, c = blockIdx.y;
    const int jt0 = c * kSymChunk;
    if (jt0 > I) return;
    const int jt1 = min(jt0 + kSymChunk, I + 1);
    __shared__ double t[kSymT * kSymLd];
    __shared__ double xi[kSymRhs * kSymT], xj[kSymRhs * kSymT];
    __shared__ double red[kBlock / 64];
    const int tid = threadIdx.x, lane = tid & 63, g = tid >> 6;
    const long long i0 = (long long)I * kSymT;
    for (int e = tid; e < nrhs * kSymT; e += kBlock) {
        const int q = e >> 6, l = e & 63;
        xi[e] = (i0 + l < n) ? x[q * ldx + i0 + l] : 0.0;
    }
    double racc[kSymRhs / 4] = {};
    double ss = 0.0;
    for (int J = jt0; J < jt1; ++J) {
        const long long j0 = (long long)J * kSymT;
        __syncthreads();                               // the previous tile's readers
        for (int e = tid; e < kSymT * kSymT; e += kBlock) {
            const int rr = e >> 6, cc = e & 63;
            const long long gr = i0 + rr, gc = j0 + cc;
            const double v = (gr < n && gc < gr) ? k[gr * ld + gc] : 0.0;
            t[rr * kSymLd + cc] = v;
            ss = __builtin_fma(v, v, ss);
        }
        for (int e = tid; e < nrhs * kSymT; e += kBlock) {
            const int q = e >> 6, l = e & 63;
            xj[e] = (j0 + l < n) ? x[q * ldx + j0 + l] : 0.0;
        }
        __syncthreads();
#pragma unroll
        for (int m = 0; m < kSymRhs / 4; ++m) {
            const int q = g + 4 * m;
            if (q < nrhs) {
                double a = 0.0, b = 0.0;
                for (int cc = 0; cc < kSymT; ++cc) {
                    a = __builtin_fma(t[lane * kSymLd + cc], xj[q * kSymT + cc], a);   // rows
                    b = __builtin_fma(t[cc * kSymLd + lane], xi[q * kSymT + cc], b);   // columns
                }
                racc[m] += a;
                if (j0 + lane < n) atomicAdd(&r[q * ldx + j0 + lane], -b);
            }
        }
    }
    if (i0 + lane < n) {
        const bool has_diag = I >= jt0 && I < jt1;
#pragma unroll
        for (int m = 0; m < kSymRhs / 4; ++m) {
            const int q = g + 4 * m;
            if (q < nrhs) {
                double v = racc[m];
                if (has_diag) v = __builtin_fma(diag[i0 + lane], xi[q * kSymT + lane], v);
                atomicAdd(&r[q * ldx + i0 + lane], -v);
            }
        }
    }
    for (int off = 32; off > 0; off >>= 1) ss += __shfl_xor(ss, off, 64);
    if (lane == 0) red[g] = ss;
    __syncthreads();
    if (tid == 0 && sumsq) atomicAdd(sumsq, red[0] + red[1] + red[2] + red[3]);
}

// ---- the variance chain (cgp_var_chain_*): every per-image variance map of a network in
// one launch.  A workgroup walks image g through the op list in LDS (slots from the host);
// the stored maps go to out (layout in cnngp.h).  Same rounding as the layer kernels it
// replaces: moments acc = x0·x0 + x1·x1 + ... then / C; conv w·Σ + b as two roundings;
// Sums as the axpby chain (c0·t0, then o + c_k·t_k).
template <typename T>
struct VarChainP {
    const T* x;
    const T* y;
    T* out;
    const cgp_var_op* ops;
    long long n1, n2, store_total;
    int nops, channels, hw_in, lds_elems, scratch;
};
// Barriers are LDS-only (lds_barrier: wait for this wave's LDS traffic, not its global
// stores): a stored map's LDS reads have returned before its global stores issue, so a
// later op may overwrite the slot while the stores drain.
// op records through the constant address space: every field is uniform, so they load
// with scalar loads into SGPRs (a generic pointer gets per-lane vector loads, and a local
// copy of the record indexed at run time would live in scratch memory)
typedef const __attribute__((address_space(4))) cgp_var_op* VarOpsC;
constexpr int kVarE = 4;   // map pixels per thread (maps up to 4·kBlock = 32x32)

template <typename T>
__global__ __launch_bounds__(kBlock) void var_chain_kernel(const VarChainP<T> p) {
    extern __shared__ __align__(16) unsigned char var_smem[];
    T* lds = reinterpret_cast<T*>(var_smem);
    const VarOpsC ops = (VarOpsC)p.ops;
    const long long n = p.n1 + p.n2;
    const int tid = threadIdx.x;
    for (long long g = blockIdx.x; g < n; g += gridDim.x) {
        const T* img = g < p.n1 ? p.x + g * p.channels * p.hw_in
                                : p.y + (g - p.n1) * p.channels * p.hw_in;
        for (int k = 0; k < p.nops; ++k) {
            const int kind = ops[k].kind;
            const int ho = ops[k].ho, wo = ops[k].wo, howo = ho * wo;
            T* dst = lds + ops[k].dst;
            if (kind == CGP_VAR_MOMENTS) {
                for (int e = tid; e < howo; e += kBlock) {
                    T acc = img[e] * img[e];
                    for (int c = 1; c < p.channels; ++c) {
                        const T v = img[(size_t)c * p.hw_in + e];
                        acc += v * v;
                    }
                    dst[e] = acc / T(p.channels);
                }
            } else if (kind == CGP_VAR_CONV) {
                // separable like the layer kernels: window sums along each input row into
                // the scratch, then along columns (a full-window conv stays parallel)
                const T* src = lds + ops[k].src[0];
                T* hs = lds + p.scratch;
                const int h = ops[k].h, w = ops[k].w, taps = ops[k].taps;
                const int off = ops[k].offset, st = ops[k].stride, dl = ops[k].dilation;
                const T wt = (T)ops[k].weight, b = (T)ops[k].bias;
                const FastDiv fwo = make_fastdiv((unsigned)wo);
                // up to kVarE elements per thread (maps of at most kVarE·kBlock pixels),
                // their window sums interleaved tap by tap (independent LDS chains)
                int rr[kVarE], cc[kVarE];
                bool ok[kVarE];
                T acc[kVarE];
#pragma unroll
                for (int i = 0; i < kVarE; ++i) {
                    const int e = tid + i * kBlock;
                    ok[i] = e < h * wo;
                    rr[i] = (int)fdiv((unsigned)(ok[i] ? e : 0), fwo);
                    cc[i] = (ok[i] ? e : 0) - rr[i] * wo;
                    acc[i] = T(0);
                }
                for (int dx = 0; dx < taps; ++dx) {
#pragma unroll
                    for (int i = 0; i < kVarE; ++i) {
                        const int c = cc[i] * st + off + dx * dl;
                        if (ok[i] && c >= 0 && c < w) acc[i] += src[rr[i] * w + c];
                    }
                }
#pragma unroll
                for (int i = 0; i < kVarE; ++i)
                    if (ok[i]) hs[tid + i * kBlock] = acc[i];
                lds_barrier();
#pragma unroll
                for (int i = 0; i < kVarE; ++i) {
                    const int e = tid + i * kBlock;
                    ok[i] = e < howo;
                    rr[i] = (int)fdiv((unsigned)(ok[i] ? e : 0), fwo);
                    cc[i] = (ok[i] ? e : 0) - rr[i] * wo;
                    acc[i] = T(0);
                }
                for (int dy = 0; dy < taps; ++dy) {
#pragma unroll
                    for (int i = 0; i < kVarE; ++i) {
                        const int r = rr[i] * st + off + dy * dl;
                        if (ok[i] && r >= 0 && r < h) acc[i] += hs[r * wo + cc[i]];
                    }
                }
#pragma unroll
                for (int i = 0; i < kVarE; ++i)
                    if (ok[i]) dst[tid + i * kBlock] = wt * acc[i] + b;
            } else if (kind == CGP_VAR_HALF) {
                const T* src = lds + ops[k].src[0];
                for (int e = tid; e < howo; e += kBlock) dst[e] = src[e] / T(2);
            } else {   // CGP_VAR_SUM: c0·t0, then o + c_k·t_k (the axpby chain)
                int sl[4];
                T cf[4];
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    sl[t] = ops[k].src[t];
                    cf[t] = (T)ops[k].coef[t];
                }
                for (int e = tid; e < howo; e += kBlock) {
                    T acc = cf[0] * lds[sl[0] + e];
#pragma unroll
                    for (int t = 1; t < 4; ++t)
                        if (sl[t] >= 0) acc = acc + cf[t] * lds[sl[t] + e];
                    dst[e] = acc;
                }
            }
            lds_barrier();
            const long long sto = ops[k].store;
            if (sto >= 0) {
                T* o = p.out + n * sto + g * howo;
                for (int e = tid; e < howo; e += kBlock) o[e] = dst[e];
                const long long qs = ops[k].qstore;
                if (qs >= 0 && g < p.n1) {
                    T* q = p.out + n * p.store_total + p.n1 * qs + g * howo;
                    for (int e = tid; e < howo; e += kBlock) q[e] = T(kXVarScale) * dst[e];
                }
                lds_barrier();   // a later op may reuse the slot
            }
        }
    }
}

template <typename T>
int var_chain_impl(const cgp_var_args* a, void* stream) {
    if (!a || !a->x || !a->out || !a->ops || a->nops <= 0)
        return fail(CGP_EINVAL, "var_chain: NULL pointer or empty op list");
    if (a->n1 <= 0 || a->n2 < 0 || (a->n2 > 0 && !a->y) || a->channels <= 0 || a->h <= 0 ||
        a->w <= 0 || a->store_total <= 0)
        return fail(CGP_EINVAL, "var_chain: bad sizes");
    const long long lds = (long long)a->lds_elems * (long long)sizeof(T);
    if (a->lds_elems <= 0 || lds > 64 * 1024)
        return fail(CGP_EINVAL, "var_chain: LDS footprint %lld bytes out of range", lds);
    VarChainP<T> p;
    p.x = static_cast<const T*>(a->x);
    p.y = static_cast<const T*>(a->y ? a->y : a->x);
    p.out = static_cast<T*>(a->out);
    p.ops = a->ops;
    p.n1 = a->n1;
    p.n2 = a->n2;
    p.store_total = a->store_total;
    p.nops = a->nops;
    p.channels = a->channels;
    p.hw_in = a->h * a->w;
    p.lds_elems = a->lds_elems;
    p.scratch = a->scratch;
    if (a->scratch < 0 || a->scratch >= a->lds_elems)
        return fail(CGP_EINVAL, "var_chain: scratch offset out of range");
    if ((long long)a->h * a->w > (long long)kVarE * kBlock)
        return fail(CGP_EINVAL, "var_chain: maps larger than %d pixels", kVarE * kBlock);
    const long long n = a->n1 + a->n2;
    const long long grid = n < 65536 ? n : 65536;
    hipLaunchKernelGGL((var_chain_kernel<T>), dim3((unsigned)grid), dim3(kBlock), (size_t)lds,
                       as_stream(stream), p);
    return check_launch("var_chain_kernel");
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
    if (a->h <= 0 || a->w <= 0 || a->ho <= 0 || a->wo <= 0 || (long long)a->h * a->w >= (1 << 24))
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

// persistent grid: exactly as many workgroups as can be resident at once (registers and
// LDS both counted by the occupancy query), so no workgroup starts late
template <typename T, int TAPS>
int launch_conv(const ConvP<T>& p, size_t lds, hipStream_t s) {
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, conv_cov_kernel<T, TAPS>, kBlock,
                                                     lds) != hipSuccess || per_cu < 1) {
        (void)hipGetLastError();
        per_cu = 1;
    }
    const long long grid = std::min<long long>(p.nchunks, (long long)per_cu * device_cus());
    hipLaunchKernelGGL((conv_cov_kernel<T, TAPS>), dim3((unsigned)grid), dim3(kBlock), lds, s,
                       p);
    return check_launch("conv_cov_kernel");
}

template <typename T, class G, int PRE, bool POST, bool ADD>
int launch_geo(const cgp_conv_args* a, hipStream_t s) {
    using L = GeoLayout<T, G>;
    GeoP<T> p;
    p.in = static_cast<const T*>(a->in);
    p.in_y = static_cast<const T*>(a->in_y);
    p.out = static_cast<T*>(a->out);
    p.addend = static_cast<const T*>(a->addend);
    p.pre_xx = static_cast<const T*>(a->pre_xx);
    p.pre_yy = static_cast<const T*>(a->pre_yy);
    p.post_xx = static_cast<const T*>(a->post_xx);
    p.post_yy = static_cast<const T*>(a->post_yy);
    p.nmaps = a->nmaps;
    p.nchunks = (a->nmaps + L::MB - 1) / L::MB;
    p.n2 = make_fastdiv((unsigned)(a->n2 > 0 ? a->n2 : 1));
    p.channels = a->channels;
    p.pre = a->pre;
    p.post = a->post;
    p.add = a->addend != nullptr;
    p.same = a->same;
    p.diag = a->diag;
    p.weight = (T)a->weight;
    p.bias = (T)a->bias;
    const size_t lds = (size_t)L::ELEMS * sizeof(T);
    auto kern = conv_geo_kernel<T, G, PRE, POST, ADD>;
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, kBlock, lds) != hipSuccess ||
        per_cu < 1) {
        (void)hipGetLastError();
        per_cu = 1;
    }
    const long long grid = std::min<long long>(p.nchunks, (long long)per_cu * device_cus());
    hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(kBlock), lds, s, p);
    return check_launch("conv_geo_kernel");
}

// the fused (pre, post, add) combinations the program fuser emits
template <typename T, class G>
int launch_geo_mode(const cgp_conv_args* a, hipStream_t s, bool* handled) {
    const bool post = a->post == CGP_POST_RELU, add = a->addend != nullptr;
    *handled = true;
    switch (a->pre * 4 + post * 2 + add) {
        case 0: return launch_geo<T, G, CGP_PRE_NONE, false, false>(a, s);
        case 2: return launch_geo<T, G, CGP_PRE_NONE, true, false>(a, s);
        case 1: return launch_geo<T, G, CGP_PRE_NONE, false, true>(a, s);
        case 3: return launch_geo<T, G, CGP_PRE_NONE, true, true>(a, s);
        case 6: return launch_geo<T, G, CGP_PRE_RELU, true, false>(a, s);
        case 10: return launch_geo<T, G, CGP_PRE_MOMENTS, true, false>(a, s);
        case 8: return launch_geo<T, G, CGP_PRE_MOMENTS, false, false>(a, s);
    }
    *handled = false;
    return CGP_OK;
}

// compile-time-geometry launch; *handled = false when the shape/mode is not in the table
template <typename T>
int conv_geo_impl(const cgp_conv_args* a, void* stream, bool* handled) {
    *handled = false;
    if (a->dilation != 1 || a->maps_per_block != 0 || (a->flags & CGP_FLAG_EXACT_RELU))
        return CGP_OK;
    hipStream_t s = as_stream(stream);
#define CGP_GEO_CASE(h_, w_, ho_, wo_, k_, s_, o_)                                         \
    if (a->h == h_ && a->w == w_ && a->ho == ho_ && a->wo == wo_ && a->taps == k_ &&       \
        a->stride == s_ && a->offset == o_)                                               \
        return launch_geo_mode<T, Geo<h_, w_, ho_, wo_, k_, s_, o_>>(a, s, handled);
    CGP_GEOMETRIES(CGP_GEO_CASE)
#undef CGP_GEO_CASE
    return CGP_OK;
}

template <typename T>
int conv_impl(const cgp_conv_args* a, void* stream) {
    int rc = conv_out_check(a);
    if (rc) return rc;
    if (!(a->flags & CGP_FLAG_GENERIC_CONV)) {
        bool handled = false;
        rc = conv_geo_impl<T>(a, stream, &handled);
        if (rc || handled) return rc;
    }
    const int hw = a->h * a->w;
    // zero halo around each staged map: every tap read lands inside the padded plane
    const int span = (a->taps - 1) * a->dilation;
    const int plo = a->offset < 0 ? -a->offset : 0;
    const int phi_r = std::max(0, (a->ho - 1) * a->stride + a->offset + span - (a->h - 1));
    const int phi_c = std::max(0, (a->wo - 1) * a->stride + a->offset + span - (a->w - 1));
    const int hp = a->h + plo + phi_r, wp = a->w + plo + phi_c;
    int mpb = maps_per_chunk(hw, a->maps_per_block);
    auto lds_of = [&](int m) {
        const size_t in_elems = ((size_t)m * hp * wp + 1) & ~(size_t)1;  // 16-B aligned
        return (in_elems + (size_t)m * hp * a->wo) * sizeof(T);
    };
    while (mpb > 1 && lds_of(mpb) > (size_t)kMaxLds) --mpb;
    if (lds_of(mpb) > (size_t)kMaxLds)
        return fail(CGP_EINVAL, "conv: one %dx%d map does not fit the LDS budget", a->h, a->w);
    if ((long long)mpb * hw > kChunkElems && (long long)mpb * hw >= (1LL << 30))
        return fail(CGP_EINVAL, "conv: chunk too large");
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
    p.nchunks = (a->nmaps + mpb - 1) / mpb;
    p.n2 = make_fastdiv((unsigned)(a->n2 > 0 ? a->n2 : 1));
    p.dw = make_fastdiv((unsigned)a->w);
    p.dhw = make_fastdiv((unsigned)hw);
    p.dwo = make_fastdiv((unsigned)a->wo);
    p.dhowo = make_fastdiv((unsigned)(a->ho * a->wo));
    p.h = a->h;
    p.w = a->w;
    p.ho = a->ho;
    p.wo = a->wo;
    p.hp = hp;
    p.wp = wp;
    p.plo_r = plo;
    p.plo_c = plo;
    p.c0 = a->offset + plo;
    p.r0 = a->offset + plo;
    p.taps = a->taps;
    p.stride = a->stride;
    p.dil = a->dilation;
    p.channels = a->channels;
    p.pre = a->pre;
    p.post = a->post;
    p.add = a->addend != nullptr;
    p.same = a->same;
    p.diag = a->diag;
    p.exact = (a->flags & CGP_FLAG_EXACT_RELU) != 0;
    p.mpb = mpb;
    p.hs_offset = (int)(((size_t)mpb * hp * wp + 1) & ~(size_t)1);
    p.weight = (T)a->weight;
    p.bias = (T)a->bias;
    const size_t lds = lds_of(mpb);
    hipStream_t s = as_stream(stream);
    switch (a->taps) {
        case 1: return launch_conv<T, 1>(p, lds, s);
        case 2: return launch_conv<T, 2>(p, lds, s);
        case 3: return launch_conv<T, 3>(p, lds, s);
        case 4: return launch_conv<T, 4>(p, lds, s);
        case 5: return launch_conv<T, 5>(p, lds, s);
        case 7: return launch_conv<T, 7>(p, lds, s);
        default: return launch_conv<T, 0>(p, lds, s);
    }
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
    p.n2 = make_fastdiv((unsigned)a->n2);
    p.dhw = make_fastdiv((unsigned)a->hw);
    p.hw = a->hw;
    p.same = a->same;
    p.diag = a->diag;
    p.exact = (a->flags & CGP_FLAG_EXACT_RELU) != 0;
    // one chunk of whole maps per workgroup, at most kEMax elements per thread
    p.mpb = std::max(1, kChunkElems / a->hw);
    if (a->hw > kChunkElems) return fail(CGP_EINVAL, "relu: map of %d pixels too large", a->hw);
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
                       as_stream(stream), x, y, nmaps, make_fastdiv((unsigned)n2),
                       make_fastdiv((unsigned)hw), c, hw, diag, mpb, xy);
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

// rocBLAS state per device, created on first use and kept for the process lifetime: the
// handle, the lock that serialises its users (a handle carries one stream), and a device
// word for potrf's info (no allocation per call).  Callers on different devices never
// contend: the registry lock is held only for the lookup.
struct BlasDev {
    rocblas_handle h = nullptr;
    std::mutex mu;
    int64_t* dinfo = nullptr;
    int64_t* dinfos = nullptr;     // one info word per diagonal block (chol_blocked)
    int64_t ninfos = 0;
    hipEvent_t ev[4] = {};         // cgp_chol_solve_f64 phase marks (created on first solve)
    double phase_ms[3] = {};       // jitter, factor, potrs of the last solve
    bool timed = false;
};
std::mutex g_blas_reg_mu;
std::map<int, BlasDev*> g_blas;

int blas_dev(hipStream_t s, BlasDev** out) {
    int dev = 0;
    CGP_HIP(stream_device(s, &dev));
    BlasDev* b = nullptr;
    {
        std::lock_guard<std::mutex> lk(g_blas_reg_mu);
        auto it = g_blas.find(dev);
        if (it == g_blas.end()) it = g_blas.emplace(dev, new BlasDev).first;
        b = it->second;
    }
    std::lock_guard<std::mutex> lk(b->mu);
    if (!b->h) {
        int cur = 0;
        CGP_HIP(hipGetDevice(&cur));
        CGP_HIP(hipSetDevice(dev));
        rocblas_handle nh;
        rocblas_status st = rocblas_create_handle(&nh);
        hipError_t e = hipSuccess;
        if (st == rocblas_status_success)
            e = hipMalloc(reinterpret_cast<void**>(&b->dinfo), sizeof(int64_t));
        (void)hipSetDevice(cur);
        if (st != rocblas_status_success)
            return fail(CGP_EBLAS, "rocblas_create_handle: %s", rocblas_status_to_string(st));
        if (e != hipSuccess) {
            (void)rocblas_destroy_handle(nh);
            return fail(CGP_EHIP, "blas: info word: %s", hipGetErrorString(e));
        }
        b->h = nh;
    }
    *out = b;
    return CGP_OK;
}

#define CGP_BLAS(call)                                                                 \
    do {                                                                               \
        rocblas_status st_ = (call);                                                   \
        if (st_ != rocblas_status_success)                                             \
            return fail(CGP_EBLAS, "%s: %s", #call, rocblas_status_to_string(st_));    \
    } while (0)

// Blocked right-looking Cholesky of the column-major LOWER triangle (= the row-major upper
// triangle the reference's files fill), panel nb:
//   for each diagonal block k:  A11 = L11·L11ᵀ (rocsolver dpotrf_64 on nb × nb),
//                               A21 ← A21·L11⁻ᵀ (dtrsm), A22 ← A22 − A21·A21ᵀ (dsyrk, lower).
// The trailing dsyrk carries ~all of the n³/3 flops at nb = 2048; rocSOLVER's own potrf
// blocks far smaller and reached 33-35 TF at n = 60 000 on the MI355X, this form 58.9 TF
// (0.75 of the fp64 peak; tools/solve_bench.hip, profiles/r3).  Only the lower triangle is
// read or written, so the NaN strictly-upper part stays untouched.  Each block's potrf
// writes its own info word; *info = the first failing leading minor (1-based), 0 if PD.
#ifndef CGP_CHOL_NB
#define CGP_CHOL_NB 2048
#endif
int64_t chol_nb() {
    static const int64_t nb = [] {
        const char* e = getenv("CGP_CHOL_NB");
        const long long v = e ? atoll(e) : 0;
        return v >= 64 ? (int64_t)v : (int64_t)CGP_CHOL_NB;
    }();
    return nb;
}

int chol_blocked(BlasDev* b, hipStream_t s, double* a, int64_t n, int64_t lda, int64_t nb,
                 int64_t* info) {
    rocblas_handle h = b->h;
    const int64_t nblk = (n + nb - 1) / nb;
    if (b->ninfos < nblk) {   // on the stream's device (the caller's current one may differ)
        int dev = 0, cur = 0;
        CGP_HIP(stream_device(s, &dev));
        CGP_HIP(hipGetDevice(&cur));
        CGP_HIP(hipSetDevice(dev));
        if (b->dinfos) (void)hipFree(b->dinfos);
        b->dinfos = nullptr;
        b->ninfos = 0;
        const hipError_t e = hipMalloc(reinterpret_cast<void**>(&b->dinfos), sizeof(int64_t) * nblk);
        (void)hipSetDevice(cur);
        if (e != hipSuccess) return fail(CGP_EHIP, "chol: info words: %s", hipGetErrorString(e));
        b->ninfos = nblk;
    }
    CGP_HIP(hipMemsetAsync(b->dinfos, 0, sizeof(int64_t) * nblk, s));
    CGP_BLAS(rocblas_set_pointer_mode(h, rocblas_pointer_mode_host));
    const double one = 1.0, mone = -1.0;
    for (int64_t blk = 0; blk < nblk; ++blk) {
        const int64_t k = blk * nb, kb = n - k < nb ? n - k : nb, m = n - k - kb;
        double* a11 = a + k * lda + k;
        CGP_BLAS(rocsolver_dpotrf_64(h, rocblas_fill_lower, kb, a11, lda, b->dinfos + blk));
        if (m <= 0) break;
        double* a21 = a11 + kb;
        double* a22 = a + (k + kb) * lda + (k + kb);
        CGP_BLAS(rocblas_dtrsm_64(h, rocblas_side_right, rocblas_fill_lower,
                                  rocblas_operation_transpose, rocblas_diagonal_non_unit, m, kb,
                                  &one, a11, lda, a21, lda));
        CGP_BLAS(rocblas_dsyrk_64(h, rocblas_fill_lower, rocblas_operation_none, m, kb, &mone, a21,
                                  lda, &one, a22, lda));
    }
    std::vector<int64_t> hinfo(nblk);
    CGP_HIP(hipMemcpyAsync(hinfo.data(), b->dinfos, sizeof(int64_t) * nblk,
                           hipMemcpyDeviceToHost, s));
    CGP_HIP(hipStreamSynchronize(s));
    *info = 0;
    for (int64_t blk = 0; blk < nblk; ++blk)
        if (hinfo[blk] > 0) {
            *info = blk * nb + hinfo[blk];
            break;
        }
    return CGP_OK;
}

}  // namespace

// ==================================================================================
// C ABI
// ==================================================================================
extern "C" {

int cgp_abi_version(void) { return CGP_ABI_VERSION; }

double cgp_net_xvar_scale(void) { return kXVarScale; }
const char* cgp_last_error(void) { return g_last_error.c_str(); }
size_t cgp_conv_args_size(void) { return sizeof(cgp_conv_args); }
size_t cgp_relu_args_size(void) { return sizeof(cgp_relu_args); }
size_t cgp_var_op_size(void) { return sizeof(cgp_var_op); }
size_t cgp_var_args_size(void) { return sizeof(cgp_var_args); }
int cgp_var_chain_f64(const cgp_var_args* a, void* stream) { return var_chain_impl<double>(a, stream); }
int cgp_var_chain_f32(const cgp_var_args* a, void* stream) { return var_chain_impl<float>(a, stream); }

int cgp_selftest(void) {
    // FastDiv against exact division: every divisor the kernels use, edge numerators
    const unsigned divs[] = {1, 2, 3, 5, 7, 8, 14, 28, 49, 196, 784, 1000, 1024, 4095, 4096,
                             40000, 65535, 1000003u, 0x7fffffffu};
    unsigned long long seed = 0x9e3779b97f4a7c15ull;
    for (unsigned d : divs) {
        const FastDiv f = make_fastdiv(d);
        const unsigned edge[] = {0u, 1u, d - 1, d, d + 1, 2 * d - 1, 0x7ffffffeu, 0x7fffffffu};
        for (unsigned n : edge)
            if (n < 0x80000000u && fdiv(n, f) != n / d)
                return fail(CGP_EINVAL, "fastdiv %u / %u", n, d);
        for (int k = 0; k < 200000; ++k) {
            seed = seed * 6364136223846793005ull + 1442695040888963407ull;
            const unsigned n = (unsigned)(seed >> 33) & 0x7fffffffu;
            if (fdiv(n, f) != n / d) return fail(CGP_EINVAL, "fastdiv %u / %u", n, d);
        }
    }
    return CGP_OK;
}

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
int cgp_scale_batch_f64(int32_t count, const double* const* src, double* const* dst,
                        const int64_t* n, double alpha, void* stream) {
    if (count < 0 || (count > 0 && (!src || !dst || !n)))
        return fail(CGP_EINVAL, "scale_batch: bad arguments");
    for (int base = 0; base < count; base += kScaleBatch) {
        ScaleBatch b{};
        long long most = 0;
        const int m = count - base < kScaleBatch ? count - base : kScaleBatch;
        for (int k = 0; k < m; ++k) {
            b.src[k] = src[base + k];
            b.dst[k] = dst[base + k];
            b.n[k] = n[base + k];
            if (b.n[k] < 0 || (b.n[k] > 0 && (!b.src[k] || !b.dst[k])))
                return fail(CGP_EINVAL, "scale_batch: buffer %d", base + k);
            if (b.n[k] > most) most = b.n[k];
        }
        if (most == 0) continue;
        hipLaunchKernelGGL(scale_batch_kernel, dim3(grid_for(most), m), dim3(kBlock), 0,
                           as_stream(stream), b, alpha);
        const int rc = check_launch("scale_batch_kernel");
        if (rc != CGP_OK) return rc;
    }
    return CGP_OK;
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

int cgp_sym_mirror_f64(double* k, int64_t n, int64_t ldk, double* diag, void* stream) {
    if (!k || !diag || n <= 0 || ldk < n)
        return fail(CGP_EINVAL, "sym_mirror: bad arguments (n=%lld ldk=%lld)", (long long)n,
                    (long long)ldk);
    const long long tiles = (n + kSymT - 1) / kSymT;
    if (tiles > 65535) return fail(CGP_EINVAL, "sym_mirror: n=%lld too large", (long long)n);
    hipLaunchKernelGGL(sym_mirror_kernel, dim3((unsigned)tiles, (unsigned)tiles), dim3(kBlock),
                       0, as_stream(stream), k, (long long)n, (long long)ldk, diag);
    return check_launch("sym_mirror_kernel");
}

int cgp_sym_residual_f64(const double* k, int64_t n, int64_t ldk, const double* diag,
                         const double* x, double* r, int64_t nrhs, int64_t ldx, double* sumsq,
                         void* stream) {
    if (!k || !diag || !x || !r || !sumsq || n <= 0 || ldk < n || nrhs <= 0 || ldx < n)
        return fail(CGP_EINVAL, "sym_residual: bad arguments (n=%lld nrhs=%lld)",
                    (long long)n, (long long)nrhs);
    const long long tiles = (n + kSymT - 1) / kSymT;
    const long long chunks = (tiles + kSymChunk - 1) / kSymChunk;
    if (tiles > 65535) return fail(CGP_EINVAL, "sym_residual: n=%lld too large", (long long)n);
    hipStream_t s = as_stream(stream);
    for (int64_t q0 = 0; q0 < nrhs; q0 += kSymRhs) {
        // the tiles' squares once: only the first group of right-hand sides adds them up
        hipLaunchKernelGGL(sym_residual_kernel, dim3((unsigned)tiles, (unsigned)chunks),
                           dim3(kBlock), 0, s, k, (long long)n, (long long)ldk, diag,
                           x + q0 * ldx, r + q0 * ldx,
                           (int)std::min<int64_t>(kSymRhs, nrhs - q0), (long long)ldx,
                           q0 == 0 ? sumsq : nullptr);
        const int rc = check_launch("sym_residual_kernel");
        if (rc) return rc;
    }
    return CGP_OK;
}

int cgp_chol_solve_f64(double* k, int64_t n, int64_t ldk, double* bt, int64_t nrhs,
                       int64_t ldb, double jitter, int64_t* info, void* stream) {
    return cgp_chol_solve_f64_timed(k, n, ldk, bt, nrhs, ldb, jitter, info, nullptr, stream);
}

int cgp_chol_solve_f64_timed(double* k, int64_t n, int64_t ldk, double* bt, int64_t nrhs,
                             int64_t ldb, double jitter, int64_t* info, double* phase_ms,
                             void* stream) {
    if (phase_ms)
        for (int q = 0; q < 3; ++q) phase_ms[q] = -1.0;   // no phases unless the solve ran
    if (!k || !bt || !info) return fail(CGP_EINVAL, "chol_solve: NULL argument");
    if (n <= 0 || ldk < n || nrhs <= 0 || ldb < n)
        return fail(CGP_EINVAL, "chol_solve: bad sizes n=%lld ldk=%lld nrhs=%lld ldb=%lld",
                    (long long)n, (long long)ldk, (long long)nrhs, (long long)ldb);
    hipStream_t s = as_stream(stream);
    BlasDev* b = nullptr;
    int rc = blas_dev(s, &b);
    if (rc) return rc;
    std::lock_guard<std::mutex> lk(b->mu);
    rocblas_handle h = b->h;
    CGP_BLAS(rocblas_set_stream(h, s));
    if (!b->ev[0]) {
        int dev = 0, cur = 0;
        CGP_HIP(stream_device(s, &dev));
        CGP_HIP(hipGetDevice(&cur));
        CGP_HIP(hipSetDevice(dev));
        hipError_t e = hipSuccess;
        for (int q = 0; q < 4 && e == hipSuccess; ++q) e = hipEventCreate(&b->ev[q]);
        (void)hipSetDevice(cur);
        if (e != hipSuccess) return fail(CGP_EHIP, "chol: events: %s", hipGetErrorString(e));
    }
    b->timed = false;
    CGP_HIP(hipEventRecord(b->ev[0], s));
    if (jitter != 0.0) {
        hipLaunchKernelGGL(diag_add_kernel, dim3(grid_for(n)), dim3(kBlock), 0, s, k,
                           (long long)n, (long long)ldk, jitter);
        rc = check_launch("diag_add_kernel");
        if (rc) return rc;
    }
    CGP_HIP(hipEventRecord(b->ev[1], s));
    // row-major upper triangle == column-major lower triangle
    int64_t hinfo = -1;
    const int64_t nb = chol_nb();
    if (n > nb) {
        rc = chol_blocked(b, s, k, n, ldk, nb, &hinfo);
        if (rc) return rc;
    } else {
        CGP_BLAS(rocsolver_dpotrf_64(h, rocblas_fill_lower, n, k, ldk, b->dinfo));
        CGP_HIP(hipMemcpyAsync(&hinfo, b->dinfo, sizeof(int64_t), hipMemcpyDeviceToHost, s));
        CGP_HIP(hipStreamSynchronize(s));
    }
    CGP_HIP(hipEventRecord(b->ev[2], s));
    *info = hinfo;
    if (hinfo == 0)
        CGP_BLAS(rocsolver_dpotrs_64(h, rocblas_fill_lower, n, nrhs, k, ldk, bt, ldb));
    CGP_HIP(hipEventRecord(b->ev[3], s));
    CGP_HIP(hipStreamSynchronize(s));
    for (int q = 0; q < 3; ++q) {
        float ms = 0.f;
        CGP_HIP(hipEventElapsedTime(&ms, b->ev[q], b->ev[q + 1]));
        b->phase_ms[q] = ms;
        if (phase_ms) phase_ms[q] = ms;    // this call's own phases, under the device lock
    }
    b->timed = true;
    return CGP_OK;
}

int cgp_chol_last_phases(void* stream, double* ms) {
    if (!ms) return fail(CGP_EINVAL, "chol_last_phases: NULL argument");
    BlasDev* b = nullptr;
    const int rc = blas_dev(as_stream(stream), &b);
    if (rc) return rc;
    std::lock_guard<std::mutex> lk(b->mu);
    if (!b->timed) return fail(CGP_EINVAL, "chol_last_phases: no solve on this device yet");
    for (int q = 0; q < 3; ++q) ms[q] = b->phase_ms[q];
    return CGP_OK;
}

int cgp_gemm_f64(const double* a, const double* b, double* c, int64_t m, int64_t n,
                 int64_t kdim, void* stream) {
    if (!a || !b || !c || m <= 0 || n <= 0 || kdim <= 0)
        return fail(CGP_EINVAL, "gemm: bad arguments");
    BlasDev* bd = nullptr;
    int rc = blas_dev(as_stream(stream), &bd);
    if (rc) return rc;
    std::lock_guard<std::mutex> lk(bd->mu);
    rocblas_handle h = bd->h;
    CGP_BLAS(rocblas_set_stream(h, as_stream(stream)));
    const double one = 1.0, zero = 0.0;
    CGP_BLAS(rocblas_set_pointer_mode(h, rocblas_pointer_mode_host));
    // row-major C = A·B  <=>  column-major Cᵀ = Bᵀ·Aᵀ
    CGP_BLAS(rocblas_dgemm_64(h, rocblas_operation_none, rocblas_operation_none, n, m, kdim,
                              &one, b, n, a, kdim, &zero, c, n));
    return CGP_OK;
}

int cgp_pred_var_f64(const double* k, int64_t n, int64_t ldk, double* kxz, int64_t m,
                     int64_t ldz, const double* kz_diag, double* var, void* stream) {
    if (!k || !kxz || !kz_diag || !var) return fail(CGP_EINVAL, "pred_var: NULL argument");
    if (n <= 0 || ldk < n || m < 0 || ldz < n)
        return fail(CGP_EINVAL, "pred_var: bad sizes n=%lld ldk=%lld m=%lld ldz=%lld",
                    (long long)n, (long long)ldk, (long long)m, (long long)ldz);
    if (m == 0) return CGP_OK;
    hipStream_t s = as_stream(stream);
    BlasDev* bd = nullptr;
    int rc = blas_dev(s, &bd);
    if (rc) return rc;
    {
        std::lock_guard<std::mutex> lk(bd->mu);
        rocblas_handle h = bd->h;
        CGP_BLAS(rocblas_set_stream(h, s));
        CGP_BLAS(rocblas_set_pointer_mode(h, rocblas_pointer_mode_host));
        const double one = 1.0;
        // column-major: L = the factor's lower triangle (n×n, Kxx = L·Lᵀ), B = Kxz (n×m,
        // ld ldz).  L·V = B  <=>  V = U⁻ᵀ Kxz with U = Lᵀ the row-major upper factor.
        CGP_BLAS(rocblas_dtrsm_64(h, rocblas_side_left, rocblas_fill_lower,
                                  rocblas_operation_none, rocblas_diagonal_non_unit, n, m,
                                  &one, k, ldk, kxz, ldz));
    }
    const unsigned grid = (unsigned)(m < 65536 ? m : 65536);
    hipLaunchKernelGGL(row_sumsq_sub_kernel, dim3(grid), dim3(kBlock), 0, s, kxz,
                       (long long)m, (long long)n, (long long)ldz, kz_diag, var);
    return check_launch("row_sumsq_sub_kernel");
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
