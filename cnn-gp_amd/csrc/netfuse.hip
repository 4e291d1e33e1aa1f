// netfuse.hip — the whole pair program of a network in ONE kernel (cgp_net_*).
//
// The layer-by-layer path (cnngp.hip) streams every pair map through HBM once per fused
// op: ~100-500 KB of traffic per pair, so it is HBM-bound.  Here one workgroup (two
// waves) owns one (i, j) pair at a time and runs every op of the network on LDS-resident
// planes; the only global traffic per pair is the two input images and the per-image
// variance maps the ReLUs read (both shared by many pairs, so L2/MALL-resident) plus
// the one K[i, j] it writes.  The kernel is fp64-VALU bound.
//
// Reference semantics: moments kernels.py:44-47, Conv2d.propagate kernels.py:92-98,
// ReLU.propagate kernels.py:134-165, Sequential kernels.py:184-187, Sum/Mixture
// kernels.py:220-254.  The host (cnn_gp/netplan.py) lowers the module tree into a list
// of cgp_net_op over LDS slots; this file only executes the list.
//
// Per pair, per conv: a row pass writes horizontal window sums of every input row into
// the row-sum scratch `hs` ([HSR][WO]; rows outside the input are zero), then a column
// pass finishes the windows for R3 output rows per item, applies w·Σ + b, the ReLU (with
// variances prefetched before the row pass) and the residual add, and writes the output
// slot.  Geometry is compile time (one instantiation per conv shape the reference
// configs use), so every LDS offset inside a pass is an immediate.

#include "cgp_common.h"


#include <map>
#include <mutex>
#include <utility>
#include <algorithm>
#include <climits>

using namespace cgp;

namespace {

constexpr int kNT = 128;  // threads per workgroup (one pair): two waves
// threads of a workgroup carrying NP pairs: NP == 2 is two one-pair halves on four waves
// (units u and u + 1, the same image i: the i-side variance loads of the halves meet in
// L1 and each barrier serves both pairs; net_kernel); the small-map stages pack 4 / 16
// pairs on two waves.  Ops only ever run on one half (NP = 1) or on NP = 4 / 16.  (Four
// one-pair slices on 512 threads measured -15% fp64: LDS then admits 2 workgroups per CU.)
constexpr int kSplit = 2;
template <int NP>
constexpr int kNTof = NP == 2 ? kSplit * kNT : kNT;
// pair units a workgroup takes per step of the walk
template <int NP>
constexpr int kUnitsOf = NP == 2 ? kSplit : NP;
constexpr int kSTL = 3;             // log2(kST) (16² / 32² supertiles measured ±0.7%)
constexpr int kST = 1 << kSTL;      // supertile edge: pairs are walked in 8x8 (i, j) blocks
constexpr int kEw = 4;          // elementwise ops: pixels per thread per pass

// R | len outputs per item, chosen to minimise rounds·(per-item cost) with ≤ 8 outputs
// (register budget); ties go to the larger R (fewer LDS reads per output).
constexpr int pick_r(int lines, int len, int taps, int s, int epi, int nt) {
    int best = 1;
    long long best_cost = LLONG_MAX;
    for (int r = 1; r <= 8 && r <= len; ++r) {
        if (len % r) continue;
        const int items = lines * (len / r);
        const int rounds = (items + nt - 1) / nt;
        const long long cost = (long long)rounds * (epi * r + (r - 1) * s + taps);
        if (cost < best_cost || (cost == best_cost && r > best)) {
            best = r;
            best_cost = cost;
        }
    }
    return best;
}

// NP_: pairs per workgroup (their items share the passes; per-pair counts below)
template <int H_, int W_, int HO_, int WO_, int TAPS_, int S_, int OFF_, int NP_ = 1>
struct NG {
    static constexpr int H = H_, W = W_, HO = HO_, WO = WO_, TAPS = TAPS_, S = S_, OFF = OFF_;
    static constexpr int NP = NP_;
    static constexpr int NT = kNT;
    static_assert(NP_ != 2, "two-pair workgroups run their ops as one-pair halves");
    static constexpr int HW = H * W, HOWO = HO * WO;
    static constexpr bool POINT = TAPS == 1 && OFF == 0;
    static constexpr bool REDUCE = HO == 1 && WO == 1 && OFF == 0 && TAPS == H && TAPS == W;
    static constexpr int HSR = (HO - 1) * S + TAPS;           // hs rows; row q <-> input q+OFF
    static constexpr int Q0 = OFF < 0 ? -OFF : 0;              // first hs row backed by input
    static constexpr int Q1 = HSR < H - OFF ? HSR : H - OFF;   // one past the last
    static constexpr int NVR = Q1 - Q0;                        // input rows the row pass reads
    static constexpr int R2 = pick_r(NVR * NP, WO, TAPS, S, 2, NT);
    static constexpr int R3 = pick_r(WO * NP, HO, TAPS, S, 8, NT);
    static constexpr int WIN2 = (R2 - 1) * S + TAPS, WIN3 = (R3 - 1) * S + TAPS;
    static constexpr int NG2 = WO / R2, NH = NVR * NG2, KH = (NP * NH + NT - 1) / NT;
    static constexpr int NG3 = HO / R3, NV = NG3 * WO, KV = (NP * NV + NT - 1) / NT;
    static constexpr int NZ = (HSR - NVR) * WO;                // zero cells of hs
    // windows of at most 3 taps (the ResNets' 3x3 convs) run in one pass straight from the
    // source slot: no row-sum scratch, so a smaller arena
    static constexpr bool DIRECT = !POINT && !REDUCE && TAPS <= 3;
    static constexpr int HS_ELEMS = (POINT || REDUCE || DIRECT) ? 2 : HSR * WO;
};

// The fused kernel's conv shapes: (H, W, HO, WO, taps, stride, offset) — every conv of the
// reference configs plus their CIFAR-size analogues.
#define CGP_NET_GEOMETRIES(X)          \
    X(28, 28, 28, 28, 7, 1, -3)        \
    X(28, 28, 28, 28, 4, 1, -1)        \
    X(28, 28, 28, 28, 3, 1, -1)        \
    X(28, 28, 28, 28, 1, 1, 0)         \
    X(28, 28, 14, 14, 3, 2, -1)        \
    X(28, 28, 14, 14, 1, 2, 0)         \
    X(28, 28, 1, 1, 28, 1, 0)          \
    X(14, 14, 14, 14, 3, 1, -1)        \
    X(14, 14, 7, 7, 3, 2, -1)          \
    X(14, 14, 7, 7, 1, 2, 0)           \
    X(7, 7, 7, 7, 3, 1, -1)            \
    X(7, 7, 1, 1, 7, 1, 0)             \
    X(1, 1, 1, 1, 1, 1, 0)             \
    X(32, 32, 32, 32, 3, 1, -1)        \
    X(32, 32, 32, 32, 1, 1, 0)         \
    X(32, 32, 16, 16, 3, 2, -1)        \
    X(32, 32, 16, 16, 1, 2, 0)         \
    X(16, 16, 16, 16, 3, 1, -1)        \
    X(16, 16, 8, 8, 3, 2, -1)          \
    X(16, 16, 8, 8, 1, 2, 0)           \
    X(8, 8, 8, 8, 3, 1, -1)            \
    X(8, 8, 1, 1, 8, 1, 0)             \
    X(14, 14, 1, 1, 14, 1, 0)          \
    X(16, 16, 1, 1, 16, 1, 0)          \
    X(32, 32, 1, 1, 32, 1, 0)

struct GeoRow {
    int h, w, ho, wo, taps, s, off, hs_elems;
};
#define CGP_NET_ROW(h, w, ho, wo, k, s, o) {h, w, ho, wo, k, s, o, NG<h, w, ho, wo, k, s, o>::HS_ELEMS},
constexpr GeoRow kGeoTable[] = {CGP_NET_GEOMETRIES(CGP_NET_ROW)};
#undef CGP_NET_ROW
constexpr int kNumGeo = sizeof(kGeoTable) / sizeof(kGeoTable[0]);

// out[o] = Σ_{t<TAPS} w[o·S + t], o < R.  Stride 1 with TAPS ≥ 4: outputs in groups of
// g ≤ TAPS share the common core of their windows; the suffix sums of the first window run
// through the core and the taps after it are prefix sums, so a group costs TAPS + 2g - 4
// adds instead of g(TAPS-1) (7x7: 17 per pass instead of 42).  The round-3 form kept the
// core apart (TAPS + 3g - 6: 22) and measured 2.5% slower on ConvNet GP
// (profiles/r4/ab_r4l_window_sums.log).
template <typename T, int TAPS, int O0, int G, int N, int R>
__device__ __forceinline__ void win_group(const T (&w)[N], T (&out)[R]) {
    T core = w[O0 + G - 1];
#pragma unroll
    for (int t = O0 + G; t < O0 + TAPS; ++t) core += w[t];
    if constexpr (G == 1) {
        out[O0] = core;
    } else {
        // suffix sums of the first window that end in the core, prefix sums of the taps
        // after it (van Herk / Gil-Werman): TAPS + 2G - 4 adds
        T suf[G], right[G];
        suf[G - 1] = core;
#pragma unroll
        for (int o = G - 2; o >= 0; --o) suf[o] = w[O0 + o] + suf[o + 1];
        right[1] = w[O0 + TAPS];
#pragma unroll
        for (int o = 2; o < G; ++o) right[o] = right[o - 1] + w[O0 + TAPS + o - 1];
        out[O0] = suf[0];
#pragma unroll
        for (int o = 1; o < G; ++o) out[O0 + o] = suf[o] + right[o];
    }
}

template <typename T, int TAPS, int O0, int N, int R>
__device__ __forceinline__ void win_groups(const T (&w)[N], T (&out)[R]) {
    if constexpr (O0 < R) {
        constexpr int G = (R - O0) < TAPS ? (R - O0) : TAPS;
        win_group<T, TAPS, O0, G, N, R>(w, out);
        win_groups<T, TAPS, O0 + TAPS, N, R>(w, out);
    }
}

template <typename T, int TAPS, int S, int R>
__device__ __forceinline__ void win_sums(const T (&w)[(R - 1) * S + TAPS], T (&out)[R]) {
    if constexpr (S == 1 && TAPS >= 4 && R > 1) {
        win_groups<T, TAPS, 0, (R - 1) * S + TAPS, R>(w, out);
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

// threadIdx.x through an opaque move: per-thread index math of one op is then recomputed
// inside the op instead of being hoisted out of the pair loop, where it would hold
// registers for every geometry at once (hoisted: -1% fp64, scratch spills in the head
// programs)
// (thread index within its 128-thread half: a two-pair workgroup runs one pair per half)
__device__ __forceinline__ int opaque_tid() {
    static_assert(kNT == 128, "opaque_tid masks to 128-thread halves");
    int t;
    asm volatile("v_and_b32 %0, 0x7f, %1" : "=v"(t) : "v"((int)threadIdx.x));
    return t;
}

// a / d for a >= 0 as an unsigned division (a constant d costs a mul-hi and a shift; the
// signed form needs three more fix-up ops)
__device__ __forceinline__ int udiv(int a, int d) { return (int)((unsigned)a / (unsigned)d); }

// the op table through a generic pointer: per-lane vector loads (the constant address
// space's scalar loads measured -7% on ConvNet: SMEM returns count in lgkmcnt, so every
// LDS wait also drains them)
typedef const cgp_net_op* OpsC;
__device__ __forceinline__ OpsC ops_c(const cgp_net_op* p) { return (OpsC)p; }
__device__ __forceinline__ cgp_net_op load_op(OpsC r) {
    cgp_net_op o;
    o.kind = r->kind;
    o.code = r->code;
    o.src = r->src;
    o.dst = r->dst;
    o.add = r->add;
    o.ws_in = r->ws_in;
    o.ws_out = r->ws_out;
    o.relu = r->relu;
    o.h = r->h;
    o.w = r->w;
    o.div_m = r->div_m;
    o.div_s = r->div_s;
    o.dst2 = r->dst2;
    o.zero_halo = r->zero_halo;
    o.weight = r->weight;
    o.bias = r->bias;
    o.var_x = r->var_x;
    o.var_y = r->var_y;
    o.var2_x = r->var2_x;
    o.var2_y = r->var2_y;
    return o;
}

// global-address-space views: pointers read from the op table are generic, and flat
// loads would also count in lgkmcnt, so every LDS wait would drain them
template <typename T>
using GP = const __attribute__((address_space(1))) T*;
template <typename T>
__device__ __forceinline__ GP<T> gptr(const void* p) {
    return (GP<T>)(const T*)p;
}

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, 64);
    return v;
}

template <typename T>
struct NetP {
    const T* __restrict__ x;
    const T* __restrict__ y;
    T* __restrict__ out;
    const T* __restrict__ kdiag;
    const cgp_net_op* __restrict__ ops;
    unsigned long long* work;   // per-XCD unit counters, zeroed per launch
    long long ldo, units, ubeg, uend;
    unsigned n1, n2, nbi, nbj;
    int nops, channels, hw_in, same, final_slot, hs, lds_elems, exact, final_stage, part;
};

// The pairs an op works on.  NP == 1: (i, j), uniform.  NP > 1: pair q of the group is
// (tab[q], tab[kMaxNP + q]) from the workgroup's pair table in LDS, unit u0 + q.
constexpr int kMaxNP = 16;
// LDS the kernel declares statically (pair table, SUM partials, program records, the
// work-counter slots) on top of the dynamic arenas: every LDS check (net_impl, net_wpe,
// cgp_net_static_lds for the host's planner) counts this reserve
constexpr long long kStaticLds = 1536;
struct Pairs {
    unsigned i, j;
    const unsigned* tab;
    long long u0;
    void* red;   // one-pair code: the pair's two wave partial sums (CGP_NET_CODE_SUM)
};
template <int NP>
__device__ __forceinline__ void pair_q(const Pairs& pr, int q, unsigned& iq, unsigned& jq) {
    if constexpr (NP == 1) {
        iq = pr.i;
        jq = pr.j;
    } else {
        iq = pr.tab[q];
        jq = pr.tab[kMaxNP + q];
    }
}

// EXACT (CGP_FLAG_EXACT_RELU) is a separate instantiation: a call to the out-of-line
// relu_exact would make every register live across it caller-saved
template <bool EXACT, typename T>
__device__ __forceinline__ T relu_of(T c, T v1, T v2, const PolyTab& tab) {
    if constexpr (EXACT)
        return relu_exact_inl(c, v1, v2);
    else
        return relu_fast(c, v1, v2, tab);
}
// The fp64 closed form reads scaled x-side variance maps (relu_q_n: the host passes
// v × cgp_net_xvar_scale() = v/16 from ABI 9, v/4 before, for f64 launches without
// CGP_FLAG_EXACT_RELU) and, when the producing conv scaled its weight and bias by 1/4
// (QIN), a quartered input.
template <typename T, bool EX>
constexpr bool kQuarter = !EX && sizeof(T) == 8;

// R ReLUs in place: v[k] = relu(v[k], u1[k], u2[k]) (QIN: v holds c/4; AD: the fp64 form
// may take the range-adaptive polynomial, see relu_q_n).  The fp32 closed form keeps its
// full polynomial: its adaptive form measured neutral (the fp32 kernel is bound by its
// per-op latency chain, not by issue; profiles/r3/ab_r3f_relu_adapt_f32.log)
template <bool EXACT, bool QIN, typename T, int R, int AD = 0>
__device__ __forceinline__ void relu_n(T (&v)[R], const T (&u1)[R], const T (&u2)[R],
                                       const PolyTab& tab, unsigned long long seg = ~0ull) {
    if constexpr (EXACT) {
#pragma unroll
        for (int k = 0; k < R; ++k) v[k] = relu_exact_inl(v[k], u1[k], u2[k]);
    } else if constexpr (sizeof(T) == 8) {
        relu_q_n<R, QIN, AD>(v, u1, u2, tab, seg);
    } else {
        relu_fast_n<R>(v, u1, u2, tab);
    }
}

// Elementwise-op map sizes with a compile-time instantiation (cgp_net_resolution); any
// other size runs the generic runtime-size path.
#define CGP_NET_RESOLUTIONS(X) X(28, 28) X(14, 14) X(7, 7) X(32, 32) X(16, 16) X(8, 8) X(1, 1)

struct ResRow {
    int h, w;
};
#define CGP_NET_RES_ROW(h, w) {h, w},
constexpr ResRow kResTable[] = {CGP_NET_RESOLUTIONS(CGP_NET_RES_ROW)};
#undef CGP_NET_RES_ROW
constexpr int kNumRes = sizeof(kResTable) / sizeof(kResTable[0]);
constexpr int res_index(int h, int w) {
    for (int n = 0; n < kNumRes; ++n)
        if (kResTable[n].h == h && kResTable[n].w == w) return n;
    return -1;
}

// Output stage shared by every op: v (R results at LDS offsets at[k] of the dst/add
// class, variance-map pixels px[k]) -> [ReLU] -> [+ add] -> dst, and optionally
// relu(result) -> dst2 (the next block's ReLU branch input, saving a separate op).
// An op has the ReLU or dst2, never both, so one set of prefetched variances (u1, u2)
// serves either.
template <typename T, bool EX, bool DU, int R, int AD = 0>
__device__ __forceinline__ void net_out(T* __restrict__ lds, const cgp_net_op& op, T (&v)[R],
                                        const int (&at)[R], const bool (&ok)[R],
                                        const T (&u1)[R], const T (&u2)[R],
                                        const PolyTab& tab, unsigned long long seg = ~0ull) {
    if (op.relu) relu_n<EX, kQuarter<T, EX>, T, R, AD>(v, u1, u2, tab, seg);
    if (op.add >= 0) {
#pragma unroll
        for (int k = 0; k < R; ++k)
            if (ok[k]) v[k] += lds[op.add + at[k]];
    }
#pragma unroll
    for (int k = 0; k < R; ++k)
        if (ok[k]) lds[op.dst + at[k]] = v[k];
    if (DU && op.dst2 >= 0) {
        relu_n<EX, false, T, R, AD>(v, u1, u2, tab, seg);
#pragma unroll
        for (int k = 0; k < R; ++k)
            if (ok[k]) lds[op.dst2 + at[k]] = v[k];
    }
}

// A pointer every lane holds the same value of (an op-record field) as a scalar: loads
// through it take the SGPR-base form (global_load … vOFF, s[BASE] offset:IMM), so a
// variance load costs no 64-bit VALU address arithmetic
__device__ __forceinline__ GP<char> ubase(const void* p) {
    const unsigned long long v = (unsigned long long)p;
    const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)v);
    const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(v >> 32));
    return (GP<char>)(const char*)(((unsigned long long)hi << 32) | lo);
}

// variances for the op's ReLU (var_x/var_y) or its dst2 ReLU (var2_x/var2_y).  x / y are
// uniform bases; xo / yo the byte offsets of the pair's maps when they differ per lane
// (multi-pair stages), else 0 with the image offset folded into the base.  ldx(px, k)
// reads pixel px + k of the x-side map: px is the per-lane part (one 32-bit offset
// register shared by both sides when the offsets are folded), k a compile-time step
// that lands in the instruction's immediate offset.  Per-lane offsets are 32-bit: the
// multi-pair maps are at most 32x32, and net_impl bounds n1, n2 so they cannot wrap.
template <typename T>
struct VarSrc {
    GP<char> x, y;
    unsigned xo, yo;
    bool on;
    __device__ __forceinline__ T ldx(unsigned px, int k = 0) const {
        return *(GP<T>)(x + (size_t)(xo + px * (unsigned)sizeof(T)) + k * (int)sizeof(T));
    }
    __device__ __forceinline__ T ldy(unsigned px, int k = 0) const {
        return *(GP<T>)(y + (size_t)(yo + px * (unsigned)sizeof(T)) + k * (int)sizeof(T));
    }
};
// UNI: i and j are the same in every lane (one pair per workgroup), so their offsets fold
// into the scalar bases
template <typename T, bool UNI>
__device__ __forceinline__ VarSrc<T> var_maps(const void* vx, const void* vy, bool on,
                                              unsigned i, unsigned j, int hw) {
    VarSrc<T> r;
    r.on = on;
    r.x = ubase(vx);
    r.y = ubase(vy);
    if constexpr (UNI) {
        r.x += (size_t)i * (size_t)hw * sizeof(T);   // scalar 64-bit arithmetic
        r.y += (size_t)j * (size_t)hw * sizeof(T);
        r.xo = r.yo = 0;
    } else {
        r.xo = i * (unsigned)hw * (unsigned)sizeof(T);
        r.yo = j * (unsigned)hw * (unsigned)sizeof(T);
    }
    return r;
}
template <typename T, bool UNI>
__device__ __forceinline__ VarSrc<T> var_src(const cgp_net_op& op, unsigned i, unsigned j,
                                             int hw) {
    const bool two = op.dst2 >= 0;
    return var_maps<T, UNI>(two ? op.var2_x : op.var_x, two ? op.var2_y : op.var_y,
                            op.relu != 0 || two, i, j, hw);
}

// ---- CGP_NET_CONV -------------------------------------------------------------------
// G::NP pairs: item it of a pass belongs to pair q = it / (items per pair) and works on
// that pair's LDS arena (q · lds_elems) and variance maps.
// Range-adaptive ReLU in a conv epilogue (relu_q_n): one-pair code votes over the wave
// (AD 1: both waves of a pair hold the same items of it in every workgroup); multi-pair
// stages vote per vote group (AD 2, below).
template <int NP>
constexpr int kAdaptOf = NP == 1 ? 1 : 2;
// Wave priority: a conv raises its waves' issue priority (s_setprio 2) while it sends its
// variance loads and window reads and drops it for the arithmetic epilogue, so the memory
// requests of a wave entering an op go out ahead of the other waves' long ALU runs and
// their latency overlaps that work.  Measured (one B = 1024 Kxz tile,
// profiles/r3/ab_r3u_prio.log): ConvNet +4.5-5%, Residual +4-5%, mnist_as_tf +3% (its 28x28
// head; the multi-pair stages do not move), but the cifar10 head (32x32 maps, four waves
// per SIMD) -3%: applied to maps of at most 28x28 pixels.  Priority 1 / 2 / 3 measure the
// same; raised over the variance loads only, or the window reads only, it loses half or
// more of the gain (profiles/r3/ab_r3x_prio_span.log); around the elementwise ops' loads
// it adds nothing.
constexpr int kPrio = 2;
constexpr int kPrioMaxHW = 28 * 28;
template <int NP, int HW>
constexpr bool kPrioOn = HW <= kPrioMaxHW;
template <int NP, int HW>
__device__ __forceinline__ void prio_mem() {
    if constexpr (kPrioOn<NP, HW>) __builtin_amdgcn_s_setprio(kPrio);
}
template <int NP, int HW>
__device__ __forceinline__ void prio_alu() {
    if constexpr (kPrioOn<NP, HW>) __builtin_amdgcn_s_setprio(0);
}
// Vote groups of a multi-pair stage (AD 2).  Items of pair q are [q·PER, (q+1)·PER) and
// item it runs on lane it % 64 of wave it / 64, so which items of a pair share a wave
// depends on the pair's slot q in the workgroup — a vote over "this pair's lanes of this
// wave" would make a pair's polynomial choice depend on its slot, i.e. on its place in the
// tile (1-ulp differences between a tile and a single-pair forward, found at round 4).
// Instead every pair's items are cut at the same local offsets: every offset at which a
// wave boundary can fall for SOME slot, {64k mod PER}.  A group then never straddles a
// wave, and it is the same set of the pair's pixels in every slot, so a pair's result
// depends on its own pixels only.
template <int PER, int NPR>
struct VoteCuts {
    int n = 0;
    int at[64] = {};
    constexpr VoteCuts() {
        for (int off = 1; off < PER && n < 64; ++off) {
            bool cut = false;
            for (int k = 1; 64 * k < NPR * PER; ++k) cut = cut || (64 * k) % PER == off;
            if (cut) at[n++] = off;
        }
    }
};
// the lanes of this wave in item it's vote group (a mask over the wave's 64 lanes)
template <int PER, int NPR>
__device__ __forceinline__ unsigned long long vote_lanes(int it) {
    constexpr VoteCuts<PER, NPR> cuts{};
    const int wb = it & ~63, q = udiv(it, PER), l = it - q * PER;
    int lo = 0, hi = PER;
#pragma unroll
    for (int k = 0; k < cuts.n; ++k) {
        if (cuts.at[k] <= l) lo = cuts.at[k];
        if (cuts.at[k] > l && cuts.at[k] < hi) hi = cuts.at[k];
    }
    int a = q * PER + lo - wb, b = q * PER + hi - wb;
    a = a < 0 ? 0 : a;
    b = b > 64 ? 64 : b;
    const unsigned long long top = b >= 64 ? ~0ull : ((1ull << b) - 1ull);
    return top & ~((1ull << a) - 1ull);
}
#ifndef CGP_NET_RES_UNDEF
#define CGP_NET_RES_UNDEF 1
#endif
// PRE: weight and bias arrive already scaled (a compiled program's records, prog_recs)
template <typename T, bool EX, bool DU, class G, bool PRE = false>
__device__ __forceinline__ void net_conv(T* __restrict__ lds, const cgp_net_op& op,
                                         const NetP<T>& p, const Pairs& pr) {
    constexpr int NP = G::NP;
    const int tid = opaque_tid();
    const PolyTab tab = poly_table();
    // a conv feeding the fp64 closed-form ReLU produces c/4 (exact: w/4, b/4) for relu_q_n
    const T qs = !PRE && kQuarter<T, EX> && op.relu ? T(0.25) : T(1);
    const T w = T(op.weight) * qs, b = T(op.bias) * qs;
    const int arena = NP == 1 ? 0 : p.lds_elems;
    prio_mem<NP, G::HW>();
    const VarSrc<T> vs0 = var_src<T, NP == 1>(op, pr.i, pr.j, G::HOWO);   // NP == 1
    auto vs_of = [&](int q) {
        if constexpr (NP == 1) {
            return vs0;
        } else {
            unsigned iq, jq;
            pair_q<NP>(pr, q, iq, jq);
            return var_src<T, false>(op, iq, jq, G::HOWO);
        }
    };
    const T* __restrict__ src = lds + op.src;
    const int wsi = op.ws_in, wso = op.ws_out;

    if constexpr (G::REDUCE && NP == 1) {
        prio_alu<NP, G::HW>();
        // 1x1 output from a full-plane window: a block reduction — or, after a conv marked
        // CGP_NET_CODE_SUM, the wave partial sums that conv left (the map was never stored)
        const bool from_sum = (op.code & CGP_NET_CODE_FROM_SUM) != 0;
        T* part = from_sum ? static_cast<T*>(pr.red)
                           : lds + p.part;   // off the scratch's zero rows (cgp_net_args.part)
        if (!from_sum) {
            T acc = T(0);
#pragma unroll
            for (int k = 0; k < (G::HW + G::NT - 1) / G::NT; ++k) {
                const int px = tid + k * G::NT;
                if (G::HW % G::NT == 0 || px < G::HW) {
                    const int r = udiv(px, G::W), c = px - r * G::W;
                    acc += src[r * wsi + c];
                }
            }
            acc = wave_sum(acc);
            if ((tid & 63) == 0) part[tid >> 6] = acc;
            lds_barrier();
        }
        if (tid == 0) {
            T tot = part[0];
#pragma unroll
            for (int k = 1; k < G::NT / 64; ++k) tot += part[k];
            T v[1] = {fma_t(w, tot, b)};
            const int at[1] = {0};
            const bool ok[1] = {true};
            T u1[1] = {T(1)}, u2[1] = {T(1)};
            if (vs0.on) {
                u1[0] = vs0.ldx(0);
                u2[0] = vs0.ldy(0);
            }
            net_out<T, EX, DU, 1>(lds, op, v, at, ok, u1, u2, tab);
        }
    } else if constexpr (G::REDUCE) {
        prio_alu<NP, G::HW>();
        // NP pairs: G::NT / NP lanes per pair (within one wave) sum its map, then a
        // segmented butterfly; the group's first lane finishes the pair
        constexpr int TPP = G::NT / NP;
        static_assert(TPP <= 64 && G::NT % NP == 0, "reduce groups must not straddle waves");
        const int q = udiv(tid, TPP), lane = tid - q * TPP;
        const T* srcq = src + q * arena;
        T acc = T(0);
#pragma unroll
        for (int k = 0; k < (G::HW + TPP - 1) / TPP; ++k) {
            const int px = lane + k * TPP;
            if (G::HW % TPP == 0 || px < G::HW) {
                const int r = udiv(px, G::W), c = px - r * G::W;
                acc += srcq[r * wsi + c];
            }
        }
#pragma unroll
        for (int m = TPP / 2; m >= 1; m >>= 1) acc += __shfl_xor(acc, m, 64);
        if (lane == 0) {
            const VarSrc<T> vs = vs_of(q);
            T v[1] = {fma_t(w, acc, b)};
            const int at[1] = {q * arena};
            const bool ok[1] = {true};
            T u1[1] = {T(1)}, u2[1] = {T(1)};
            if (vs.on) {
                u1[0] = vs.ldx(0);
                u2[0] = vs.ldy(0);
            }
            net_out<T, EX, DU, 1>(lds, op, v, at, ok, u1, u2, tab);
        }
    } else if constexpr (G::POINT) {
        prio_alu<NP, G::HW>();
        constexpr int N = NP * G::HOWO;
        constexpr int KP = (N + G::NT - 1) / G::NT;
        T u1[KP], u2[KP], v[KP];
        int at[KP];
        bool ok[KP];
#pragma unroll
        for (int k = 0; k < KP; ++k) {
            const int e = tid + k * G::NT;
            ok[k] = N % G::NT == 0 || e < N;
            const int ec = ok[k] ? e : 0;
            const int q = NP == 1 ? 0 : udiv(ec, G::HOWO), pc = ec - q * G::HOWO;
            const int r = udiv(pc, G::WO), c = pc - r * G::WO;
            const VarSrc<T> vs = vs_of(q);
            at[k] = q * arena + r * wso + c;
            u1[k] = (vs.on && ok[k]) ? vs.ldx((unsigned)pc) : T(1);
            u2[k] = (vs.on && ok[k]) ? vs.ldy((unsigned)pc) : T(1);
            v[k] = fma_t(w, src[q * arena + (r * G::S) * wsi + c * G::S], b);
        }
        net_out<T, EX, DU, KP, NP == 1 ? 1 : 0>(lds, op, v, at, ok, u1, u2, tab);
    } else if constexpr (G::DIRECT) {
        // one pass: item (q, g3, c) sums its WIN3 x TAPS input window straight from the
        // source slot (row sums, then column sums: the separable path's order, so the
        // same bits); rows outside the map read as zero, columns outside are the slot's
        // zero halo
        constexpr int NVT = NP * G::NV;
        T u1[G::KV][G::R3], u2[G::KV][G::R3];
#pragma unroll
        for (int kv = 0; kv < G::KV; ++kv) {
            const int it = tid + kv * G::NT;
            const int itc = (NVT % G::NT == 0 || it < NVT) ? it : 0;
            const int q = NP == 1 ? 0 : udiv(itc, G::NV), l = itc - q * G::NV;
            const int g3 = udiv(l, G::WO), c = l - g3 * G::WO;
            const VarSrc<T> vs = vs_of(q);
#pragma unroll
            for (int k = 0; k < G::R3; ++k) {
                const unsigned px0 = (unsigned)(g3 * G::R3 * G::WO + c);
                u1[kv][k] = vs.on ? vs.ldx(px0, k * G::WO) : T(1);
                u2[kv][k] = vs.on ? vs.ldy(px0, k * G::WO) : T(1);
            }
        }
        // outputs that land on the source (in place, or dst2 on the source) are stored
        // after every item has read its window
        const int s_lo = op.src - wsi, s_hi = op.src + G::H * wsi;
        auto hits = [&](int d) {
            return d >= 0 && d - wso < s_hi && d + G::HO * wso > s_lo;
        };
        const bool hazard = hits(op.dst) || (DU && hits(op.dst2));
        T res[G::KV][G::R3];
#if CGP_NET_RES_UNDEF
        // an idle item's outputs are never stored: defined by an empty asm, not by 7 zero
        // moves per item and op
#pragma unroll
        for (int kv = 0; kv < G::KV; ++kv)
#pragma unroll
            for (int k = 0; k < G::R3; ++k) asm volatile("" : "=v"(res[kv][k]));
#endif
#pragma unroll
        for (int kv = 0; kv < G::KV; ++kv) {
            const int it = tid + kv * G::NT;
            if (NVT % G::NT == 0 || it < NVT) {
                const int q = NP == 1 ? 0 : udiv(it, G::NV), l = it - q * G::NV;
                const int g3 = udiv(l, G::WO), c = l - g3 * G::WO;
                const T* base = src + q * arena + c * G::S + G::OFF;
                const int r0 = g3 * G::R3 * G::S + G::OFF;
                T rs[G::WIN3];
#pragma unroll
                for (int t = 0; t < G::WIN3; ++t) {
                    const bool lo = G::OFF + t < 0, hi = (G::NG3 - 1) * G::R3 * G::S + G::OFF + t >= G::H;
                    const int r = r0 + t;
                    const bool in = (!lo || r >= 0) && (!hi || r < G::H);
                    const T* row = base + (in ? r : 0) * wsi;
                    T a = row[0];
#pragma unroll
                    for (int dx = 1; dx < G::TAPS; ++dx) a += row[dx];
                    rs[t] = in ? a : T(0);
                }
                T o[G::R3];
                win_sums<T, G::TAPS, G::S, G::R3>(rs, o);
#pragma unroll
                for (int k = 0; k < G::R3; ++k) res[kv][k] = fma_t(w, o[k], b);
#pragma unroll
                for (int k = 0; k < G::R3; ++k)
                    asm volatile("" : "+v"(u1[kv][k]), "+v"(u2[kv][k]));
            }
        }
        prio_alu<NP, G::HW>();
        if (hazard) lds_barrier();
#pragma unroll
        for (int kv = 0; kv < G::KV; ++kv) {
            const int it = tid + kv * G::NT;
            if (NVT % G::NT == 0 || it < NVT) {
                const int q = NP == 1 ? 0 : udiv(it, G::NV), l = it - q * G::NV;
                const int g3 = udiv(l, G::WO), c = l - g3 * G::WO;
                int at[G::R3];
                bool ok[G::R3];
#pragma unroll
                for (int k = 0; k < G::R3; ++k) {
                    at[k] = q * arena + (g3 * G::R3 + k) * wso + c;
                    ok[k] = true;
                }
                net_out<T, EX, DU, G::R3, kAdaptOf<NP>>(lds, op, res[kv], at, ok, u1[kv],
                                                        u2[kv], tab,
                                                        NP == 1 ? ~0ull : vote_lanes<G::NV, NP>(it));
            }
        }
    } else {
        T* __restrict__ hs = lds + p.hs;
        constexpr int NHT = NP * G::NH, NVT = NP * G::NV, NZT = NP * G::NZ;
        // variances of this thread's outputs, in flight during the row pass
        T u1[G::KV][G::R3], u2[G::KV][G::R3];
        if (vs0.on) {
#pragma unroll
            for (int kv = 0; kv < G::KV; ++kv) {
                const int it = tid + kv * G::NT;
                const int itc = (NVT % G::NT == 0 || it < NVT) ? it : 0;
                const int q = NP == 1 ? 0 : udiv(itc, G::NV), l = itc - q * G::NV;
                const int g3 = udiv(l, G::WO), c = l - g3 * G::WO;
                const VarSrc<T> vs = vs_of(q);
#pragma unroll
                for (int k = 0; k < G::R3; ++k) {
                    const unsigned px0 = (unsigned)(g3 * G::R3 * G::WO + c);
                    u1[kv][k] = vs.ldx(px0, k * G::WO);
                    u2[kv][k] = vs.ldy(px0, k * G::WO);
                }
            }
        } else {
#pragma unroll
            for (int kv = 0; kv < G::KV; ++kv)
#pragma unroll
                for (int k = 0; k < G::R3; ++k) u1[kv][k] = u2[kv][k] = T(1);
        }
        // row pass: hs[q][c] = Σ_t in[q + OFF][c·S + OFF + t]
#pragma unroll
        for (int kh = 0; kh < G::KH; ++kh) {
            const int it = tid + kh * G::NT;
            if (NHT % G::NT == 0 || it < NHT) {
                const int q = NP == 1 ? 0 : udiv(it, G::NH), l = it - q * G::NH;
                const int qi = udiv(l, G::NG2), g2 = l - qi * G::NG2;
                const T* row = lds + (op.src + q * arena + (G::Q0 + qi + G::OFF) * wsi +
                                      g2 * G::R2 * G::S + G::OFF);
                T win[G::WIN2];
#pragma unroll
                for (int t = 0; t < G::WIN2; ++t) win[t] = row[t];
                T o[G::R2];
                win_sums<T, G::TAPS, G::S, G::R2>(win, o);
                T* h = hs + q * arena + (G::Q0 + qi) * G::WO + g2 * G::R2;
#pragma unroll
                for (int t = 0; t < G::R2; ++t) h[t] = o[t];
            }
        }
        // hs rows outside the input are zero (the scratch is shared by every conv); skipped
        // when the host proved they still are (CGP_NET_CODE_HS_CLEAN)
        if constexpr (G::NZ > 0) {
            if (!(op.code & CGP_NET_CODE_HS_CLEAN)) {
#pragma unroll
                for (int z0 = 0; z0 < NZT; z0 += G::NT) {
                    const int z = z0 + tid;
                    if (NZT % G::NT == 0 || z < NZT) {
                        const int q = NP == 1 ? 0 : udiv(z, G::NZ), zl = z - q * G::NZ;
                        hs[q * arena + (zl < G::Q0 * G::WO ? zl : zl + G::NVR * G::WO)] = T(0);
                    }
                }
            }
        }
        lds_barrier();
        // column pass + output stage (uniform branches outside the per-pixel loops: each
        // stage is one basic block, so the R3 independent ReLUs interleave).  A conv marked
        // CGP_NET_CODE_SUM (one pair) keeps its outputs in registers and leaves only their
        // wave sums for the reduction that follows
        const bool to_sum = NP == 1 && (op.code & CGP_NET_CODE_SUM) != 0;
        T sacc = T(0);
#pragma unroll
        for (int kv = 0; kv < G::KV; ++kv) {
            const int it = tid + kv * G::NT;
            if (NVT % G::NT == 0 || it < NVT) {
                const int q = NP == 1 ? 0 : udiv(it, G::NV), l = it - q * G::NV;
                const int g3 = udiv(l, G::WO), c = l - g3 * G::WO;
                const T* col = lds + (p.hs + q * arena + g3 * G::R3 * G::S * G::WO + c);
                T win[G::WIN3];
#pragma unroll
                for (int t = 0; t < G::WIN3; ++t) win[t] = col[t * G::WO];
                // the variances are first needed here: without this fence the compiler
                // folds u1·u2 (the ReLU's t) into the load block at the op start and
                // waits for the loads there, before the row pass
#pragma unroll
                for (int k = 0; k < G::R3; ++k) asm volatile("" : "+v"(u1[kv][k]), "+v"(u2[kv][k]));
                T o[G::R3], v[G::R3];
                win_sums<T, G::TAPS, G::S, G::R3>(win, o);
                prio_alu<NP, G::HW>();
                int at[G::R3];
                bool ok[G::R3];
#pragma unroll
                for (int k = 0; k < G::R3; ++k) {
                    v[k] = fma_t(w, o[k], b);
                    at[k] = q * arena + (g3 * G::R3 + k) * wso + c;
                    ok[k] = true;
                }
                if (to_sum) {
                    if (op.relu) relu_n<EX, kQuarter<T, EX>, T, G::R3, 1>(v, u1[kv], u2[kv], tab);
#pragma unroll
                    for (int k = 0; k < G::R3; ++k) sacc += v[k];
                } else {
                    net_out<T, EX, DU, G::R3, kAdaptOf<NP>>(lds, op, v, at, ok, u1[kv], u2[kv],
                                                            tab,
                                                            NP == 1 ? ~0ull
                                                                    : vote_lanes<G::NV, NP>(it));
                }
            }
        }
        if constexpr (NP == 1) {
            if (to_sum) {
                sacc = wave_sum(sacc);
                if ((tid & 63) == 0) static_cast<T*>(pr.red)[tid >> 6] = sacc;
            }
        }
    }
}

// ---- elementwise ops: RELU, LINEAR, MOMENTS -------------------------------------------
// One pass: KE pixels per thread at e = base + k·NT + tid over the NP pairs' maps
// (pair q = e / hw; NP > 1 needs the compile-time size W_).
template <typename T, bool EX, bool DU, int KIND, int KE, int W_, int NP>
__device__ __forceinline__ void elem_pass(T* __restrict__ lds, const cgp_net_op& op,
                                          const NetP<T>& p, const Pairs& pr, int tid,
                                          int base, int hw, const PolyTab& tab) {
    static_assert(NP == 1 || W_ > 0, "multi-pair elementwise ops need a compile-time size");
    const int wd = W_ ? W_ : op.w, ws = op.ws_out;
    const int arena = NP == 1 ? 0 : p.lds_elems;
    const FastDiv fw{op.div_m, op.div_s, (unsigned)op.w};
    // RELU reads (var_x, var_y) = variances of src (an elementwise ReLU has no dst2);
    // LINEAR may carry a dst2 ReLU with (var2_x, var2_y)
    auto vs_of = [&](unsigned iq, unsigned jq) {
        return KIND == CGP_NET_RELU
                   ? var_maps<T, NP == 1>(op.var_x, op.var_y, true, iq, jq, hw)
                   : var_src<T, NP == 1>(op, iq, jq, hw);
    };
    const VarSrc<T> vs0 = vs_of(pr.i, pr.j);
    // the pair's images (MOMENTS, one pair per half: i, j uniform) as scalar byte bases;
    // pixel offsets stay 32-bit unsigned, so every load is SGPR base + VGPR offset with no
    // 64-bit VALU address arithmetic (an image is at most C·hw·8 bytes)
    const GP<char> xi = ubase(p.x) + (size_t)pr.i * p.channels * hw * sizeof(T);
    const GP<char> yj = ubase(p.y) + (size_t)pr.j * p.channels * hw * sizeof(T);
    auto img = [](GP<char> b, unsigned e) {
        return *(GP<T>)(b + (size_t)(e * (unsigned)sizeof(T)));
    };
    const int n = NP * hw;
    // waves with no pixel in this pass skip the ReLUs (uniform per wave)
    const bool live = base + (tid & ~63) < n;
    T a[KE], u1[KE], u2[KE];
    int at[KE];
    bool ok[KE];
#pragma unroll
    for (int k = 0; k < KE; ++k) {
        const int e = base + k * kNT + tid;
        ok[k] = e < n;
        const int ec = ok[k] ? e : 0;
        const int q = NP == 1 ? 0 : ec / hw, pc = ec - q * hw;
        const int r = W_ ? udiv(pc, W_) : (int)fdiv((unsigned)pc, fw);
        at[k] = q * arena + r * ws + (pc - r * wd);
        VarSrc<T> vs = vs0;
        if constexpr (NP > 1) {
            unsigned iq, jq;
            pair_q<NP>(pr, q, iq, jq);
            vs = vs_of(iq, jq);
        }
        u1[k] = (vs.on && ok[k]) ? vs.ldx((unsigned)pc) : T(1);
        u2[k] = (vs.on && ok[k]) ? vs.ldy((unsigned)pc) : T(1);
        if constexpr (KIND == CGP_NET_RELU) {
            a[k] = lds[op.src + at[k]];
        } else if constexpr (KIND == CGP_NET_MOMENTS) {
            static_assert(NP == 1, "moments run one pair per workgroup (half)");
            T acc = img(xi, (unsigned)pc) * img(yj, (unsigned)pc);
            for (int ch = 1; ch < p.channels; ++ch) {
                const unsigned e = (unsigned)(ch * hw + pc);
                acc += img(xi, e) * img(yj, e);
            }
            a[k] = acc;
        } else {
            a[k] = T(op.weight) * lds[op.src + at[k]] + T(op.bias) * lds[op.add + at[k]];
        }
    }
    if constexpr (KIND == CGP_NET_MOMENTS) {
        // the channel mean (x / 1 == x: a uniform branch, so one-channel inputs run no
        // division at all)
        if (p.channels != 1) {
#pragma unroll
            for (int k = 0; k < KE; ++k) a[k] = a[k] / T(p.channels);
        }
    }
    if constexpr (KIND == CGP_NET_RELU) {
        if (live) relu_n<EX, false, T, KE, NP == 1 ? 1 : 0>(a, u1, u2, tab);
        if (op.add >= 0) {
#pragma unroll
            for (int k = 0; k < KE; ++k)
                if (ok[k]) a[k] += lds[op.add + at[k]];
        }
    }
#pragma unroll
    for (int k = 0; k < KE; ++k)
        if (ok[k]) lds[op.dst + at[k]] = a[k];
    if constexpr (KIND == CGP_NET_LINEAR && DU) {
        if (op.dst2 >= 0) {
            if (live) relu_n<EX, false, T, KE, NP == 1 ? 1 : 0>(a, u1, u2, tab);
#pragma unroll
            for (int k = 0; k < KE; ++k)
                if (ok[k]) lds[op.dst2 + at[k]] = a[k];
        }
    }
}

// compile-time map size: passes of at most kEw pixels per thread, the last one sized to
// what is left (28x28: 4 + 3)
template <typename T, bool EX, bool DU, int KIND, int H_, int W_, int NP, int PI>
__device__ __forceinline__ void elem_passes(T* __restrict__ lds, const cgp_net_op& op,
                                            const NetP<T>& p, const Pairs& pr, int tid,
                                            const PolyTab& tab) {
    constexpr int KF = (NP * H_ * W_ + kNT - 1) / kNT;
    if constexpr (PI * kEw < KF) {
        constexpr int KE = KF - PI * kEw < kEw ? KF - PI * kEw : kEw;
        elem_pass<T, EX, DU, KIND, KE, W_, NP>(lds, op, p, pr, tid, PI * kEw * kNT, H_ * W_,
                                               tab);
        elem_passes<T, EX, DU, KIND, H_, W_, NP, PI + 1>(lds, op, p, pr, tid, tab);
    }
}

// H_ = W_ = 0: runtime map size (generic path, one pair per workgroup).
template <typename T, bool EX, bool DU, int KIND, int H_, int W_, int NP>
__device__ __forceinline__ void net_elem(T* __restrict__ lds, const cgp_net_op& op,
                                         const NetP<T>& p, const Pairs& pr) {
    const int tid = opaque_tid();
    const PolyTab tab = poly_table();
    if constexpr (H_ == 0) {
        const int hw = op.h * op.w;
        for (int base = 0; base < hw; base += kEw * kNT)
            elem_pass<T, EX, DU, KIND, kEw, 0, 1>(lds, op, p, pr, tid, base, hw, tab);
    } else {
        elem_passes<T, EX, DU, KIND, H_, W_, NP, 0>(lds, op, p, pr, tid, tab);
    }
}

// Stage boundary (CGP_NET_LOAD / CGP_NET_STORE): the map of each of the NP pairs moves
// between its slot and the unit's state record, state[(u - ubeg) · code + add + pixel].
template <typename T, int KIND, int NP>
__device__ __forceinline__ void net_move(T* __restrict__ lds, const cgp_net_op& op,
                                         const NetP<T>& p, const Pairs& pr) {
    const int tid = opaque_tid();
    const int hw = op.h * op.w, n = NP * hw;
    const int arena = NP == 1 ? 0 : p.lds_elems;
    T* state = const_cast<T*>(static_cast<const T*>(op.var_x));
    for (int e = tid; e < n; e += kNT) {
        const int q = NP == 1 ? 0 : e / hw, l = e - q * hw;
        const int r = l / op.w, c = l - r * op.w;
        // the state buffer holds the units of this launch, [ubeg, uend)
        const size_t g = (size_t)(pr.u0 + q - p.ubeg) * (size_t)op.code + (size_t)op.add +
                         (size_t)l;
        if constexpr (KIND == CGP_NET_LOAD)
            lds[op.dst + q * arena + r * op.ws_out + c] = state[g];
        else
            state[g] = lds[op.src + q * arena + r * op.ws_in + c];
    }
}

// The same move for a compiled program (geometry, slot and pitches compile-time): pass k
// covers elements e = k·kNT + tid of the NP pairs' H×W maps, all passes unrolled.  The
// launch's state base (u0 − ubeg)·code + add is scalar (u0 is uniform), so an element's
// global address is that SGPR base plus a 32-bit lane offset q·code + l, and its LDS cell
// q·arena + r·ws + c comes from compile-time divisions: about 12 VALU per element where
// the generic loop above spent about 25 (64-bit address math, signed divisions by runtime
// sizes; ISA count, tools/isa_attrib.py).  CGP_NET_MOVE_C=0 keeps the generic loop.
#ifndef CGP_NET_MOVE_C
#define CGP_NET_MOVE_C 1
#endif
template <typename T, int KIND, int NP, int H_, int W_, int SLOT, int WS>
__device__ __forceinline__ void net_move_c(T* __restrict__ lds, const cgp_net_op& op,
                                           const NetP<T>& p, const Pairs& pr) {
    const int tid = opaque_tid();
    constexpr int HW = H_ * W_, N = NP * HW, KP = (N + kNT - 1) / kNT;
    const int arena = NP == 1 ? 0 : p.lds_elems;
    const unsigned long long u0 =
        ((unsigned long long)__builtin_amdgcn_readfirstlane((unsigned)((unsigned long long)pr.u0 >> 32)) << 32) |
        __builtin_amdgcn_readfirstlane((unsigned)pr.u0);
    const unsigned code = (unsigned)__builtin_amdgcn_readfirstlane(op.code);
    const GP<char> base = ubase(op.var_x) +
                          ((size_t)(u0 - (unsigned long long)p.ubeg) * code + (size_t)op.add) *
                              sizeof(T);
#pragma unroll
    for (int k = 0; k < KP; ++k) {
        const int e = k * kNT + tid;
        if (N % kNT == 0 || e < N) {
            const unsigned q = NP == 1 ? 0u : (unsigned)udiv(e, HW);
            const unsigned l = (unsigned)e - q * (unsigned)HW;
            const unsigned r = (unsigned)udiv((int)l, W_), c = l - r * (unsigned)W_;
            T* cell = lds + (SLOT + (int)q * arena + (int)(r * (unsigned)WS + c));
            typedef __attribute__((address_space(1))) T* GW;   // the state record, writable
            GW g = (GW)(base + (size_t)((q * code + l) * (unsigned)sizeof(T)));
            if constexpr (KIND == CGP_NET_LOAD)
                *cell = *g;
            else
                *g = *cell;
        }
    }
}

// Zero the halo cells of the slot whose pixel (0, 0) is at `origin` (code = (HL << 8) |
// gap, see cgp_net_op.zero_halo): HL cells before it and `gap` after each of the h rows.
// Disjoint from every data cell, so it needs no barrier against the op's own writes.
template <typename T, int NT>
__device__ __forceinline__ void zero_halos(T* lds, int origin, int code, int h, int w, int ws,
                                           int tid) {
    if (!code) return;
    const int hl = code >> 8, gap = code & 0xff;
    for (int e = tid; e < hl + h * gap; e += NT) {
        int cell;
        if (e < hl) {
            cell = origin - hl + e;
        } else {
            const int r = (e - hl) / gap;
            cell = origin + r * ws + w + (e - hl - r * gap);
        }
        lds[cell] = T(0);
    }
}

// pair walk: supertile s (kST x kST pairs) -> (bi, bj); same tiles enumerate the upper
// triangle (bi <= bj) row-major
__device__ __forceinline__ void tri_decode(unsigned s, unsigned nb, unsigned& bi,
                                           unsigned& bj) {
    const double a = 2.0 * nb + 1.0;
    long long r = (long long)((a - sqrt(a * a - 8.0 * (double)s)) * 0.5);
    auto off = [nb](long long q) { return q * (long long)nb - q * (q - 1) / 2; };
    if (r < 0) r = 0;
    while (r > 0 && off(r) > (long long)s) --r;
    while (off(r + 1) <= (long long)s) ++r;
    bi = (unsigned)r;
    bj = (unsigned)(r + ((long long)s - off(r)));
}

// tile unit u (supertile, pair within it) -> (i, j); false if outside the tile
template <typename T>
__device__ __forceinline__ bool unit_pair(const NetP<T>& p, long long u, unsigned& i,
                                          unsigned& j) {
    const unsigned s = (unsigned)(u >> (2 * kSTL)), q = (unsigned)u & (kST * kST - 1u);
    unsigned bi, bj;
    if (p.same) {
        tri_decode(s, p.nbi, bi, bj);
    } else {
        bi = s / p.nbj;
        bj = s - bi * p.nbj;
    }
    i = bi * kST + (q >> kSTL);
    j = bj * kST + (q & (kST - 1u));
    return u < p.units && i < p.n1 && j < p.n2;
}

constexpr int geo_index(int h, int w, int ho, int wo, int k, int s, int o) {
    for (int n = 0; n < kNumGeo; ++n) {
        const GeoRow& g = kGeoTable[n];
        if (g.h == h && g.w == w && g.ho == ho && g.wo == wo && g.taps == k && g.s == s &&
            g.off == o)
            return n;
    }
    return -1;
}

// a geometry / map size is instantiated for NP pairs when the NP maps fit the passes
// (NP·h·w <= 1024: 4 pairs at <= 16x16, 16 at <= 8x8); the host stages networks to match
#define CGP_NET_FITS(h, w) (NP == 1 || (h) * (w) * NP <= 1024)

#define CGP_NET_CASE(h, w, ho, wo, k, s, o)                                          \
    case geo_index(h, w, ho, wo, k, s, o):                                           \
        if constexpr (CGP_NET_FITS(h, w))                                            \
            net_conv<T, EX, DU, NG<h, w, ho, wo, k, s, o, NP>>(lds, op, p, pr);      \
        break;

#define CGP_NET_RES_CASE(h, w)                                                        \
    case res_index(h, w):                                                             \
        if constexpr (CGP_NET_FITS(h, w)) net_elem<T, EX, DU, KIND, h, w, NP>(lds, op, p, pr); \
        break;

// only the ReLU is worth a per-size instantiation (MOMENTS runs once per pair, LINEAR
// only for Mixture / multi-term Sum); fewer cases also keep the SGPR budget.  Multi-pair
// stages run compile-time sizes only (the host keeps moments and other sizes at NP = 1).
template <typename T, bool EX, bool DU, int KIND, int NP>
__device__ __forceinline__ void net_elem_dispatch(T* __restrict__ lds, const cgp_net_op& op,
                                                  const NetP<T>& p, const Pairs& pr) {
    if constexpr (KIND == CGP_NET_RELU || (KIND == CGP_NET_LINEAR && NP > 1)) {
        switch (op.code) {
            CGP_NET_RESOLUTIONS(CGP_NET_RES_CASE)
        default:
            if constexpr (NP == 1) net_elem<T, EX, DU, KIND, 0, 0, 1>(lds, op, p, pr);
            break;
        }
    } else if constexpr (NP == 1) {
        net_elem<T, EX, DU, KIND, 0, 0, 1>(lds, op, p, pr);
    }
}

template <typename T, bool EX, bool DU, int NP>
__device__ __forceinline__ void net_op(T* __restrict__ lds, const cgp_net_op& op,
                                       const NetP<T>& p, const Pairs& pr, int tid) {
    if (op.zero_halo) {
#pragma unroll
        for (int q = 0; q < NP; ++q) {
            const int qa = NP == 1 ? 0 : q * p.lds_elems;
            zero_halos<T, kNT>(lds + qa, op.dst, op.zero_halo & 0xffff, op.h, op.w,
                                     op.ws_out, tid);
            zero_halos<T, kNT>(lds + qa, op.dst2, (unsigned)op.zero_halo >> 16, op.h, op.w,
                       op.ws_out, tid);
        }
    }
    switch (op.kind) {
    case CGP_NET_CONV:
        switch (op.code & CGP_NET_CODE_GEOMETRY) {
            CGP_NET_GEOMETRIES(CGP_NET_CASE)
        default:
            break;
        }
        break;
    case CGP_NET_RELU:
        net_elem_dispatch<T, EX, DU, CGP_NET_RELU, NP>(lds, op, p, pr);
        break;
    case CGP_NET_MOMENTS:
        net_elem_dispatch<T, EX, DU, CGP_NET_MOMENTS, NP>(lds, op, p, pr);
        break;
    case CGP_NET_LINEAR:
        net_elem_dispatch<T, EX, DU, CGP_NET_LINEAR, NP>(lds, op, p, pr);
        break;
    case CGP_NET_LOAD:
        net_move<T, CGP_NET_LOAD, NP>(lds, op, p, pr);
        break;
    case CGP_NET_STORE:
        net_move<T, CGP_NET_STORE, NP>(lds, op, p, pr);
        break;
    default:
        break;
    }
}

// ---- compiled programs ------------------------------------------------------------
// The lowered op lists of the reference configs (tools/gen_net_programs.py ->
// net_programs.h).  A program kernel runs its ops as straight-line code: kind, geometry,
// LDS offsets and strides are immediates, only weight / bias / variance pointers are read
// from the launch's op records.  The host picks it with cgp_net_program().
// compiled programs take their convs' ReLU scaling (w/4, b/4) from prog_recs, applied once
// per workgroup (two VALU ops less per conv and pair); CGP_NET_PRESCALE=0: per op as before
#ifndef CGP_NET_PRESCALE
#define CGP_NET_PRESCALE 1
#endif
constexpr bool kNetPrescale = CGP_NET_PRESCALE != 0;
struct ProgOp {
    int kind, code, src, dst, add, ws_in, ws_out, relu, h, w, dst2, zero_halo;
};
struct ProgInfo {
    int first, nops, pairs, dual, lds_elems, sizes;
};
#include "net_programs.h"
constexpr int kNumProgs = sizeof(kProgs) / sizeof(kProgs[0]);

// The runtime fields of a compiled program's op records (weight, bias, variance / state
// pointers), copied into LDS once per workgroup: an op then starts with an LDS read of its
// pointers instead of a dependent global load of its record (round 4, one B = 1024 Kxz tile,
// two rounds in one call, profiles/r4/ab_r4d_rec_pre.log: ConvNet +1.2%, mnist_as_tf +1.8%,
// cifar10 +2.7%).  Issuing op k + 1's variance loads at the end of op k instead measured
// -2.8% on ConvNet and neutral elsewhere (same log): the wave priority already overlaps them.
struct ProgRec {
    double weight, bias;
    const void* var_x;
    const void* var_y;
    const void* var2_x;
    const void* var2_y;
};
template <int PID>
constexpr int kRecsOf = PID >= 0 ? kProgs[PID < 0 ? 0 : PID].nops : 1;

// op K of program PID as a record: compile-time fields from the program, runtime ones
// (weight, bias, variance / state pointers) from the launch's op records
template <int PID, int K>
__device__ __forceinline__ cgp_net_op prog_op(const ProgRec* recs) {
    constexpr ProgOp o = kProgOps[kProgs[PID].first + K];
    const ProgRec& rt = recs[K];
    cgp_net_op op;
    op.kind = o.kind;
    op.code = o.code;
    op.src = o.src;
    op.dst = o.dst;
    op.add = o.add;
    op.ws_in = o.ws_in;
    op.ws_out = o.ws_out;
    op.relu = o.relu;
    op.h = o.h;
    op.w = o.w;
    op.div_m = 0;
    op.div_s = 0;
    op.dst2 = o.dst2;
    op.zero_halo = o.zero_halo;
    op.weight = rt.weight;
    op.bias = rt.bias;
    op.var_x = rt.var_x;
    op.var_y = rt.var_y;
    op.var2_x = rt.var2_x;
    op.var2_y = rt.var2_y;
    return op;
}
// the conv geometry of a program op
template <int PID, int K, int NP>
struct ProgGeo {
    static constexpr ProgOp o = kProgOps[kProgs[PID].first + K];
    static constexpr GeoRow g = kGeoTable[o.code & CGP_NET_CODE_GEOMETRY];
    using G = NG<g.h, g.w, g.ho, g.wo, g.taps, g.s, g.off, NP>;
};
template <typename T, bool DU, int NP, int PID, int K>
__device__ __forceinline__ void prog_ops(T* __restrict__ lds, const NetP<T>& p, const Pairs& pr,
                                         int tid, const ProgRec* recs) {
    constexpr ProgInfo I = kProgs[PID];
    if constexpr (K < I.nops) {
        constexpr ProgOp o = kProgOps[I.first + K];
        const cgp_net_op op = prog_op<PID, K>(recs);
        if constexpr (o.zero_halo != 0) {
#pragma unroll
            for (int q = 0; q < NP; ++q) {
                const int qa = q * I.lds_elems;
                zero_halos<T, kNT>(lds + qa, o.dst, o.zero_halo & 0xffff, o.h, o.w,
                                         o.ws_out, tid);
                zero_halos<T, kNT>(lds + qa, o.dst2, (unsigned)o.zero_halo >> 16, o.h, o.w,
                                         o.ws_out,
                           tid);
            }
        }
        if constexpr (o.kind == CGP_NET_CONV) {
            net_conv<T, false, DU, typename ProgGeo<PID, K, NP>::G, kNetPrescale>(lds, op, p,
                                                                                 pr);
        } else if constexpr (o.kind == CGP_NET_RELU || o.kind == CGP_NET_LINEAR ||
                             o.kind == CGP_NET_MOMENTS) {
            net_elem<T, false, DU, o.kind, o.h, o.w, NP>(lds, op, p, pr);
        } else if constexpr (o.kind == CGP_NET_LOAD || o.kind == CGP_NET_STORE) {
            if constexpr (CGP_NET_MOVE_C)
                net_move_c<T, o.kind, NP, o.h, o.w, o.kind == CGP_NET_LOAD ? o.dst : o.src,
                           o.kind == CGP_NET_LOAD ? o.ws_out : o.ws_in>(lds, op, p, pr);
            else
                net_move<T, o.kind, NP>(lds, op, p, pr);
        }
        lds_barrier();
        prog_ops<T, DU, NP, PID, K + 1>(lds, p, pr, tid, recs);
    }
}

// the compiled program whose op list equals ops[0, nops) field by field (host memory), +1;
// 0 if none
int prog_match(const cgp_net_op* ops, int nops, int pairs, int dual, int lds_elems,
               int itemsize) {
    for (int k = 0; k < kNumProgs; ++k) {
        const ProgInfo& I = kProgs[k];
        if (I.nops != nops || I.pairs != pairs || I.dual != dual || I.lds_elems != lds_elems ||
            !(I.sizes & itemsize))
            continue;
        bool eq = true;
        for (int n = 0; n < nops && eq; ++n) {
            const ProgOp& o = kProgOps[I.first + n];
            const cgp_net_op& r = ops[n];
            eq = o.kind == r.kind && o.code == r.code && o.src == r.src && o.dst == r.dst &&
                 o.add == r.add && o.ws_in == r.ws_in && o.ws_out == r.ws_out &&
                 o.relu == r.relu && o.h == r.h && o.w == r.w && o.dst2 == r.dst2 &&
                 o.zero_halo == r.zero_halo;
        }
        if (eq) return k + 1;
    }
    return 0;
}

// WPE: waves per SIMD the register allocation targets (amdgpu_waves_per_eu).  LDS caps
// the resident workgroups per CU (two waves each) at 160 KB / footprint, so allocating
// registers for more waves than that only forces spills; net_launch picks WPE from the
// LDS footprint (net_wpe).  NP: pairs per workgroup (1; 2 on four waves, sharing image i;
// 4 / 16 for small-map stages).
// PID >= 0: compiled program PID instead of the op-record interpreter.
template <typename T, bool EX, bool DU, int WPE, int NP, int PID = -1>
__global__ __launch_bounds__(kNTof<NP>) __attribute__((amdgpu_waves_per_eu(WPE))) void net_kernel(const NetP<T> p) {
    extern __shared__ __align__(16) unsigned char smem_raw[];
    __shared__ unsigned pair_tab[2 * kMaxNP];
    __shared__ T red_part[kUnitsOf<NP> * (kNT / 64)];   // CGP_NET_CODE_SUM partials
    T* lds = reinterpret_cast<T*>(smem_raw);
    const int tid = threadIdx.x;
    constexpr int UN = kUnitsOf<NP>;
    for (int e = tid; e < UN * p.lds_elems; e += kNTof<NP>) lds[e] = T(0);   // halos stay zero
    // a FROM_SUM reduction reads these: zeroed, so an op list that breaks the SUM / FROM_SUM
    // contract (cgp_net_validate) reads zeros, never another launch's LDS
    if (tid < UN * (kNT / 64)) red_part[tid] = T(0);
    __shared__ ProgRec prog_recs[kRecsOf<PID>];
    __shared__ long long next_u[2];
    static_assert(sizeof(pair_tab) + sizeof(red_part) + sizeof(prog_recs) + sizeof(next_u) <=
                      kStaticLds,
                  "static LDS beyond the reserve the host checks count (kStaticLds)");
    if constexpr (PID >= 0) {
        for (int k = tid; k < kRecsOf<PID>; k += kNTof<NP>) {
            const cgp_net_op& r = p.ops[k];
            // a conv feeding the fp64 closed-form ReLU runs on w/4, b/4 (net_conv): scaled
            // here once per workgroup (exact) instead of per op and pair
            const ProgOp& o = kProgOps[kProgs[PID < 0 ? 0 : PID].first + k];
            const double qs =
                kNetPrescale && kQuarter<T, false> && o.kind == CGP_NET_CONV && o.relu ? 0.25 : 1.0;
            prog_recs[k] = ProgRec{r.weight * qs, r.bias * qs, r.var_x, r.var_y, r.var2_x,
                                   r.var2_y};
        }
    }
    lds_barrier();
    // XCD-contiguous work ranges: workgroup b runs on XCD b % 8, so each XCD walks one
    // contiguous run of supertiles and its L2 holds the images/variances they share.
    // Ranges and groups are whole multiples of NP units.
    const unsigned xcd = blockIdx.x % 8;
    const long long span = p.uend - p.ubeg;
    const long long per = ((span + 7) / 8 + UN - 1) / UN * UN;
    const long long beg = p.ubeg + (long long)xcd * per;
    const long long end = beg + per < p.uend ? beg + per : p.uend;
    // the XCD's workgroups take its units in order from one counter, so the pairs in
    // flight on an XCD stay one contiguous window (a few supertiles) whose images and
    // variance maps its L2 holds; a static stride lets workgroups drift apart and the
    // window (and L2 misses) grow.  The next group's index is fetched one pair ahead.
    // two slots used alternately (next_u): a slot is rewritten two advances later, after
    // every thread has passed the barrier of the advance in between, so one barrier suffices
    int adv = 0;
    unsigned long long* ctr = p.work + xcd;
    unsigned long long grab = 0;   // thread 0: the counter value fetched one pair ahead
    if (tid == 0) grab = atomicAdd(ctr, 1ull);
    auto advance = [&]() {
        if (tid == 0) next_u[adv] = beg + (long long)grab * UN;
        lds_barrier();
        const long long v = next_u[adv];
        adv ^= 1;
        return v;
    };
    for (long long u = advance(); u < end; u = advance()) {
        if (tid == 0) grab = atomicAdd(ctr, 1ull);
        Pairs pr;
        pr.tab = pair_tab;
        pr.u0 = u;
        pr.red = red_part;
        if constexpr (NP == 2) {
            // one-pair slices sharing the workgroup's barriers: waves 2q, 2q + 1 run unit
            // u + q (the next j of the same image i), each on its own arena.  The pair is
            // uniform per wave, so each slice runs the one-pair code (scalar variance-map
            // bases)
            // every wave decodes the group's units (scalar); the group is skipped only when
            // none of them is evaluated, so all waves agree at every barrier
            const int q = __builtin_amdgcn_readfirstlane(tid >> 7);
            unsigned iq = 0, jq = 0;
            bool vq = false, wq = false, any = false;
#pragma unroll
            for (int s = 0; s < UN; ++s) {
                unsigned is = 0, js = 0;
                const bool vs = u + s < end && unit_pair(p, u + s, is, js);
                const bool ws = vs && !(p.same && js <= is);
                any |= ws;
                if (s == q) {
                    iq = is;
                    jq = js;
                    vq = vs;
                    wq = ws;
                }
            }
            if (!any) {   // below the diagonal of a same tile (or outside): K[i, i] only
                if (p.final_stage && p.same && (tid & (kNT - 1)) == 0 && vq && jq == iq)
                    p.out[(long long)iq * p.ldo + iq] = p.kdiag[iq];
                continue;
            }
            Pairs ph;
            ph.tab = pair_tab;
            ph.u0 = u + q;
            ph.red = red_part + q * (kNT / 64);
            // a slice without a pair computes on clamped indices and stores nothing
            ph.i = __builtin_amdgcn_readfirstlane(vq ? iq : 0u);
            ph.j = __builtin_amdgcn_readfirstlane(vq ? jq : 0u);
            T* lh = lds + q * p.lds_elems;
            const int ht = tid & (kNT - 1);
            if constexpr (PID < 0) {
                for (int k = 0; k < p.nops; ++k) {
                    const cgp_net_op op = load_op(ops_c(p.ops) + k);
                    net_op<T, EX, DU, 1>(lh, op, p, ph, ht);
                    lds_barrier();
                }
            } else {
                prog_ops<T, DU, 1, PID, 0>(lh, p, ph, ht, prog_recs);
            }
            if (p.final_stage && ht == 0 && vq) {
                if (wq) {
                    const T v = lh[p.final_slot];
                    p.out[(long long)ph.i * p.ldo + ph.j] = v;
                    if (p.same) p.out[(long long)ph.j * p.ldo + ph.i] = v;
                } else if (ph.j == ph.i) {
                    p.out[(long long)ph.i * p.ldo + ph.i] = p.kdiag[ph.i];
                }
            }
        } else {
            if constexpr (NP == 1) {
                if (!unit_pair(p, u, pr.i, pr.j)) continue;
                pr.i = __builtin_amdgcn_readfirstlane(pr.i);   // uniform: scalar map offsets
                pr.j = __builtin_amdgcn_readfirstlane(pr.j);
                if (p.same && pr.j <= pr.i) {
                    if (p.final_stage && pr.j == pr.i && tid == 0)
                        p.out[(long long)pr.i * p.ldo + pr.i] = p.kdiag[pr.i];
                    continue;
                }
            } else {
                // the group's pair table; pairs outside the tile are computed on clamped
                // indices and never stored
                if (tid < NP) {
                    unsigned iq = 0, jq = 0;
                    unit_pair(p, u + tid, iq, jq);
                    pair_tab[tid] = iq < p.n1 ? iq : p.n1 - 1;
                    pair_tab[kMaxNP + tid] = jq < p.n2 ? jq : p.n2 - 1;
                }
                pr.i = pr.j = 0;
                lds_barrier();
            }
            if constexpr (PID < 0) {
                for (int k = 0; k < p.nops; ++k) {
                    const cgp_net_op op = load_op(ops_c(p.ops) + k);
                    net_op<T, EX, DU, NP>(lds, op, p, pr, tid);
                    lds_barrier();
                }
            } else {
                prog_ops<T, DU, NP, PID, 0>(lds, p, pr, tid, prog_recs);
            }
            if (p.final_stage) {
                if constexpr (NP == 1) {
                    if (tid == 0) {
                        const T v = lds[p.final_slot];
                        p.out[(long long)pr.i * p.ldo + pr.j] = v;
                        if (p.same) p.out[(long long)pr.j * p.ldo + pr.i] = v;
                    }
                } else if (tid < NP) {
                    unsigned iq, jq;
                    if (u + tid < end && unit_pair(p, u + tid, iq, jq)) {
                        if (!p.same || jq > iq) {
                            const T v = lds[tid * p.lds_elems + p.final_slot];
                            p.out[(long long)iq * p.ldo + jq] = v;
                            if (p.same) p.out[(long long)jq * p.ldo + iq] = v;
                        } else if (jq == iq) {
                            p.out[(long long)iq * p.ldo + iq] = p.kdiag[iq];
                        }
                    }
                }
            }
        }
        lds_barrier();
    }
}

// waves per SIMD the LDS footprint of a workgroup allows (`waves` waves per workgroup,
// 4 SIMDs per CU), clamped to the instantiated register targets 3..5
constexpr int net_wpe(long long lds_bytes, int cap = 5, int waves = kNT / 64) {
    const long long wg = (160LL * 1024) / (lds_bytes + kStaticLds);
    const long long w = wg * waves / 4;
    return w < 3 ? 3 : (w > cap ? cap : (int)w);
}
// register target cap of the fp64 compiled programs (6 waves per SIMD: -1…-2% on the
// ResNets; the multi-pair stages at 4: slower than their 13 spilled VGPRs at 5,
// profiles/r3/ab_r3r_mp_wpe.log); the fp32 programs keep the plain 4 / 5 targets (from
// their LDS capped at 6 / 8: within ±1% except Residual +5%)
constexpr int kProgWpeMax = 5;

// the instantiation for (EX, DU, pairs, LDS footprint of the workgroup): the fp64 closed
// form — the production path — has a register target per occupancy level; fp32 one per
// (DU, pairs); the exact ReLU runs one pair per workgroup
template <typename T, int NP>
const void* net_fn_np(bool du, long long lds_bytes) {
    switch (net_wpe(lds_bytes, 5, kNTof<NP> / 64)) {
    case 3: return du ? (const void*)net_kernel<T, false, true, 3, NP>
                      : (const void*)net_kernel<T, false, false, 3, NP>;
    case 4: return du ? (const void*)net_kernel<T, false, true, 4, NP>
                      : (const void*)net_kernel<T, false, false, 4, NP>;
    default:   // the interpreter's dual-output instantiation spills at 5 waves: 4
        return du ? (const void*)net_kernel<T, false, true, 4, NP>
                  : (const void*)net_kernel<T, false, false, 5, NP>;
    }
}
template <typename T>
const void* net_fn(bool ex, bool du, int np, long long lds_bytes) {
    if (ex) {
        if (np != 1) return nullptr;
        return du ? (const void*)net_kernel<T, true, true, 3, 1>
                  : (const void*)net_kernel<T, true, false, 3, 1>;
    }
    if constexpr (sizeof(T) == 8) {
        switch (np) {
        case 1: return net_fn_np<T, 1>(du, lds_bytes);
        case 2: return net_fn_np<T, 2>(du, lds_bytes);
        case 4: return net_fn_np<T, 4>(du, lds_bytes);
        case 16: return net_fn_np<T, 16>(du, lds_bytes);
        default: return nullptr;
        }
    }
    // fp32: one register target per (DU, pairs)
    switch (np) {
    case 1: return du ? (const void*)net_kernel<T, false, true, 4, 1>
                      : (const void*)net_kernel<T, false, false, 5, 1>;
    case 2: return du ? (const void*)net_kernel<T, false, true, 4, 2>
                      : (const void*)net_kernel<T, false, false, 5, 2>;
    case 4: return du ? (const void*)net_kernel<T, false, true, 4, 4>
                      : (const void*)net_kernel<T, false, false, 5, 4>;
    case 16: return du ? (const void*)net_kernel<T, false, true, 4, 16>
                       : (const void*)net_kernel<T, false, false, 5, 16>;
    default: return nullptr;
    }
}

// program kernels: fp64 register target from the program's LDS footprint, fp32 as net_fn
template <typename T, int PID>
const void* prog_fn_one() {
    constexpr ProgInfo I = kProgs[PID];
    if constexpr ((I.sizes & (int)sizeof(T)) == 0) {
        return nullptr;
    } else {
        constexpr long long bytes =
            (long long)I.lds_elems * (long long)sizeof(T) * kUnitsOf<I.pairs>;
        constexpr int wpe = sizeof(T) == 8 ? net_wpe(bytes, kProgWpeMax, kNTof<I.pairs> / 64)
                                           : (I.dual ? 4 : 5);
        return (const void*)net_kernel<T, false, I.dual != 0, wpe, I.pairs, PID>;
    }
}
template <typename T>
const void* prog_fn(int pid) {
    switch (pid) {
#define CGP_PROG_CASE(k) \
    case k: return prog_fn_one<T, k>();
        CGP_NET_PROGRAMS(CGP_PROG_CASE)
#undef CGP_PROG_CASE
    default: return nullptr;
    }
}

// threads of a workgroup of np pairs (kNTof at run time)
int net_threads(int np) { return np == 2 ? kNTof<2> : kNT; }
// pair units (arenas) a workgroup of np pairs holds
int net_units(int np) { return np == 2 ? kUnitsOf<2> : np; }

int net_occupancy(const void* fn, int lds_bytes, int threads) {
    if (lds_bytes > 64 * 1024 &&
        hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, lds_bytes) !=
            hipSuccess) {
        (void)hipGetLastError();
        return 0;
    }
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, fn, threads, lds_bytes) != hipSuccess) {
        (void)hipGetLastError();
        return 0;
    }
    return n;
}

template <typename T>
int net_occupancy_for(int lds_bytes, int flags, int np) {
    const void* fn = net_fn<T>(flags & CGP_FLAG_EXACT_RELU, flags & CGP_FLAG_NET_DUAL, np,
                               (long long)lds_bytes * net_units(np));
    return fn ? net_occupancy(fn, lds_bytes * net_units(np), net_threads(np)) : 0;
}

// Per-XCD unit counters for a launch: 8 × u64 slots of a 64-slot ring owned by the launch
// stream (one ring per (device, stream), allocated on the device that owns the stream),
// zeroed on that stream.  A slot is reused only by a later launch on the same stream, i.e.
// after this one has drained; launches on other streams never see it.  A ring lives as
// long as the process (a stream destroyed and re-created at the same address reuses its
// ring, which is safe: the old stream's launches have drained by then).  (Per-launch
// hipMallocAsync/hipFreeAsync was measured 5% slower on mnist_as_tf: the pool operations
// open gaps between back-to-back kernels.)
unsigned long long* work_counters(hipStream_t s) {
    constexpr int kSlots = 64;
    struct Ring {
        unsigned long long* buf = nullptr;
        unsigned next = 0;
    };
    static std::mutex mu;
    static std::map<std::pair<int, hipStream_t>, Ring> rings;
    int dev = 0;
    if (stream_device(s, &dev) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    unsigned long long* slot = nullptr;
    {
        std::lock_guard<std::mutex> lock(mu);
        Ring& r = rings[{dev, s}];
        if (!r.buf) {
            int cur = 0;
            hipError_t e = hipGetDevice(&cur);
            if (e == hipSuccess && cur != dev) e = hipSetDevice(dev);
            if (e == hipSuccess)
                e = hipMalloc(&r.buf, sizeof(unsigned long long) * 8 * kSlots);
            if (cur != dev) (void)hipSetDevice(cur);
            if (e != hipSuccess) {
                (void)hipGetLastError();
                r.buf = nullptr;
                return nullptr;
            }
        }
        slot = r.buf + 8 * (r.next++ % kSlots);
    }
    if (hipMemsetAsync(slot, 0, sizeof(unsigned long long) * 8, s) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    return slot;
}

template <typename T>
int net_launch(const NetP<T>& p, bool ex, bool du, int np, long long lds_bytes, int program,
               void* stream) {
    const long long wg_bytes = lds_bytes * net_units(np);
    const void* fn = program > 0 && !ex ? prog_fn<T>(program - 1) : net_fn<T>(ex, du, np, wg_bytes);
    if (!fn) return fail(CGP_EINVAL, "net: no instantiation for %d pairs per workgroup", np);
    const int per_cu = net_occupancy(fn, (int)wg_bytes, net_threads(np));
    if (per_cu <= 0)
        return fail(CGP_EINVAL, "net: kernel cannot be resident with %lld B LDS", wg_bytes);
    const long long groups = (p.uend - p.ubeg + net_units(np) - 1) / net_units(np);
    long long grid = (long long)per_cu * device_cus();
    if (grid > groups) grid = groups;
    grid = (grid + 7) / 8 * 8;                  // whole XCD rounds
    NetP<T> arg = p;
    hipStream_t s = as_stream(stream);
    arg.work = work_counters(s);
    if (!arg.work) return fail(CGP_EHIP, "net: work counters");
    void* args[] = {&arg};
    const hipError_t e = hipLaunchKernel(fn, dim3((unsigned)grid), dim3(net_threads(np)), args,
                                         (size_t)wg_bytes, s);
    if (e != hipSuccess) return fail(CGP_EHIP, "net_kernel launch: %s", hipGetErrorString(e));
    return check_launch("net_kernel");
}

template <typename T>
int net_impl(const cgp_net_args* a, void* stream) {
    if (!a) return fail(CGP_EINVAL, "net: args is NULL");
    if (!a->x || !a->y || !a->out || !a->ops || a->nops <= 0)
        return fail(CGP_EINVAL, "net: NULL pointer or empty op list");
    if (a->n1 <= 0 || a->n2 <= 0 || a->n1 >= (1LL << 31) || a->n2 >= (1LL << 31) ||
        a->ldo < a->n2)
        return fail(CGP_EINVAL, "net: bad sizes n1=%lld n2=%lld ldo=%lld", (long long)a->n1,
                    (long long)a->n2, (long long)a->ldo);
    if (a->same && (a->n1 != a->n2 || !a->kdiag))
        return fail(CGP_EINVAL, "net: same tile needs n1 == n2 and kdiag");
    if (a->channels <= 0 || a->h <= 0 || a->w <= 0)
        return fail(CGP_EINVAL, "net: bad image shape");
    const long long lds_bytes = (long long)a->lds_elems * (long long)sizeof(T);
    if (a->lds_elems <= 0 || lds_bytes + kStaticLds > 160 * 1024)
        return fail(CGP_EINVAL, "net: LDS footprint %lld bytes out of range", lds_bytes);
    if (a->final_slot < 0 || a->final_slot >= a->lds_elems || a->hs < 0 ||
        a->hs >= a->lds_elems || a->part < 0 || a->part + 2 > a->lds_elems)
        return fail(CGP_EINVAL, "net: slot offsets out of range");
    NetP<T> p;
    p.x = static_cast<const T*>(a->x);
    p.y = static_cast<const T*>(a->y);
    p.out = static_cast<T*>(a->out);
    p.kdiag = static_cast<const T*>(a->kdiag);
    p.ops = a->ops;
    p.ldo = a->ldo;
    p.n1 = (unsigned)a->n1;
    p.n2 = (unsigned)a->n2;
    p.nbi = (unsigned)((a->n1 + kST - 1) / kST);
    p.nbj = (unsigned)((a->n2 + kST - 1) / kST);
    const long long tiles = a->same ? (long long)p.nbi * (p.nbi + 1) / 2
                                    : (long long)p.nbi * p.nbj;
    if (tiles * kST * kST >= (1LL << 40)) return fail(CGP_EINVAL, "net: tile too large");
    p.units = tiles * kST * kST;
    p.nops = a->nops;
    p.channels = a->channels;
    p.hw_in = a->h * a->w;
    p.same = a->same;
    p.final_slot = a->final_slot;
    p.hs = a->hs;
    p.part = a->part;
    p.lds_elems = a->lds_elems;
    p.exact = (a->flags & CGP_FLAG_EXACT_RELU) ? 1 : 0;
    const int np = a->pairs <= 0 ? 1 : a->pairs;
    if (np != 1 && np != 2 && np != 4 && np != kMaxNP)
        return fail(CGP_EINVAL, "net: %d pairs per workgroup (1, 2, 4 or 16)", np);
    if (lds_bytes * net_units(np) + kStaticLds > 160 * 1024)
        return fail(CGP_EINVAL, "net: %d pairs need %lld B LDS (+ %lld B static)", np,
                    lds_bytes * net_units(np), kStaticLds);
    // multi-pair stages address a pair's variance maps (<= 8 * threads / np pixels) with
    // 32-bit byte offsets (VarSrc)
    if (np > 1 && (a->n1 > a->n2 ? a->n1 : a->n2) * (8LL * net_threads(np) / np) *
                          (long long)sizeof(T) >= (1LL << 32))
        return fail(CGP_EINVAL, "net: %lld images too many for %d pairs per workgroup",
                    (long long)(a->n1 > a->n2 ? a->n1 : a->n2), np);
    if (a->unit_begin == 0 && a->unit_end == 0) {
        p.ubeg = 0;
        p.uend = p.units;
    } else {
        p.ubeg = a->unit_begin;
        p.uend = a->unit_end;
    }
    if (p.ubeg < 0 || p.uend > p.units || p.ubeg >= p.uend || p.ubeg % np)
        return fail(CGP_EINVAL, "net: unit range [%lld, %lld) of %lld", (long long)p.ubeg,
                    (long long)p.uend, (long long)p.units);
    p.final_stage = a->final_stage;
    const bool du = (a->flags & CGP_FLAG_NET_DUAL) != 0;
    const int prog = a->program;
    if (prog < 0 || prog > kNumProgs)
        return fail(CGP_EINVAL, "net: program %d of %d", prog, kNumProgs);
    if (prog > 0) {
        const ProgInfo& I = kProgs[prog - 1];
        if (I.nops != a->nops || I.pairs != np || I.dual != (du ? 1 : 0) ||
            I.lds_elems != a->lds_elems || !(I.sizes & (int)sizeof(T)))
            return fail(CGP_EINVAL, "net: program %d does not fit this op list", prog);
    }
    return net_launch<T>(p, p.exact != 0, du, np, lds_bytes, prog, stream);
}

}  // namespace

extern "C" {

int cgp_net_geometry(int32_t h, int32_t w, int32_t ho, int32_t wo, int32_t taps,
                     int32_t stride, int32_t offset) {
    for (int k = 0; k < kNumGeo; ++k) {
        const GeoRow& g = kGeoTable[k];
        if (g.h == h && g.w == w && g.ho == ho && g.wo == wo && g.taps == taps &&
            g.s == stride && g.off == offset)
            return k;
    }
    return -1;
}

int cgp_net_resolution(int32_t h, int32_t w) { return res_index(h, w); }

size_t cgp_net_op_size(void) { return sizeof(cgp_net_op); }
size_t cgp_net_args_size(void) { return sizeof(cgp_net_args); }

int cgp_net_supertile(void) { return kST; }

int cgp_net_units(int32_t pairs) { return net_units(pairs <= 0 ? 1 : pairs); }

int cgp_net_hs_elems(int32_t code) {
    return (code >= 0 && code < kNumGeo) ? kGeoTable[code].hs_elems : -1;
}

int cgp_net_occupancy(int32_t lds_bytes, int32_t f64, int32_t flags, int32_t pairs) {
    if (pairs <= 0) pairs = 1;
    if (lds_bytes <= 0 || (long long)lds_bytes * pairs > 160 * 1024) return 0;
    return f64 ? net_occupancy_for<double>(lds_bytes, flags, pairs)
               : net_occupancy_for<float>(lds_bytes, flags, pairs);
}

int cgp_net_static_lds(void) { return (int)kStaticLds; }

int cgp_net_validate(const cgp_net_op* ops, int32_t nops, int32_t pairs) {
    if (!ops || nops <= 0) return fail(CGP_EINVAL, "net_validate: NULL or empty op list");
    const int np = pairs <= 0 ? 1 : pairs;
    auto geo = [](const cgp_net_op& r) -> const GeoRow* {
        const int g = r.code & CGP_NET_CODE_GEOMETRY;
        return r.kind == CGP_NET_CONV && r.code >= 0 && g < kNumGeo ? &kGeoTable[g] : nullptr;
    };
    for (int k = 0; k < nops; ++k) {
        const cgp_net_op& r = ops[k];
        const bool sum = r.kind == CGP_NET_CONV && r.code >= 0 && (r.code & CGP_NET_CODE_SUM);
        const bool from = r.kind == CGP_NET_CONV && r.code >= 0 && (r.code & CGP_NET_CODE_FROM_SUM);
        if (sum) {
            const GeoRow* g = geo(r);
            const bool point = g && g->taps == 1 && g->off == 0;
            const bool reduce = g && g->ho == 1 && g->wo == 1 && g->off == 0 &&
                                g->taps == g->h && g->taps == g->w;
            if (!g || g->taps <= 3 || point || reduce)
                return fail(CGP_EINVAL, "net_validate: op %d: CGP_NET_CODE_SUM needs a separable "
                                        "conv (more than 3 taps, not pointwise, not a reduction)", k);
            if (r.add >= 0 || r.dst2 >= 0)
                return fail(CGP_EINVAL, "net_validate: op %d: CGP_NET_CODE_SUM with an addend or "
                                        "a second output", k);
            if (np > 2)
                return fail(CGP_EINVAL, "net_validate: op %d: CGP_NET_CODE_SUM in a %d-pair stage "
                                        "(one pair per workgroup or half only)", k, np);
            if (k + 1 >= nops || !(ops[k + 1].kind == CGP_NET_CONV && ops[k + 1].code >= 0 &&
                                   (ops[k + 1].code & CGP_NET_CODE_FROM_SUM)) ||
                ops[k + 1].src != r.dst)
                return fail(CGP_EINVAL, "net_validate: op %d: CGP_NET_CODE_SUM not followed by the "
                                        "CGP_NET_CODE_FROM_SUM reduction of its map", k);
            for (int m = k + 2; m < nops; ++m)
                if (ops[m].src == r.dst || ops[m].add == r.dst)
                    return fail(CGP_EINVAL, "net_validate: op %d reads the map of SUM op %d, "
                                            "which is never stored", m, k);
        }
        if (from) {
            const GeoRow* g = geo(r);
            const bool reduce = g && g->ho == 1 && g->wo == 1 && g->off == 0 &&
                                g->taps == g->h && g->taps == g->w;
            if (!reduce || np > 2)
                return fail(CGP_EINVAL, "net_validate: op %d: CGP_NET_CODE_FROM_SUM needs a "
                                        "one-pair full-map reduction", k);
            if (k == 0 || !(ops[k - 1].kind == CGP_NET_CONV && ops[k - 1].code >= 0 &&
                            (ops[k - 1].code & CGP_NET_CODE_SUM)))
                return fail(CGP_EINVAL, "net_validate: op %d: CGP_NET_CODE_FROM_SUM without a "
                                        "CGP_NET_CODE_SUM conv before it", k);
        }
    }
    return CGP_OK;
}

int cgp_net_program(const cgp_net_op* ops, int32_t nops, int32_t pairs, int32_t flags,
                    int32_t lds_elems, int32_t itemsize) {
    if (!ops || nops <= 0) return 0;
    return prog_match(ops, nops, pairs <= 0 ? 1 : pairs, (flags & CGP_FLAG_NET_DUAL) ? 1 : 0,
                      lds_elems, itemsize);
}

int cgp_net_f64(const cgp_net_args* args, void* stream) { return net_impl<double>(args, stream); }
int cgp_net_f32(const cgp_net_args* args, void* stream) { return net_impl<float>(args, stream); }

}  // extern "C"
