/*
 * cnngp.h — C ABI of the MI355X-native CNN-GP hot path (libcnngp.so).
 *
 * The reference (waleedbinkhalid74/cnn-gp) is pure Python over PyTorch; it has no FFI of
 * its own.  Each entry point below replaces the PyTorch op sequence one reference
 * function issues, so a ctypes (or any C FFI) binding can drive the whole NNGP Gram
 * recursion and the GP solve without torch compute.  Citations are
 * /root/reference/<file>:<line>.
 *
 * Conventions
 *   - Every buffer is DEVICE memory owned by the caller (torch allocates it and passes
 *     data_ptr()).  The library never frees caller memory.  rocBLAS / rocSOLVER handles
 *     are owned by the library, cached per device.
 *   - Every compute entry point is asynchronous on `stream` (a hipStream_t passed as
 *     void*; NULL = the null stream).  No host synchronisation inside, except the solve,
 *     which returns potrf's `info` to the host.
 *   - Return value: 0 on success, otherwise a CGP_E* code; cgp_last_error() returns a
 *     thread-local message for the last failure.  No C++ exception crosses the ABI.
 *   - Layouts are row-major and dense.  A "map" is one H×W spatial plane.  The pair
 *     index of a non-diagonal tile is m = i·N2 + j (i over the N1 rows, j over the N2
 *     columns); for a diagonal (diag=1) tile m = i = j.
 *   - _f64 entry points compute in double, _f32 in float (the reference's production
 *     dtype).  Scalars (weight, bias) are passed as double and rounded to the compute
 *     type inside the f32 entry points.
 */
#ifndef CNNGP_H
#define CNNGP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CGP_ABI_VERSION 11

/* error codes */
#define CGP_OK 0
#define CGP_EINVAL 1001   /* argument check failed (shapes, null pointers, ranges) */
#define CGP_EHIP 1002     /* a HIP runtime call or kernel launch failed */
#define CGP_EBLAS 1003    /* rocBLAS / rocSOLVER returned an error status */

/* cgp_conv_args.pre / .post */
#define CGP_PRE_NONE 0
#define CGP_PRE_RELU 1     /* apply the ReLU covariance map to the input while staging it */
#define CGP_PRE_MOMENTS 2  /* the input is (x, y) images; stage mean_c x·y instead of a map */
#define CGP_POST_NONE 0
#define CGP_POST_RELU 1    /* apply the ReLU covariance map to the conv output */

/* cgp_conv_args.flags / cgp_relu_args.flags */
#define CGP_FLAG_EXACT_RELU 1  /* evaluate the ReLU map op by op like the reference
                                  (correctly rounded 1/sqrt, sqrt, acos, division);
                                  default is the closed form max(c,0)/2 + sqrt(t)·x^1.5·P(x)
                                  of csrc/relu_poly.h, within 1e-14 of the exact map */
#define CGP_FLAG_GENERIC_CONV 2  /* force the generic conv kernel (tests / A-B timing) */

int cgp_abi_version(void);
/* The factor cgp_net_f64's closed-form ReLU expects on its x-side variance maps (var_x /
 * var2_x without CGP_FLAG_EXACT_RELU): 1/16 from ABI 9 (1/4 in ABI 6-8).  cgp_var_chain_*
 * writes its qstore copies with it; a host scaling maps itself uses this value. */
double cgp_net_xvar_scale(void);
const char* cgp_last_error(void);
/* sizeof of the argument structs, so an FFI can verify its mirror of the layout */
size_t cgp_conv_args_size(void);
size_t cgp_relu_args_size(void);
/* number of visible HIP devices (0 without a GPU; never fails) */
int cgp_device_count(void);
/* host-only self test of the library's integer helpers (no GPU needed); 0 = pass */
int cgp_selftest(void);

/*
 * Input moments — replaces NNGPKernel.forward's moment step, kernels.py:44-49:
 *   xy[m] = mean_c x[i,c]·y[j,c]   (diag: xy[i] = mean_c x[i,c]·y[i,c])
 * x: [n1][c][hw], y: [n2][c][hw]; xy: [n1·n2][hw] (diag: [n1][hw]).
 */
int cgp_moments_xy_f64(const double* x, const double* y, int64_t n1, int64_t n2,
                       int32_t c, int32_t hw, int32_t diag, double* xy, void* stream);
int cgp_moments_xy_f32(const float* x, const float* y, int64_t n1, int64_t n2,
                       int32_t c, int32_t hw, int32_t diag, float* xy, void* stream);
/*
 * Per-image variances — kernels.py:48-49: xx[i] = mean_c x[i,c]², yy[j] = mean_c y[j,c]².
 * Writes xx: [n1][hw] and yy: [n2][hw] (they may be one contiguous [n1+n2][hw] block).
 */
int cgp_moments_var_f64(const double* x, const double* y, int64_t n1, int64_t n2,
                        int32_t c, int32_t hw, double* xx, double* yy, void* stream);
int cgp_moments_var_f32(const float* x, const float* y, int64_t n1, int64_t n2,
                        int32_t c, int32_t hw, float* xx, float* yy, void* stream);

/*
 * Conv2d covariance stencil — replaces Conv2d.propagate, kernels.py:92-98
 * (F.conv2d with the constant kernel of kernels.py:78-88, then + var_bias):
 *   out[m,oh,ow] = weight · Σ_{a,b<taps} in[m, oh·s+off+a·d, ow·s+off+b·d] + bias
 * with zero padding outside [0,h)×[0,w).  `offset` is -padding, plus `dilation` when the
 * reference pads an even kernel to (k+1)² with a zero first row/column (kernels.py:73-84).
 * Optional fusions (one HBM pass instead of two or three):
 *   pre  = CGP_PRE_RELU:    the staged input is ReLU.propagate(in) (kernels.py:134-165),
 *                           using pre_xx/pre_yy = the variances at the ReLU's input;
 *   pre  = CGP_PRE_MOMENTS: the staged input is mean_c x·y of in (=x) and in_y (=y);
 *   post = CGP_POST_RELU:   out is ReLU.propagate of the conv output, using
 *                           post_xx/post_yy = the variances of the conv output;
 *   addend != NULL:         out += addend after everything else (Sum, kernels.py:252-254,
 *                           kernel_patch.py:43-63).
 * Variance maps (pre_xx etc.) are [n1][h·w] / [n2][h·w] at the resolution they apply to.
 */
typedef struct cgp_conv_args {
    const void* in;       /* [nmaps][h][w]; or x [n1][channels][h][w] with CGP_PRE_MOMENTS */
    const void* in_y;     /* y [n2][channels][h][w] with CGP_PRE_MOMENTS, else NULL */
    void* out;            /* [nmaps][ho][wo] */
    const void* addend;   /* [nmaps][ho][wo] or NULL */
    const void* pre_xx;   /* CGP_PRE_RELU: [n1][h][w] */
    const void* pre_yy;   /* CGP_PRE_RELU: [n2][h][w] */
    const void* post_xx;  /* CGP_POST_RELU: [n1][ho][wo] */
    const void* post_yy;  /* CGP_POST_RELU: [n2][ho][wo] */
    int64_t nmaps;        /* n1·n2, or n1 when diag */
    int64_t n1, n2;
    int32_t h, w, ho, wo;
    int32_t taps, offset, stride, dilation;
    int32_t channels;     /* CGP_PRE_MOMENTS only */
    int32_t pre, post;
    int32_t same, diag;   /* KernelPatch.same / .diag (kernel_patch.py:4-30) */
    int32_t maps_per_block; /* 0 = library default */
    int32_t flags;          /* CGP_FLAG_* */
    int32_t reserved;
    double weight, bias;
} cgp_conv_args;
int cgp_conv_f64(const cgp_conv_args* args, void* stream);
int cgp_conv_f32(const cgp_conv_args* args, void* stream);

/*
 * ReLU covariance map on the pair maps — ReLU.propagate, kernels.py:134-165:
 *   t = xx[i]·yy[j] + f32_tiny; cos = clamp(xy·rsqrt(t), -1, 1);
 *   sin = sqrt(max(t - xy², 0)); out = (sin + (π - acos(cos))·xy) / 2π
 * same && !diag: out[i,i] = xx[i]/2; same && diag: out = xx/2.  Optional out += addend.
 * In-place (out == xy) is allowed.
 */
typedef struct cgp_relu_args {
    const void* xy;      /* [nmaps][hw] */
    void* out;           /* [nmaps][hw] */
    const void* addend;  /* [nmaps][hw] or NULL */
    const void* xx;      /* [n1][hw] variances at the ReLU input */
    const void* yy;      /* [n2][hw] */
    int64_t nmaps, n1, n2;
    int32_t hw, same, diag, flags;   /* flags: CGP_FLAG_* */
} cgp_relu_args;
int cgp_relu_f64(const cgp_relu_args* args, void* stream);
int cgp_relu_f32(const cgp_relu_args* args, void* stream);

/*
 * ReLU on the per-image variances — kernels.py:154-164: xx' = xx/2;
 * yy' = xx' if same else yy/2.  xx: [n1][hw], yy: [n2][hw].
 */
int cgp_var_relu_f64(const double* xx, const double* yy, int64_t n1, int64_t n2, int32_t hw,
                     int32_t same, double* xx_out, double* yy_out, void* stream);
int cgp_var_relu_f32(const float* xx, const float* yy, int64_t n1, int64_t n2, int32_t hw,
                     int32_t same, float* xx_out, float* yy_out, void* stream);

/*
 * out = alpha·a + beta·b (b may be NULL: out = alpha·a), n elements.  The unfused form
 * of Sum (alpha = beta = 1, kernel_patch.py:43-63) and Mixture (kernels.py:220-225).
 * Products and the sum are rounded separately (no FMA contraction), like torch.
 */
int cgp_axpby_f64(double alpha, const double* a, double beta, const double* b, double* out,
                  int64_t n, void* stream);
int cgp_axpby_f32(double alpha, const float* a, double beta, const float* b, float* out,
                  int64_t n, void* stream);

/*
 * dst[k] = alpha·src[k] (n[k] elements) for count buffers, in one launch per 32 (host
 * arrays of device pointers).  No reference counterpart: it fills the quartered x-side
 * variance maps the fp64 closed-form ReLU of cgp_net_f64 reads (one launch per tile instead
 * of one cgp_axpby_f64 per map; cnn_gp/netplan.py).
 */
int cgp_scale_batch_f64(int32_t count, const double* const* src, double* const* dst,
                        const int64_t* n, double alpha, void* stream);

/* load_kern's float32 → float64 widening, classify_gp.py:45-48 */
int cgp_cast_f32_f64(const float* in, double* out, int64_t n, void* stream);
/* dst[c][r] = src[r][c]; src [rows][cols] row-major */
int cgp_transpose_f64(const double* src, int64_t rows, int64_t cols, double* dst, void* stream);

/*
 * GP solve — replaces classify_gp.solve_system + diag_add (classify_gp.py:17-36):
 * scipy.linalg.solve(K, Y, assume_a='pos', lower=False) reads only the UPPER triangle
 * of the row-major K (its strictly-lower tiles are NaN in the reference's HDF5 files).
 *   K:  [n][ldk] row-major fp64; overwritten by the Cholesky factor of the column-major
 *       view's lower triangle (= the row-major upper triangle): for n > CGP_CHOL_NB (env,
 *       default 2048) a blocked right-looking factorisation (rocsolver_dpotrf_64 per
 *       diagonal block, rocblas_dtrsm_64 panel, rocblas_dsyrk_64 trailing update), else
 *       rocsolver_dpotrf_64 on the whole matrix; then rocsolver_dpotrs_64.
 *   bt: the right-hand sides TRANSPOSED, [nrhs][ldb] row-major (= column-major n×nrhs);
 *       overwritten by the solution (transposed).
 *   jitter is added to K's diagonal first (diag_add, classify_gp.py:30-36).
 *   *info (host): 0 = success; > 0 = the leading minor of that order is not positive
 *   definite (scipy raises LinAlgError in that case).
 * Synchronises `stream` before returning.
 */
int cgp_chol_solve_f64(double* k, int64_t n, int64_t ldk, double* bt, int64_t nrhs,
                       int64_t ldb, double jitter, int64_t* info, void* stream);
/*
 * Phase times (ms, HIP events on the call's stream) of the last cgp_chol_solve_f64 on
 * `stream`'s device: ms[0] = jitter (diag_add, classify_gp.py:30-36), ms[1] = the
 * Cholesky factorisation, ms[2] = dpotrs (0 when the factorisation failed).  Lets a
 * caller split the solve_system wall time of classify_gp.py:17-27 (no reference
 * counterpart: the reference times nothing).  CGP_EINVAL before any solve on that device.
 */
int cgp_chol_last_phases(void* stream, double* ms);
/*
 * ABI 10: cgp_chol_solve_f64 that also returns ITS OWN phase times in phase_ms[3] (ms:
 * jitter, factor, potrs; NULL: none), taken under the device's solver lock — another
 * thread's solve on the same device cannot overwrite them between the call and a later
 * cgp_chol_last_phases.  phase_ms is -1 in every slot when the call fails before timing.
 */
int cgp_chol_solve_f64_timed(double* k, int64_t n, int64_t ldk, double* bt, int64_t nrhs,
                             int64_t ldb, double jitter, int64_t* info, double* phase_ms,
                             void* stream);
/*
 * ABI 11: the solution check (no reference counterpart: scipy's solve never hands back a
 * wrong factor silently; rocSOLVER / rocBLAS factorisations in processes sharing one GPU
 * have, with info = 0 — round 5).  classify_gp.py:17-27's system K·X = Y, K given by its
 * row-major upper triangle, the triangle cgp_chol_solve_f64 reads and overwrites:
 *   cgp_sym_mirror_f64: K[i][j] = K[j][i] for every i > j (the strictly-lower triangle,
 *     unread by the solve, takes the system) and diag[i] = K[i][i] ([n], device).  Call
 *     before the factorisation (after any jitter: diag then holds K + jitter·I's).
 *   cgp_sym_residual_f64: r −= (L + Lᵀ + diag(d))·X with L the strictly-lower triangle
 *     of k: X and r are [nrhs][ldx] row-major (transposed, as cgp_chol_solve_f64's bt);
 *     r holds Y on entry and Y − K·X on return; *sumsq (device) += Σ_{i>j} K[i][j]² (so
 *     ‖K‖_F² = 2·sumsq + Σ d²).  Atomic accumulation: the last bits vary run to run.
 * One pass over the lower triangle each (n²/2 · 8 bytes read; the mirror writes as much).
 */
int cgp_sym_mirror_f64(double* k, int64_t n, int64_t ldk, double* diag, void* stream);
int cgp_sym_residual_f64(const double* k, int64_t n, int64_t ldk, const double* diag,
                         const double* x, double* r, int64_t nrhs, int64_t ldx, double* sumsq,
                         void* stream);
/*
 * Row-major C[m][n] = A[m][kdim] @ B[kdim][n] (fp64, rocBLAS) — the Kxz @ α product of
 * print_accuracy, classify_gp.py:39-42.
 */
int cgp_gemm_f64(const double* a, const double* b, double* c, int64_t m, int64_t n,
                 int64_t kdim, void* stream);
/*
 * GP predictive variance of m test points (the Kv_diag / Kt_diag
 * datasets save_kernel.py:33-36 writes are the prior variances this subtracts from):
 *   var[t] = kz_diag[t] − Kzx[t,:] · Kxx⁻¹ · Kxz[:,t]
 * given the factor cgp_chol_solve_f64 left in k (row-major upper triangle U, Kxx = UᵀU;
 * only that triangle is read, the NaN lower tiles of the reference's files are ignored).
 *   kxz: Kzx as [m][ldz] row-major (one test point per row, ldz >= n) — overwritten by
 *        V = U⁻ᵀ Kxz (rocblas_dtrsm_64, in place), so var[t] = kz_diag[t] − Σ_r V[t][r]².
 *   kz_diag: [m] prior variances (DiagIterator output); var: [m] out (may alias kz_diag).
 */
int cgp_pred_var_f64(const double* k, int64_t n, int64_t ldk, double* kxz, int64_t m,
                     int64_t ldz, const double* kz_diag, double* var, void* stream);
/* out[r] = argmax_c a[r][c] (first maximum, like torch.argmax), a: [rows][cols] */
int cgp_argmax_rows_f64(const double* a, int64_t rows, int64_t cols, int64_t* out,
                        void* stream);


/* ---------------------------------------------------------------------------------
 * Whole-network pair kernel.  Replaces the per-layer loop of Sequential.propagate
 * (kernels.py:184-187) over ALL layers for a tile: one workgroup owns one (i, j) pair
 * at a time and carries its covariance map through every op in LDS; only the images,
 * the per-image variance maps (read-only, L2-resident) and the final K[i, j] touch
 * global memory.  The host lowers the module tree to a list of cgp_net_op over LDS
 * "slots" (row-major planes with zero column halos) and supplies the
 * variance maps from the per-image pipeline (cgp_conv_* / cgp_var_relu_* on xx, yy).
 *
 *   CGP_NET_MOMENTS  dst = mean_c x_i[c]·y_j[c]                   kernels.py:44-47
 *   CGP_NET_CONV     dst = w·Σ_window src + b  [→ ReLU] [+ add]    kernels.py:92-98
 *   CGP_NET_RELU     dst = relu(src)           [+ add]            kernels.py:134-165
 *   CGP_NET_LINEAR   dst = weight·src + bias·add   (Sum / Mixture: kernels.py:220-254)
 *   CGP_NET_LOAD / CGP_NET_STORE   move a map between a slot and the per-unit state
 *                    record (var_x = the state buffer of the launch's units: record of
 *                    unit u at (u - unit_begin)·code elements; add = the map's offset in
 *                    the record) at a stage boundary
 *
 * Stages.  A network whose tail runs on small maps (a ResNet's 14x14 and 7x7 blocks)
 * is split at the resolution drops: the tail stages run several pairs per workgroup
 * (`pairs` = 4 at <= 16x16, 16 at <= 8x8), so a small map's ops still fill the
 * workgroup; the live maps cross a boundary through the state buffer.
 *
 * Same tiles (same=1) evaluate only i < j, mirror K[j, i] = K[i, j] (the recursion is
 * symmetric in (i, j) when y = x) and take K[i, i] = kdiag[i] — the per-image
 * pipeline's final value, which is exactly what the reference's same/diag override of
 * every ReLU (kernels.py:155-162) makes the (i, i) pair map equal to.
 * --------------------------------------------------------------------------------- */
#define CGP_NET_CONV 0
#define CGP_NET_RELU 1
#define CGP_NET_MOMENTS 2
#define CGP_NET_LINEAR 3
#define CGP_NET_LOAD 4     /* stage input:  slot dst <- state[unit][add .. add + h·w) */
#define CGP_NET_STORE 5    /* stage output: state[unit][add .. add + h·w) <- slot src */
/* CONV code flag: a separable conv writes the rows of its row-sum scratch that lie outside
 * its input as zeros before its column pass; with this flag it skips them (the host has
 * proved no op since their last zeroing wrote there — cyclically over the stage's op
 * list, which repeats for every pair a workgroup walks).  The scratch is the LDS arena's
 * first cells: separable row passes write their input rows there and a one-pair
 * full-map reduction its two wave partial sums. */
#define CGP_NET_CODE_HS_CLEAN 0x100
/* CONV code flags of a map that only a full-map reduction reads (ABI 9; the host sets
 * both or neither):
 *   CGP_NET_CODE_SUM       a separable conv does not store its output map: each wave adds
 *                          its outputs (after the ReLU) into the pair's two wave partial sums
 *   CGP_NET_CODE_FROM_SUM  the next op, a full-map reduction (1x1 output, window = map) of
 *                          that map, reads those partial sums instead of the map
 * Preconditions (cgp_net_validate checks them on a host copy of the op list; the kernels
 * do not, since the list they read is in device memory):
 *   - SUM only on a separable conv: more than 3 taps, not pointwise, not a full-map
 *     reduction (the direct, pointwise and reduction forms store their map regardless);
 *   - SUM with add < 0 and dst2 < 0 (the summed outputs are the conv+ReLU values only);
 *   - one pair per workgroup or half (pairs 1 or 2): multi-pair stages ignore both flags;
 *   - the op right after a SUM conv is the FROM_SUM reduction of its dst map, and no later
 *     op reads that map (it is never stored); FROM_SUM only right after a SUM conv.
 * A list that breaks them reads zeroed partial sums (deterministic, wrong). */
#define CGP_NET_CODE_SUM 0x200
#define CGP_NET_CODE_FROM_SUM 0x400
#define CGP_NET_CODE_GEOMETRY 0xff  /* the cgp_net_geometry() code in the low bits */

typedef struct cgp_net_op {
    int32_t kind;          /* CGP_NET_* */
    int32_t code;          /* CONV: cgp_net_geometry(), | CGP_NET_CODE_HS_CLEAN when the row
                              sums' zero rows are known to be zero already, | CGP_NET_CODE_SUM
                              / CGP_NET_CODE_FROM_SUM for a map only a reduction reads;
                              RELU/LINEAR/MOMENTS: cgp_net_resolution() of the map, or -1
                              (generic) */
    int32_t src, dst, add; /* LDS element offsets of the slots' (0, 0) pixel; add < 0: none */
    int32_t ws_in, ws_out; /* row strides (elements) of the src slot / dst and add slots */
    int32_t relu;          /* CONV: apply the ReLU map to the conv output (then + add) */
    int32_t h, w;          /* RELU / LINEAR / MOMENTS: map size (CONV: output size) */
    uint32_t div_m, div_s; /* w as a multiply-high divisor (host: make_fastdiv(w)) */
    int32_t dst2;          /* CONV/RELU/LINEAR: also write relu(result) here (< 0: no) */
    int32_t zero_halo;     /* before the op, zero the halo cells of the dst slot (bits 0-15)
                              and of the dst2 slot (bits 16-31), each (HL << 8) | gap:
                              HL cells before pixel (0, 0) and `gap` = ws_out - w cells
                              after every row; 0 = none.  Set on a slot placed on cells
                              another slot used as data (the LDS arena is shared across
                              map sizes). */
    double weight, bias;   /* CONV: w·Σ + b;  LINEAR: dst = weight·src + bias·add */
    const void* var_x;     /* ReLU input variances of the x images, [n1][h·w]; for
                              cgp_net_f64 without CGP_FLAG_EXACT_RELU: SCALED by
                              cgp_net_xvar_scale() (v/16 from ABI 9, v/4 before; the
                              scaled closed form; var2_x likewise) */
    const void* var_y;     /* ... of the y images, [n2][h·w] */
    const void* var2_x;    /* dst2's ReLU: variances of the result, [n1][h·w] */
    const void* var2_y;    /* [n2][h·w] */
} cgp_net_op;

typedef struct cgp_net_args {
    const void* x;         /* images [n1][channels][h][w] */
    const void* y;         /* images [n2][channels][h][w] (== x when same) */
    void* out;             /* K tile [n1][ldo] */
    const void* kdiag;     /* same tiles: K[i, i] (the per-image final variance), [n1] */
    const cgp_net_op* ops; /* DEVICE array of nops ops */
    int64_t n1, n2, ldo;
    int32_t nops, channels, h, w;
    int32_t same;          /* 1: y is x (Kxx diagonal tile) */
    int32_t final_slot;    /* LDS offset of the 1x1 result */
    int32_t hs;            /* LDS offset of the row-sum scratch */
    int32_t lds_elems;     /* LDS footprint of ONE pair (elements of the compute type) */
    int32_t flags;         /* CGP_FLAG_EXACT_RELU */
    int32_t pairs;         /* pairs per workgroup: 1; 2 = two one-pair slices of a 256-thread
                              workgroup (units u, u + 1: the same image i), any op list; or
                              4 / 16 for a stage whose maps are at most 16x16 / 8x8 (each
                              pair gets its own lds_elems arena) */
    int64_t unit_begin;    /* the tile's pair units this launch covers, [begin, end): unit */
    int64_t unit_end;      /* u = 64·supertile + 8·(i % 8) + j % 8; 0, 0 = the whole tile */
    int32_t final_stage;   /* 1: write K (the last stage); 0: the ops end in CGP_NET_STORE */
    int32_t program;       /* 0: interpret the op records; k > 0: run compiled program k,
                              the value cgp_net_program() returned for these records */
    int32_t part;          /* LDS offset of the two wave partial sums of a one-pair
                              full-map reduction (ABI 8): cells the host keeps off the
                              scratch's zero rows (CGP_NET_CODE_HS_CLEAN) */
} cgp_net_args;

/*
 * The per-image variance maps of a network in ONE launch (replaces the layer-by-layer
 * variance pipeline of cnn_gp/program.py Plan.run_variances: one launch per op).  A self
 * pair's recursion is linear (kernels.py:44-49 moments of x with itself, :92-98 convs,
 * :154-164 the ReLU of a variance is xx/2, :252-254 Sums), so one workgroup walks an image
 * through the whole op list in LDS and stores the maps the whole-network kernel reads.
 *   CGP_VAR_MOMENTS  dst = mean_c x·x                       (src unused)
 *   CGP_VAR_CONV     dst = w·Σ_window src + b   (zero padding; row sums, then columns)
 *   CGP_VAR_HALF     dst = src / 2
 *   CGP_VAR_SUM      dst = c0·t0 (+ c_k·t_k, k = 1..3, left to right; term slot -1 ends)
 * A value is stored when store >= 0: image g's map at out[n·store + g·ho·wo] (n = n1 + n2
 * images, the x images first), and, for g < n1, cgp_net_xvar_scale() × the map at
 * out[n·store_total + n1·qstore + g·ho·wo] when qstore >= 0 (the scaled x-side maps of
 * cgp_net_f64; store_total = Σ of every stored value's ho·wo).  Slots are LDS element
 * offsets, maps row-major [ho][wo].
 */
#define CGP_VAR_MOMENTS 0
#define CGP_VAR_CONV 1
#define CGP_VAR_HALF 2
#define CGP_VAR_SUM 3
typedef struct cgp_var_op {
    int32_t kind;
    int32_t dst;
    int32_t src[4];        /* CONV / HALF: src[0]; SUM: terms, -1 after the last */
    int32_t h, w, ho, wo;  /* input and output map sizes */
    int32_t taps, offset, stride, dilation;   /* CONV, as cgp_conv_args */
    int64_t store;         /* per-image element offset of the stored map, -1: not stored */
    int64_t qstore;        /* ... of its scaled x-side copy, -1: none */
    double weight, bias;   /* CONV */
    double coef[4];        /* SUM */
} cgp_var_op;
typedef struct cgp_var_args {
    const void* x;         /* images [n1][channels][h][w] */
    const void* y;         /* images [n2][channels][h][w] (n2 = 0: x only, e.g. same tiles) */
    void* out;             /* stored maps, see above */
    const cgp_var_op* ops; /* DEVICE array of nops ops */
    int64_t n1, n2;
    int64_t store_total;   /* Σ ho·wo of the stored values */
    int32_t nops, channels, h, w;
    int32_t lds_elems;     /* LDS of one image (elements of the compute type), scratch incl. */
    int32_t scratch;       /* LDS offset of the convs' row-sum scratch ([h][wo] elements) */
} cgp_var_args;
size_t cgp_var_op_size(void);
size_t cgp_var_args_size(void);
int cgp_var_chain_f64(const cgp_var_args* args, void* stream);
int cgp_var_chain_f32(const cgp_var_args* args, void* stream);

/* Geometry code of a conv for CGP_NET_CONV, or -1 if the fused kernel has no
 * instantiation for it (the caller then runs the layer-by-layer path). */
int cgp_net_geometry(int32_t h, int32_t w, int32_t ho, int32_t wo, int32_t taps,
                     int32_t stride, int32_t offset);
/* elements of row-sum scratch the conv of geometry `code` needs (-1: bad code) */
int cgp_net_hs_elems(int32_t code);
/* supertile edge of the pair walk: a tile's pairs are numbered in kST×kST blocks (upper
 * triangle of blocks when same), kST² units each; hosts size unit ranges with it */
int cgp_net_supertile(void);
size_t cgp_net_op_size(void);
size_t cgp_net_args_size(void);
/* Elementwise-op size code for cgp_net_op.code, or -1 (generic runtime-size path). */
int cgp_net_resolution(int32_t h, int32_t w);
/* cgp_net_args.flags: CGP_FLAG_EXACT_RELU, and CGP_FLAG_NET_DUAL when any op has dst2
 * (selects the kernel instantiation with the dual output stage) */
#define CGP_FLAG_NET_DUAL 4
/* workgroups per CU the fused kernel reaches with lds_bytes of LDS per pair and `pairs`
 * pairs per workgroup (0 if it cannot run) */
int cgp_net_occupancy(int32_t lds_bytes, int32_t f64, int32_t flags, int32_t pairs);
/* LDS arenas (one per pair unit) a workgroup of `pairs` pairs holds: `pairs`, except for
 * the two-pair head stage, whose workgroup holds two one-pair slices.  A stage needs
 * lds_bytes × cgp_net_units(pairs) + cgp_net_static_lds() <= 160 KB. */
int cgp_net_units(int32_t pairs);
/* The compiled program (k > 0) whose op list equals ops[0, nops) (HOST memory) in every
 * field but weight, bias and the variance / state pointers, for `pairs` pairs per
 * workgroup, flags (CGP_FLAG_NET_DUAL), the per-pair LDS footprint and the item size
 * (4 or 8); 0 if none.  The library holds the lowered programs of the reference configs
 * (net_programs.h); a program kernel runs them with every offset an immediate. */
int cgp_net_program(const cgp_net_op* ops, int32_t nops, int32_t pairs, int32_t flags,
                    int32_t lds_elems, int32_t itemsize);
/* ABI 10: CGP_OK, or CGP_EINVAL (message in cgp_last_error) when the op list (HOST memory)
 * breaks the CGP_NET_CODE_SUM / CGP_NET_CODE_FROM_SUM preconditions for `pairs` pairs per
 * workgroup.  cnn_gp.netplan calls it once per stage before the first launch. */
int cgp_net_validate(const cgp_net_op* ops, int32_t nops, int32_t pairs);
/* ABI 10: bytes of LDS the fused kernel declares statically per workgroup (pair table, SUM
 * partial sums, program records, work-counter slots), on top of lds_bytes ×
 * cgp_net_units(pairs): a stage fits when the sum is <= 160 KB. */
int cgp_net_static_lds(void);
/* ABI 6: cgp_net_f64's fast path reads var_x / var2_x quartered (see cgp_net_op). */
int cgp_net_f64(const cgp_net_args* args, void* stream);
int cgp_net_f32(const cgp_net_args* args, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* CNNGP_H */
