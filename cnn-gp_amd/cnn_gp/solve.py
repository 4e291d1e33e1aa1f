"""GP solve and classification on the device (reference:
exp_mnist_resnet/classify_gp.py:17-48).

``solve_system`` is ``scipy.linalg.solve(Kxx, Y, assume_a='pos', lower=False)`` done by
rocSOLVER: Cholesky (dpotrf_64) on the UPPER triangle of the row-major Kxx — the only
triangle the reference's HDF5 files fill — then dpotrs_64.  All through libcnngp.so.
"""
from __future__ import annotations

import ctypes
import math
from typing import Optional

import numpy as np
import torch

from . import _native as N

__all__ = ("solve_system", "diag_add", "load_kern", "print_accuracy", "predict",
           "accuracy", "one_hot_pm1", "predictive_variance", "warm_up_solver", "scores",
           "cast_into", "solve_phases", "mirror_upper", "alpha_backward_error",
           "alpha_check_tol", "check_alpha", "last_alpha_check")


def _device():
    if not torch.cuda.is_available():
        raise RuntimeError("cnn_gp solve needs a HIP device (there is no CPU path)")
    return torch.device("cuda", torch.cuda.current_device())


def _stream(dev):
    return torch.cuda.current_stream(dev).cuda_stream


# --- the solution check ----------------------------------------------------------------
# A factorisation can return info = 0 and a wrong factor (round 5: rocSOLVER / rocBLAS
# factorisations in several processes sharing one GPU, profiles/r5/r5z_*, r6/r6b_*).
# scipy never does that (classify_gp.py:24-26), so every solve verifies its α against the
# whole system it solved: the system is mirrored into the strictly-lower triangle before
# the factorisation (cgp_sym_mirror_f64; the solve reads and overwrites only the upper
# one), and afterwards r = Y − K·α is formed from that triangle in one pass
# (cgp_sym_residual_f64).  The measure is the normwise backward error
#     η = ‖r‖ / (‖K‖_F·‖α‖ + ‖Y‖)      (Frobenius norms),
# which a backward-stable Cholesky solve keeps at the rounding level whatever K's
# conditioning (2.4-2.6e-17 on the gloo rehearsal's 16 384² NNGP matrices); a wrong
# factor leaves rows of the system unsatisfied — possibly only a few, e.g. the rows of one
# corrupted trailing-update tile, which is why no row sample is used.

def alpha_check_tol(n: int) -> float:
    """The bound on η: 16·√n·eps (8.6e-13 at n = 60 000, 2.1e-14 at n = 37)."""
    return 16.0 * math.sqrt(max(int(n), 1)) * 2.0 ** -52


def mirror_upper(K):
    """K[i][j] = K[j][i] for every i > j, in place (the strictly-lower triangle — NaN
    tiles in the reference's files, data.py:22-29 — takes the system the upper triangle
    holds); returns the diagonal as float64 on K's device.  A float64 contiguous device
    matrix goes through cgp_sym_mirror_f64, a host matrix through torch."""
    n = K.shape[0]
    if K.device.type == "cuda":
        if K.dtype != torch.float64 or not K.is_contiguous():
            raise ValueError("mirror_upper: a contiguous float64 device matrix")
        d = torch.empty((n,), dtype=torch.float64, device=K.device)
        with torch.cuda.device(K.device):
            N.call("cgp_sym_mirror_f64", N.ptr(K), n, K.stride(0), N.ptr(d),
                   _stream(K.device))
        return d
    il = torch.tril_indices(n, n, -1)
    K[il[0], il[1]] = K[il[1], il[0]]
    return K.diagonal().to(torch.float64).clone()


def _residual_t(K, d, xt, yt):
    """(r = Yᵀ − (K·X)ᵀ as [nrhs, n], ‖K‖_F) from K's strictly-lower triangle and d, with
    X and Y given transposed ([nrhs, n] contiguous float64, on K's device)."""
    n = K.shape[0]
    if K.device.type == "cuda":
        r = yt.clone()
        ss = torch.zeros((1,), dtype=torch.float64, device=K.device)
        with torch.cuda.device(K.device):
            N.call("cgp_sym_residual_f64", N.ptr(K), n, K.stride(0), N.ptr(d), N.ptr(xt),
                   N.ptr(r), xt.shape[0], n, N.ptr(ss), _stream(K.device))
        fro = math.sqrt(2.0 * float(ss) + float((d * d).sum()))
        return r, fro
    L = torch.tril(K.to(torch.float64), -1)
    kx = L @ xt.T + L.T @ xt.T + d[:, None] * xt.T
    return yt - kx.T, math.sqrt(2.0 * float((L * L).sum()) + float((d * d).sum()))


def alpha_backward_error(K, d, alpha, Y) -> float:
    """η of ``alpha`` for the system whose strictly-lower triangle (mirror_upper) and
    diagonal ``d`` K holds: ‖Y − K·α‖ / (‖K‖_F·‖α‖ + ‖Y‖)."""
    n = K.shape[0]
    xt = alpha.reshape(n, -1).to(K.device, torch.float64).T.contiguous()
    yt = Y.reshape(n, -1).to(K.device, torch.float64).T.contiguous()
    r, fro = _residual_t(K, d.to(K.device, torch.float64), xt, yt)
    res = float(r.norm())
    den = fro * float(xt.norm()) + float(yt.norm())
    return res / den if den > 0 else (0.0 if res == 0 else math.inf)


def check_alpha(K, d, alpha, Y, tol: Optional[float] = None) -> float:
    """Raise ``np.linalg.LinAlgError`` when α's backward error for the system K·α = Y
    (K's strictly-lower triangle and diagonal d, see mirror_upper) exceeds ``tol``
    (default alpha_check_tol(n)) or is not finite; return η otherwise."""
    n = K.shape[0]
    tol = alpha_check_tol(n) if tol is None else float(tol)
    eta = alpha_backward_error(K, d, alpha, Y)
    if not eta <= tol:
        raise np.linalg.LinAlgError(
            f"the solution fails the residual check: backward error {eta:.3e} of K·α = Y "
            f"exceeds {tol:.3e} (n = {n}); the factorisation returned info = 0 with a "
            f"wrong factor")
    return eta


# the η of the last checked solve_system per device
_CHECKS = {}


def last_alpha_check(device=None) -> Optional[float]:
    """η of the last solve_system on ``device`` that ran the solution check (None if none)."""
    dev = torch.device(device) if device is not None else _device()
    return _CHECKS.get(_dev_key(dev))


def solve_system(Kxx, Y, jitter: float = 0.0, overwrite_a: bool = False,
                 check: bool = True, check_tol: Optional[float] = None):
    """Kxx⁻¹ Y for symmetric positive-definite Kxx given by its upper triangle.

    Kxx, Y: float64 tensors (classify_gp.py:19-23 asserts the same), on the host or the
    device.  By default the caller's Kxx is left untouched (the factorisation runs on a
    device copy), as scipy leaves a C-ordered array when it copies it to Fortran order.
    With ``overwrite_a=True`` and a contiguous device Kxx, the factorisation runs in place
    and saves the copy (28.8 GB at N = 60 000): the jitter lands on Kxx's diagonal and its
    upper triangle becomes the Cholesky factor U (Kxx = UᵀU) that ``predictive_variance``
    reads.  If Kxx is not positive definite, an in-place Kxx is left partly factored.
    Returns the solution on Y's device.  Raises ``np.linalg.LinAlgError`` if Kxx
    (+ jitter·I) is not positive definite, like scipy — and, with ``check`` (default),
    also if the solution fails the residual check against the whole system (check_alpha:
    backward error above ``check_tol``, default alpha_check_tol(n)), which scipy has no
    need of: a factorisation that returns info = 0 with a wrong factor must not hand back
    its α (round 5, processes sharing one GPU).  NaN entries in the upper triangle
    therefore raise too, where scipy (check_finite=False) returns a NaN α.  The check
    mirrors the system into the strictly-lower triangle of the matrix it factors (for an
    in-place solve: Kxx's, where the reference's files hold NaN) and costs two passes over
    that triangle (≈ 10 ms at n = 60 000, beside a ≈ 1.3 s factorisation).
    """
    assert Kxx.dtype == torch.float64 and Y.dtype == torch.float64, """
    It is important that `Kxx` and `Y` are `float64`s for the inversion,
    even if they were `float32` when being calculated."""
    n = Kxx.shape[0]
    assert Kxx.dim() == 2 and Kxx.shape[1] == n and Y.shape[0] == n
    vec = Y.dim() == 1
    Y2 = Y.reshape(n, -1)
    dev = Kxx.device if Kxx.device.type == "cuda" else _device()
    with torch.cuda.device(dev):
        if Kxx.device == dev and overwrite_a and Kxx.is_contiguous():
            K = Kxx
        elif Kxx.device == dev:
            K = Kxx.clone(memory_format=torch.contiguous_format)
        else:
            K = Kxx.to(dev).contiguous()
        yd = Y2.to(dev).contiguous()
        nrhs = yd.shape[1]
        bt = torch.empty((nrhs, n), dtype=torch.float64, device=dev)
        s = _stream(dev)
        N.call("cgp_transpose_f64", N.ptr(yd), n, nrhs, N.ptr(bt), s)
        if check:                       # the system, kept below the diagonal (+ jitter)
            d = mirror_upper(K)
            if jitter:
                d += float(jitter)
            yt = bt.clone()
        info = N._i64(0)
        ms = (N._f64 * 3)(-1.0, -1.0, -1.0)
        _PHASES.pop(_dev_key(dev), None)        # a failing solve leaves no phases behind
        _CHECKS.pop(_dev_key(dev), None)
        N.check(N.load().cgp_chol_solve_f64_timed(N.ptr(K), n, n, N.ptr(bt), nrhs, n,
                                                  float(jitter), ctypes.byref(info), ms, s),
                "cgp_chol_solve_f64")
        _PHASES[_dev_key(dev)] = tuple(ms)
        if info.value > 0:
            raise np.linalg.LinAlgError(
                f"Kxx is not positive definite (leading minor of order {info.value})")
        sol = torch.empty((n, nrhs), dtype=torch.float64, device=dev)
        N.call("cgp_transpose_f64", N.ptr(bt), nrhs, n, N.ptr(sol), s)
        if check:
            r, fro = _residual_t(K, d, bt, yt)
            res = float(r.norm())
            den = fro * float(bt.norm()) + float(yt.norm())
            eta = res / den if den > 0 else (0.0 if res == 0 else math.inf)
            tol = alpha_check_tol(n) if check_tol is None else float(check_tol)
            if not eta <= tol:
                raise np.linalg.LinAlgError(
                    f"the solution fails the residual check: backward error {eta:.3e} of "
                    f"K·α = Y exceeds {tol:.3e} (n = {n}); the factorisation returned "
                    f"info = 0 with a wrong factor")
            _CHECKS[_dev_key(dev)] = eta
    sol = sol.reshape(n) if vec else sol
    return sol.to(Y.device)


# the phases of the last solve_system per device, as that call's own timed solve returned
# them (cgp_chol_solve_f64_timed: taken under the solver's device lock, so a solve on
# another thread cannot swap them); dropped at the start of every solve_system
_PHASES = {}


def _dev_key(dev) -> int:
    dev = torch.device(dev)
    return dev.index if dev.index is not None else torch.cuda.current_device()


def solve_phases(device=None) -> Optional[dict]:
    """Seconds spent in the phases of the last solve_system on ``device`` (HIP events on
    its stream): jitter (diag_add), factor (the Cholesky), potrs — or None when the last
    solve_system there raised before its solve was timed (or none ran)."""
    dev = torch.device(device) if device is not None else _device()
    ms = _PHASES.get(_dev_key(dev))
    if ms is None or min(ms) < 0:
        return None
    return {"jitter_s": ms[0] * 1e-3, "factor_s": ms[1] * 1e-3, "potrs_s": ms[2] * 1e-3}


def warm_up_solver(device=None, background: bool = True):
    """Load rocBLAS / rocSOLVER's code objects for the blocked factorisation and the solve
    (the first dpotrf / dtrsm / dsyrk / dpotrs calls of a process pay ~0.2-0.4 s for it) by
    factoring an identity of n = 6·2048 + 64 (seven diagonal blocks, trailing updates up
    to 10 k wide: rocBLAS picks its large-size kernels there; 1.2 GB, ~20 ms) on a stream
    of its own.  With ``background`` it runs on a host thread and returns the thread: the pipeline
    starts it before the Kxx build, so the loading overlaps the kernels."""
    dev = torch.device(device) if device is not None else _device()

    def run():
        with torch.cuda.device(dev):
            st = torch.cuda.Stream(dev)
            with torch.cuda.stream(st):
                n = 6 * 2048 + 64
                K = torch.zeros((n, n), dtype=torch.float64, device=dev)
                solve_system(K, torch.ones((n, 10), dtype=torch.float64, device=dev),
                             jitter=1.0, overwrite_a=True, check=False)
            st.synchronize()

    if not background:
        run()
        return None
    import threading
    t = threading.Thread(target=run, name="cgp-solver-warmup", daemon=True)
    t.start()
    return t


def predictive_variance(Kfactor, Kxz, kz_diag, overwrite_kxz: bool = False):
    """GP posterior variance of the test points: kz_diag[t] − Kzx[t]·Kxx⁻¹·Kxz[:, t].

    Kfactor: the device tensor ``solve_system(Kxx, Y, overwrite_a=True)`` leaves Kxx in
    (its upper triangle holds U, Kxx = UᵀU; the lower triangle is never read).  Kxz:
    [m, n] (one test point per row, as save_kernel.py stores Kxvx / Kxtx), kz_diag: [m]
    prior variances (the Kv_diag / Kt_diag datasets, save_kernel.py:33-36, computed with
    ``model(z, z, True, True)``).  One rocBLAS dtrsm_64 (V = U⁻ᵀ Kxz, in place) and a
    row sum of squares, through cgp_pred_var_f64.  Kxz is overwritten with V only when it
    is a contiguous float64 device tensor and ``overwrite_kxz``.  SURVEY.md §8f row 4;
    the reference's classify_gp.py stops at the posterior mean (:39-42).
    """
    dev = Kfactor.device if Kfactor.device.type == "cuda" else _device()
    n = Kfactor.shape[0]
    assert Kfactor.dtype == torch.float64 and Kfactor.dim() == 2 and Kfactor.shape[1] == n
    assert Kfactor.device == dev and Kfactor.is_contiguous(), "Kfactor: the device factor"
    assert Kxz.dim() == 2 and Kxz.shape[1] == n, (Kxz.shape, n)
    m = Kxz.shape[0]
    with torch.cuda.device(dev):
        if (overwrite_kxz and Kxz.device == dev and Kxz.dtype == torch.float64
                and Kxz.is_contiguous()):
            V = Kxz
        else:
            V = Kxz.to(dev, dtype=torch.float64).clone(memory_format=torch.contiguous_format)
        d = torch.as_tensor(kz_diag).to(dev, dtype=torch.float64).reshape(m).contiguous()
        var = torch.empty((m,), dtype=torch.float64, device=dev)
        N.call("cgp_pred_var_f64", N.ptr(Kfactor), n, n, N.ptr(V), m, n, N.ptr(d), N.ptr(var),
               _stream(dev))
    return var


def diag_add(K, diag):
    """K[i, i] += diag in place (classify_gp.py:30-36)."""
    if isinstance(K, torch.Tensor):
        K.view(K.numel())[::K.shape[-1] + 1] += diag
    elif isinstance(K, np.ndarray):
        K.flat[::K.shape[-1] + 1] += diag
    else:
        raise TypeError("What do I do with a `{}`, K={}?".format(type(K), K))


def load_kern(dset, i, device=None):
    """dataset[i] (float32) -> float64 tensor (classify_gp.py:45-48); widened on the
    device when ``device`` is a cuda device."""
    A = np.empty(dset.shape[1:], dtype=np.float32)
    if hasattr(dset, "read_direct"):
        dset.read_direct(A, source_sel=np.s_[i, :, :])
    else:
        A[...] = np.asarray(dset[i])
    t = torch.from_numpy(A)
    if device is None or torch.device(device).type != "cuda":
        return t.to(dtype=torch.float64)
    dev = torch.device(device)
    with torch.cuda.device(dev):
        src = t.to(dev)
        out = torch.empty(src.shape, dtype=torch.float64, device=dev)
        N.call("cgp_cast_f32_f64", N.ptr(src), N.ptr(out), src.numel(), _stream(dev))
    return out


def cast_into(src, dst):
    """dst (float64) ← src (float32), same shape, both contiguous on one device, through
    cgp_cast_f32_f64 (classify_gp.py:45-48's widening of the stored float32 K); the two
    ranges must not overlap (pipeline.widen_in_place guarantees it)."""
    if src.dtype != torch.float32 or dst.dtype != torch.float64 or \
            src.shape != dst.shape or src.device != dst.device or \
            not (src.is_contiguous() and dst.is_contiguous()):
        raise ValueError("cast_into: contiguous float32 src and float64 dst of one shape "
                         "on one device")
    with torch.cuda.device(dst.device):
        N.call("cgp_cast_f32_f64", N.ptr(src), N.ptr(dst), src.numel(), _stream(dst.device))
    return dst


def scores(Kxz, A):
    """Kxz @ A, the class scores of classify_gp.py:39-40, on the device (rocBLAS dgemm
    through cgp_gemm_f64): [m, n] @ [n, classes] -> [m, classes] float64."""
    dev = Kxz.device if Kxz.device.type == "cuda" else _device()
    with torch.cuda.device(dev):
        K = Kxz.to(dev, dtype=torch.float64).contiguous()
        Ad = A.to(dev, dtype=torch.float64).reshape(K.shape[1], -1).contiguous()
        m, kdim = K.shape
        ncls = Ad.shape[1]
        out = torch.empty((m, ncls), dtype=torch.float64, device=dev)
        if m:
            N.call("cgp_gemm_f64", N.ptr(K), N.ptr(Ad), N.ptr(out), m, ncls, kdim, _stream(dev))
    return out


def predict(A, Kxz):
    """argmax over classes of Kxz @ A (classify_gp.py:39-40), on the device."""
    sc = scores(Kxz, A)
    m, ncls = sc.shape
    with torch.cuda.device(sc.device):
        pred = torch.empty((m,), dtype=torch.int64, device=sc.device)
        if m:
            N.call("cgp_argmax_rows_f64", N.ptr(sc), m, ncls, N.ptr(pred), _stream(sc.device))
    return pred


def accuracy(pred, Y) -> float:
    Yt = torch.as_tensor(Y).reshape(-1).cpu()
    return float((pred.cpu() == Yt).double().mean())


def print_accuracy(A, Kxvx, Y, key):
    acc = accuracy(predict(A, Kxvx), Y)
    print(f"{key} accuracy: {acc*100}%")
    return acc


def one_hot_pm1(labels, n_classes=None):
    """Y_1hot of classify_gp.py:56-59: -1 everywhere, +1 at each label, float64."""
    labels = torch.as_tensor(labels)
    n_classes = int(labels.max()) + 1 if n_classes is None else n_classes
    Y = torch.ones((len(labels), n_classes), dtype=torch.float64).neg_()
    Y[torch.arange(len(labels)), labels] = 1.
    return Y
