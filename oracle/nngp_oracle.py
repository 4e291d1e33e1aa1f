"""CPU oracle for the CNN-GP hot path — TEST INFRASTRUCTURE ONLY.

This module is a plain-numpy restatement of the reference's NNGP kernel recursion
(/root/reference/cnn_gp/kernels.py, kernel_patch.py) and of the GP solve
(/root/reference/exp_mnist_resnet/classify_gp.py).  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import it, and
only as the checker / the timed CPU baseline — the product path (``cnn-gp_amd/cnn_gp``)
never imports, calls or falls back to it.

Parity pin: the restatement is checked against golden vectors produced by running the
reference itself in the build container (``tests/golden/make_golden.py`` →
``tests/golden/*.npz``; test ``tests/test_oracle_golden.py``).

Architectures are described by a small nested *spec* (tuples), independent of the
product's module classes:

    ("conv", dict(kernel_size=k, stride=1, padding="same", dilation=1,
                  var_weight=1.0, var_bias=0.0))
    ("relu",)
    ("seq", [spec, ...])
    ("sum", [spec, ...])
    ("mix", [spec, ...], logits)        # Mixture, logits as a list of floats

Weight convention (kernels.py:82-88): the reference stores the constant conv weight
var_weight/k² in a float32 buffer (torch's default dtype) and upcasts it with
``model.double()``.  ``weights="f32"`` (default) reproduces that; ``weights="exact"``
uses the float64 value (reference run under ``torch.set_default_dtype(float64)``).
"""
from __future__ import annotations

import math

import numpy as np

F32_TINY = float(np.finfo(np.float32).tiny)   # kernels.py:133


# ------------------------------------------------------------------------------------
# Conv2d (kernels.py:60-98)
# ------------------------------------------------------------------------------------
def conv_geometry(p: dict) -> dict:
    """Padding / kernel extent / tap offsets of Conv2d.__init__ (kernels.py:61-88)."""
    k = int(p["kernel_size"])
    d = int(p.get("dilation", 1))
    s = int(p.get("stride", 1))
    padding = p.get("padding", "same")
    zero_row = False
    if padding == "same":                              # :71-74
        pad = d * (k // 2)
        zero_row = k % 2 == 0
    else:
        pad = int(padding)
    keff = k + 1 if zero_row else k                    # :78-86
    taps = list(range(1, keff)) if zero_row else list(range(keff))
    return dict(k=k, d=d, s=s, pad=pad, keff=keff, taps=taps, zero_row=zero_row)


def conv_weight(p: dict, dtype, weights: str = "f32"):
    """The constant kernel value var_weight / k² (kernels.py:87-88)."""
    k = int(p["kernel_size"])
    val = float(p.get("var_weight", 1.0)) / k ** 2
    if weights == "f32":
        val = float(np.float32(val))   # t.ones(...) * (var_weight / k**2) in float32
    return np.asarray(val, dtype=dtype)


def conv_out_size(n: int, g: dict) -> int:
    return (n + 2 * g["pad"] - g["d"] * (g["keff"] - 1) - 1) // g["s"] + 1


def conv_maps(maps: np.ndarray, p: dict, weights: str = "f32") -> np.ndarray:
    """F.conv2d(maps[:,None], kernel, stride, padding, dilation) + var_bias.

    maps: [P, H, W] -> [P, Ho, Wo] (kernels.py:92-98).  Direct k×k tap sum, each tap
    weighted, zero padding.
    """
    dt = maps.dtype
    g = conv_geometry(p)
    P, H, W = maps.shape
    Ho, Wo = conv_out_size(H, g), conv_out_size(W, g)
    if Ho <= 0 or Wo <= 0:
        raise ValueError("conv output would be empty")
    pad = g["pad"]
    padded = np.zeros((P, H + 2 * pad, W + 2 * pad), dtype=dt)
    padded[:, pad:pad + H, pad:pad + W] = maps
    w = conv_weight(p, dt, weights)
    b = np.asarray(float(p.get("var_bias", 0.0)), dtype=dt)
    s, d = g["s"], g["d"]
    out = np.zeros((P, Ho, Wo), dtype=dt)
    for a in g["taps"]:
        for c in g["taps"]:
            out += w * padded[:, a * d:a * d + s * (Ho - 1) + 1:s, c * d:c * d + s * (Wo - 1) + 1:s]
    return out + b


# ------------------------------------------------------------------------------------
# KernelPatch state (kernel_patch.py:4-89) as a plain dict of arrays
# ------------------------------------------------------------------------------------
def make_kp(same, diag, xy, xx, yy):
    return dict(same=bool(same), diag=bool(diag), xy=xy, xx=xx, yy=yy)


def moments(x: np.ndarray, y: np.ndarray, same: bool, diag: bool):
    """NNGPKernel.forward moments (kernels.py:44-51).  x [N1,C,H,W], y [N2,C,H,W]."""
    C = x.shape[1]
    if diag:
        xy = (x * y).sum(1) / x.dtype.type(C)
    else:
        n1, n2 = x.shape[0], y.shape[0]
        xy = (x[:, None] * y[None]).sum(2).reshape(n1 * n2, *x.shape[2:]) / x.dtype.type(C)
    xx = (x * x).sum(1) / x.dtype.type(C)
    yy = (y * y).sum(1) / x.dtype.type(C)
    return make_kp(same, diag, xy, xx, yy)


def relu(kp: dict) -> dict:
    """ReLU.propagate (kernels.py:134-165)."""
    dt = kp["xy"].dtype.type
    xx, yy, xy = kp["xx"], kp["yy"], kp["xy"]
    n1, n2 = xx.shape[0], yy.shape[0]
    if kp["diag"]:
        v1, v2, c = xx, yy, xy
    else:
        H, W = xy.shape[-2:]
        c = xy.reshape(n1, n2, H, W)
        v1, v2 = xx[:, None], yy[None]
    with np.errstate(invalid="ignore", divide="ignore", over="ignore"):
        t = v1 * v2 + dt(F32_TINY)
        cos = np.clip(c * (dt(1) / np.sqrt(t)), dt(-1), dt(1))
        sin = np.sqrt(np.maximum(t - c * c, dt(0)))
        theta = np.arccos(cos)
        out = (sin + (dt(math.pi) - theta) * c) / dt(2 * math.pi)
    xx2 = xx / dt(2)
    if kp["same"]:
        yy2 = xx2
        if kp["diag"]:
            out = xx2
        else:
            out = out.copy()
            idx = np.arange(n1)
            out[idx, idx] = xx2
    else:
        yy2 = yy / dt(2)
    if not kp["diag"]:
        out = out.reshape(n1 * n2, *out.shape[2:])
    return make_kp(kp["same"], kp["diag"], out, xx2, yy2)


def _conv_kp(kp: dict, p: dict, weights: str) -> dict:
    return make_kp(kp["same"], kp["diag"], conv_maps(kp["xy"], p, weights),
                   conv_maps(kp["xx"], p, weights), conv_maps(kp["yy"], p, weights))


def _axpby(terms, kp0):
    xy = xx = yy = None
    for coef, kp in terms:
        a = (kp["xy"] * coef, kp["xx"] * coef, kp["yy"] * coef) if coef is not None else (
            kp["xy"], kp["xx"], kp["yy"])
        if xy is None:
            xy, xx, yy = a
        else:
            xy, xx, yy = xy + a[0], xx + a[1], yy + a[2]
    return make_kp(kp0["same"], kp0["diag"], xy, xx, yy)


def softmax(logits, weights: str, dt):
    """F.softmax(self.logit, dim=0) of Mixture.propagate (kernels.py:221).  The logit
    Parameter is created in torch's default dtype (float32 under weights="f32") and cast
    with the model (``.double()``), so the softmax runs in the model's dtype on the
    float32-rounded logits.  ATen's CPU softmax scales exp(x - max) by 1/Σ."""
    lg = np.asarray(logits, dtype=np.float32 if weights == "f32" else np.float64).astype(dt)
    e = np.exp(lg - lg.max())
    return e * (dt(1) / e.sum())


def propagate(spec, kp: dict, weights: str = "f32") -> dict:
    kind = spec[0]
    if kind == "conv":
        return _conv_kp(kp, spec[1], weights)
    if kind == "relu":
        return relu(kp)
    if kind == "seq":                                  # kernels.py:184-187
        for m in spec[1]:
            kp = propagate(m, kp, weights)
        return kp
    if kind == "sum":                                  # kernels.py:252-254
        outs = [propagate(m, kp, weights) for m in spec[1]]
        return _axpby([(None, o) for o in outs], kp)
    if kind == "mix":                                  # kernels.py:220-225
        dt = kp["xy"].dtype.type
        pr = softmax(spec[2], weights, dt)
        outs = [propagate(m, kp, weights) for m in spec[1]]
        return _axpby([(dt(pr[i]), o) for i, o in enumerate(outs)], kp)
    raise ValueError(f"unknown spec kind {kind!r}")


def kernel(spec, x: np.ndarray, y: np.ndarray | None = None, same=None, diag=False,
           weights: str = "f32") -> np.ndarray:
    """NNGPKernel.forward (kernels.py:18-57): [N1,C,H,W] × [N2,C,H,W] -> [N1,N2] / [N1]."""
    if y is None:
        assert same is None
        y, same = x, True
    assert x.ndim == 4 and y.ndim == 4 and x.shape[1:] == y.shape[1:]
    assert not diag or len(x) == len(y)
    kp = propagate(spec, moments(x, y, bool(same), diag), weights)
    r = kp["xy"]
    if r.shape[-2:] != (1, 1):
        raise ValueError(f"final spatial size {r.shape[-2:]} is not 1x1")
    return r.reshape(len(x)) if diag else r.reshape(len(x), len(y))


# ------------------------------------------------------------------------------------
# tile schedule + worker split (cnn_gp/data.py:11-96) and save_K (kernel_save_tools.py)
# ------------------------------------------------------------------------------------
def worker_slice(n_batches: int, worker_rank: int, n_workers: int):
    """_this_worker_batch (data.py:11-19): contiguous, balanced, first ranks get +1."""
    per = [n_batches // n_workers] * n_workers
    for r in range(n_batches % n_workers):
        per[r] += 1
    return sum(per[:worker_rank]), per[worker_rank]


def tile_schedule(n_x: int, n_x2: int | None, batch_size: int, worker_rank=0, n_workers=1):
    """ProductIterator order (data.py:22-60): list of (same, i0, j0) element offsets."""
    bx = -(-n_x // batch_size)
    if n_x2 is None:
        same = True
        bx2 = bx
        n_batches = max(1, bx * (bx + 1) // 2)
    else:
        same = False
        bx2 = -(-n_x2 // batch_size)
        n_batches = bx * bx2
    order = []
    for i in range(bx):
        if same:
            order.append((True, i, i))
        for j in range(i + 1 if same else 0, bx2):
            order.append((False, i, j))
    start, count = worker_slice(n_batches, worker_rank, n_workers)
    return [(s, i * batch_size, j * batch_size) for s, i, j in order[start:start + count]]


def gram_tiles(spec, X: np.ndarray, X2: np.ndarray | None, batch_size: int, worker_rank=0,
               n_workers=1, weights="f32") -> np.ndarray:
    """save_K's non-diag loop into a NaN-filled float32 (1,N,N2) array (kernel_save_tools.py:26-58)."""
    N = len(X)
    N2 = N if X2 is None else len(X2)
    out = np.full((1, N, N2), np.nan, dtype=np.float32)
    src2 = X if X2 is None else X2
    for same, i, j in tile_schedule(N, None if X2 is None else N2, batch_size, worker_rank,
                                    n_workers):
        x = X[i:i + batch_size]
        x2 = src2[j:j + batch_size]
        out[0, i:i + len(x), j:j + len(x2)] = kernel(spec, x, x2, same, False, weights)
    return out


# ------------------------------------------------------------------------------------
# GP solve (classify_gp.py:17-42)
# ------------------------------------------------------------------------------------
def solve_upper(K: np.ndarray, Y: np.ndarray, jitter: float = 0.0) -> np.ndarray:
    """scipy.linalg.solve(K + jitter·I, Y, assume_a='pos', lower=False): only the upper
    triangle of K is read (classify_gp.py:24-26)."""
    import scipy.linalg
    A = np.array(K, dtype=np.float64, copy=True)
    A.flat[::A.shape[-1] + 1] += jitter
    return scipy.linalg.solve(A, np.asarray(Y, dtype=np.float64), assume_a="pos", lower=False,
                              check_finite=False)


def one_hot_pm1(labels: np.ndarray, n_classes: int | None = None) -> np.ndarray:
    """classify_gp.py:56-59: -1 everywhere, +1 at the label."""
    n_classes = int(labels.max()) + 1 if n_classes is None else n_classes
    Y = -np.ones((len(labels), n_classes), dtype=np.float64)
    Y[np.arange(len(labels)), labels] = 1.0
    return Y
