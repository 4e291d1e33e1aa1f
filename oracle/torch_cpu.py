"""Multi-threaded torch-CPU restatement of the NNGP kernel recursion — TEST / BASELINE
INFRASTRUCTURE ONLY (same import rule as oracle/nngp_oracle.py: only ``tests/`` and
``bench.py``'s ``cpu_baseline`` leg use it, as the timed CPU baseline; the product path
never imports it).

SURVEY.md §8(d) prescribes the CPU baseline: the build's own torch-CPU restatement of the
reference's op sequence, on all the host cores it is given, calibrated against the
reference itself at C1 (tools/calibrate_cpu.py → profiles/r2/cpu_calibration.json).  It
runs the same torch CPU kernels the reference runs — F.conv2d of a constant k×k kernel per
layer plus the bias add (kernels.py:92-98), the ReLU map as torch pointwise ops
(kernels.py:134-165), sums and mixtures (kernels.py:220-254) — driven by the oracle's
spec walker (oracle/specs.py), so its speed is the reference's speed on the same cores.
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

from .nngp_oracle import conv_geometry, conv_weight

F32_TINY = 1.1754943508222875e-38       # torch.finfo(torch.float32).tiny, kernels.py:133


def _kernel_tensor(p, dtype):
    """The constant conv kernel of Conv2d.__init__ (kernels.py:73-88): value
    var_weight/k² rounded to float32, an extra zero row and column for even k."""
    g = conv_geometry(p)
    w = torch.full((1, 1, g["keff"], g["keff"]), float(conv_weight(p, "float64")),
                   dtype=dtype)
    if g["zero_row"]:
        w[:, :, 0, :] = 0
        w[:, :, :, 0] = 0
    return w, g


def _conv(t, p):
    w, g = _kernel_tensor(p, t.dtype)
    return F.conv2d(t, w, stride=g["s"], padding=g["pad"], dilation=g["d"]) + \
        float(p.get("var_bias", 0.0))


def _relu(kp):
    same, diag, xy, xx, yy = kp
    n1 = xx.shape[0]
    if diag:
        v1, v2, c = xx, yy, xy
    else:
        n2 = yy.shape[0]
        c = xy.view(n1, n2, *xy.shape[-2:])
        v1, v2 = xx.view(n1, 1, *xx.shape[-2:]), yy.view(1, n2, *yy.shape[-2:])
    t = v1 * v2 + F32_TINY
    cos = (c * torch.rsqrt(t)).clamp(-1, 1)
    sin = (t - c * c).clamp(min=0).sqrt()
    theta = torch.acos(cos)
    out = (sin + (math.pi - theta) * c) / (2 * math.pi)
    xx2 = xx / 2
    if same:
        yy2 = xx2
        if diag:
            out = xx2
        else:
            idx = torch.arange(n1)
            out[idx, idx] = xx2.view(n1, *xx2.shape[-2:])
    else:
        yy2 = yy / 2
    if not diag:
        out = out.view(-1, 1, *out.shape[-2:])
    return (same, diag, out, xx2, yy2)


def _axpy(terms):
    acc = None
    for coef, kp in terms:
        xy, xx, yy = kp[2:]
        if coef is not None:
            xy, xx, yy = xy * coef, xx * coef, yy * coef
        acc = (xy, xx, yy) if acc is None else (acc[0] + xy, acc[1] + xx, acc[2] + yy)
    return (terms[0][1][0], terms[0][1][1]) + acc


def _propagate(spec, kp):
    kind = spec[0]
    if kind == "conv":
        return kp[:2] + tuple(_conv(t, spec[1]) for t in kp[2:])
    if kind == "relu":
        return _relu(kp)
    if kind == "seq":
        for m in spec[1]:
            kp = _propagate(m, kp)
        return kp
    if kind == "sum":
        return _axpy([(None, _propagate(m, kp)) for m in spec[1]])
    if kind == "mix":
        lg = torch.tensor(spec[2], dtype=torch.float32).to(kp[2].dtype)
        pr = torch.softmax(lg, dim=0)
        return _axpy([(pr[i], _propagate(m, kp)) for i, m in enumerate(spec[1])])
    raise ValueError(kind)


@torch.no_grad()
def kernel(spec, x: torch.Tensor, y: torch.Tensor | None = None, same=None, diag=False):
    """[N1,C,H,W] × [N2,C,H,W] CPU tensors -> [N1,N2] (or [N1] when diag)."""
    if y is None:
        y, same = x, True
    n1, n2 = x.shape[0], y.shape[0]
    C = x.shape[1]
    if diag:
        xy = (x * y).mean(1, keepdim=True)
    else:
        xy = (x[:, None] * y[None]).mean(2).view(n1 * n2, 1, *x.shape[2:])
    xx = (x * x).mean(1, keepdim=True)
    yy = (y * y).mean(1, keepdim=True)
    _ = C
    kp = _propagate(spec, (bool(same), bool(diag), xy, xx, yy))
    r = kp[2]
    return r.view(n1) if diag else r.view(n1, n2)
