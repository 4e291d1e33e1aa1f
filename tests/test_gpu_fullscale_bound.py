"""Oracle parity of the full-scale bound build at its real size (BASELINE configs[3]).

The full-scale pipeline (tools/fullscale.py → cnn_gp.pipeline.classify_distributed →
gram.gram_strip) binds ALL 60 000 training images once (ModelKern.bind →
NNGPKernel.image_variances: one var-chain launch over the whole set) and evaluates every
B = 4096 tile from row slices [i0:i1] of those maps.  tests/test_gpu_fullgeom.py pins the
tile geometry against the oracle with 8 192 images; this test pins the slicing at the far
end of the 60 000-image bind, where the slice offsets are largest:

* the last diagonal tile, rows 55 904-60 000 (gram_strip over Kxx rows [55 904, 60 000));
* a 4096-row Kxz block, rows 55 904-60 000 of the bound 60 000 against a second bound set
  of 4 096 images (gram_strip(kern, X, X2)), i.e. the x-side maps sliced at 55 904 and the
  y-side maps at 0.

Inputs are tools/fullscale.py's own MNIST-like generator (k/255, ~60% zeros, 4-pixel
zero border; seed 0), the same 60 000 images the bench's `fullscale` leg builds from.
Sampled entries (≥ 32 per block, among them the last image 59 999 and the diagonal
K[59 999, 59 999]) are checked against ``oracle.kernel`` (reference kernels.py:18-57, one
pair at a time) at the closed-form ReLU's 1e-8 (test_gpu_fullgeom.py's bound), and against
the drop-in's per-tile call — ``model(x_i, x_j, False, False)`` on single images in the
same (i, j) orientation — for bit equality: the bound build evaluates exactly what a
forward per tile evaluates (gram.py ModelKern.bind)."""
import os
import sys

import numpy as np
import pytest
import torch

from oracle import nngp_oracle as O
from oracle import specs

import configs_util

pytestmark = pytest.mark.gpu

DEV = "cuda"
N, B = 60000, 4096
R0 = N - B                     # 55 904
RTOL = 1e-8


def _fullscale_images():
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(
        os.path.abspath(__file__))), "tools"))
    from fullscale import mnist_like
    return mnist_like(N, 1, 28, 0), mnist_like(B, 1, 28, 1)


def test_bound_build_60k_tail_vs_oracle():
    from cnn_gp import gram
    spec = specs.mnist_as_tf()
    X, Z = _fullscale_images()
    m = configs_util.model("mnist_as_tf").to(DEV, torch.float64)
    Xd, Zd = X.to(DEV), Z.to(DEV)
    kern = gram.model_kern(m)
    bound = kern.bind(Xd)
    assert bound is not None and len(bound.vx) == N, "the 60 000-image bind fell back"
    del bound
    with torch.no_grad():
        Kxx, tiles, _ = gram.gram_strip(kern, Xd, None, B, (R0, N))
        Kxz, tz, _ = gram.gram_strip(kern, Xd, Zd, B, (R0, N))
    assert tiles == [(True, R0, R0, B, B)] and tz == [(False, R0, 0, B, B)]
    Kd = Kxx[:, R0:].cpu().numpy()                    # the diagonal tile, local indices
    Ko = Kxz.cpu().numpy()
    assert np.isfinite(Kd).all() and np.isfinite(Ko).all()
    assert np.array_equal(Kd, Kd.T)
    Xh, Zh = X.numpy(), Z.numpy()
    rng = np.random.default_rng(11)
    last = B - 1                                        # image 59 999
    pick = [("xx", last, last), ("xx", last - 1, last), ("xx", 0, last), ("xx", 0, 0),
            ("xx", 95, 96), ("xz", last, 0), ("xz", last, B - 1), ("xz", 0, 0),
            ("xz", 96, 4095), ("xz", last - 7, 8)]
    while sum(p[0] == "xx" for p in pick) < 34:
        i, j = sorted(int(v) for v in rng.integers(0, B, 2))
        pick.append(("xx", i, j))
    while sum(p[0] == "xz" for p in pick) < 34:
        pick.append(("xz", int(rng.integers(96, B)), int(rng.integers(0, B))))
    worst, worst_hip = 0.0, 0.0
    for name, i, j in pick:
        gi = R0 + i
        if name == "xx" and i == j:
            ref = O.kernel(spec, Xh[gi:gi + 1])[0, 0]
            got = Kd[i, i]
            with torch.no_grad():
                hip = m(Xd[gi:gi + 1]).item()
        elif name == "xx":
            gj = R0 + j
            ref = O.kernel(spec, Xh[gi:gi + 1], Xh[gj:gj + 1], False, False)[0, 0]
            got = Kd[i, j]
            with torch.no_grad():
                hip = m(Xd[gi:gi + 1], Xd[gj:gj + 1], False, False).item()
        else:
            ref = O.kernel(spec, Xh[gi:gi + 1], Zh[j:j + 1], False, False)[0, 0]
            got = Ko[i, j]
            with torch.no_grad():
                hip = m(Xd[gi:gi + 1], Zd[j:j + 1], False, False).item()
        err = abs(got - ref) / abs(ref)
        worst = max(worst, err)
        worst_hip = max(worst_hip, abs(got - hip) / abs(hip))
        assert err < RTOL, (name, gi, j, got, ref, err)
        assert got == hip, ("bound build vs per-tile forward", name, gi, j, got, hip)
    assert len(pick) >= 64
    print(f"60k bound build, rows {R0}-{N}: {len(pick)} entries vs oracle, worst rel err "
          f"{worst:.2e}; vs single-pair forwards: bit-equal (max {worst_hip:.1e})")
