"""Oracle parity of the full-scale bound builds at their real sizes (BASELINE configs[3]
and configs[4]).

tools/fullscale.py → cnn_gp.pipeline.classify_distributed → gram.gram_strip evaluates a
rank's Kxx strip [r0, r1) from ONE bind of the images it reads (X[r0:]:
ModelKern.bind → NNGPKernel.image_variances, one var-chain launch over the set) and every
B = 4096 tile from row slices of those maps.  tests/test_gpu_fullgeom.py pins the tile
geometry against the oracle with 8 192 images; this test pins the slicing at the far end
of the full-size binds, where the slice offsets are largest:

* mnist_as_tf, N = 60 000 (configs[3]), fp64 kernels;
* cifar10, N = 50 000 images of 3×32×32 (configs[4]), fp64 kernels;
* mnist_as_tf, N = 60 000 with float32 kernels (the reference pipeline's own precision,
  exp_mnist_resnet/save_kernel.py:19-24; the bench's ``fullscale_f32`` leg) against the
  fp64 oracle on the same float32-rounded images.

Each case binds all N images and evaluates, through gram_strip with global offsets,

* the last diagonal tile, rows N − 4096 … N (image N − 1 included);
* a 4096-row Kxz block: the same rows against a second bound set of 4 096 images.

Sampled entries (≥ 34 per block, among them the last image and the diagonal K[N−1, N−1])
are checked against ``oracle.kernel`` (reference kernels.py:18-57, one pair at a time) —
1e-8 in fp64 (the closed-form ReLU's bound, test_gpu_fullgeom.py), 1e-5 in fp32 (the north
star's) — and against the drop-in's per-tile call ``model(x_i, x_j, False, False)`` on
single images in the same (i, j) orientation for bit equality.  The multi-rank pipeline's
own form — a rank whose strip starts at r0 binds only X[r0:] and evaluates the strip in
local coordinates (gram_strip(kern, row_slice(X, r0, N), None, B, (0, N − r0))) — is
checked bit-equal to the global-offset strip on the same tile.

Inputs are tools/fullscale.py's own MNIST-/CIFAR-like generator (k/255, ~60% zeros,
4-pixel zero border; seeds 0 and 1), the images the bench's full-scale legs build from.
"""
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
B = 4096
CASES = [("mnist_as_tf", 60000, "f64", 1e-8), ("cifar10", 50000, "f64", 1e-8),
         ("mnist_as_tf", 60000, "f32", 1e-5)]


def _fullscale_images(cfg, n):
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(
        os.path.abspath(__file__))), "tools"))
    from fullscale import mnist_like
    C, side = specs.GEOMETRY[cfg]
    return mnist_like(n, C, side, 0), mnist_like(B, C, side, 1)


@pytest.mark.parametrize("cfg,N,dt,rtol", CASES, ids=[f"{c}-{n}-{d}" for c, n, d, _ in CASES])
def test_bound_build_tail_vs_oracle(cfg, N, dt, rtol):
    from cnn_gp import gram
    tdt = torch.float64 if dt == "f64" else torch.float32
    R0 = N - B
    spec = specs.CONFIGS[cfg]()
    X, Z = _fullscale_images(cfg, N)
    m = configs_util.model(cfg).to(DEV, tdt)
    Xd, Zd = X.to(DEV, tdt), Z.to(DEV, tdt)
    kern = gram.model_kern(m)
    bound = kern.bind(Xd)
    assert bound is not None and len(bound.vx) == N, f"the {N}-image bind fell back"
    del bound
    with torch.no_grad():
        Kxx, tiles, _ = gram.gram_strip(kern, Xd, None, B, (R0, N), dtype=tdt)
        Kxz, tz, _ = gram.gram_strip(kern, Xd, Zd, B, (R0, N), dtype=tdt)
        # the pipeline's own form: this rank binds only X[R0:] and works in local rows
        Kloc, tl, _ = gram.gram_strip(kern, gram.row_slice(Xd, R0, N), None, B, (0, N - R0),
                                      dtype=tdt)
    assert tiles == [(True, R0, R0, B, B)] and tz == [(False, R0, 0, B, B)]
    assert tl == [(True, 0, 0, B, B)]
    Kd = Kxx[:, R0:].double().cpu().numpy()                # the diagonal tile, local indices
    Ko = Kxz.double().cpu().numpy()
    assert np.array_equal(Kloc.double().cpu().numpy(), Kd), \
        "X[r0:] bound in local rows differs from the global-offset strip"
    assert np.isfinite(Kd).all() and np.isfinite(Ko).all()
    assert np.array_equal(Kd, Kd.T)
    # what the GPU sees (float32 rounding of the k/255 pixels in the f32 case)
    Xh = Xd.double().cpu().numpy()
    Zh = Zd.double().cpu().numpy()
    rng = np.random.default_rng(11)
    last = B - 1                                        # image N − 1
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
        with torch.no_grad():
            if name == "xx" and i == j:
                ref = O.kernel(spec, Xh[gi:gi + 1])[0, 0]
                got = Kd[i, i]
                hip = m(Xd[gi:gi + 1]).item()
            elif name == "xx":
                gj = R0 + j
                ref = O.kernel(spec, Xh[gi:gi + 1], Xh[gj:gj + 1], False, False)[0, 0]
                got = Kd[i, j]
                hip = m(Xd[gi:gi + 1], Xd[gj:gj + 1], False, False).item()
            else:
                ref = O.kernel(spec, Xh[gi:gi + 1], Zh[j:j + 1], False, False)[0, 0]
                got = Ko[i, j]
                hip = m(Xd[gi:gi + 1], Zd[j:j + 1], False, False).item()
        err = abs(got - ref) / abs(ref)
        worst = max(worst, err)
        worst_hip = max(worst_hip, abs(got - hip) / abs(hip))
        assert err < rtol, (cfg, dt, name, gi, j, got, ref, err)
        assert got == hip, ("bound build vs per-tile forward", name, gi, j, got, hip)
    assert len(pick) >= 64
    print(f"{cfg} {dt} {N}-image bound build, rows {R0}-{N}: {len(pick)} entries vs oracle, "
          f"worst rel err {worst:.2e} (bound {rtol:g}); single-pair forwards and the "
          f"X[r0:] local strip bit-equal")
