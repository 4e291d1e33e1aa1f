"""Parity at the full-scale tile geometry (BASELINE configs[3] / [4]: tools/fullscale.py
and bench.py's full-scale legs run B = 4096 tiles with the production state chunking).

For mnist_as_tf and cifar10, one diagonal 4096² tile (same=True) and one 4096 × 4096
off-diagonal tile are evaluated exactly as the full-scale pipeline evaluates them — the
default ``netplan.CHUNK_BYTES`` (no monkeypatch), so the staged ResNet programs run in
several launch groups per tile with state-buffer offsets past 2³² bytes — and sampled
entries are checked against ``oracle.kernel`` (one pair at a time):

* the pair units on both sides of every production chunk boundary (u = k·chunk − 1 and
  k·chunk, decoded through the supertile walk), for both tiles;
* tile corners and supertile seams, random interior pairs;
* diagonal entries K[i, i] (the variance chain's final value);
* images alternate uniform / MNIST-like (4-pixel zero border, ~60% zero pixels, k/255:
  the f32_tiny path of zero-variance pixels).

Tolerances: float64 1e-8 with the closed-form ReLU, 1e-10 with the op-by-op ReLU
(set_exact_relu; one-stage program); float32 kernels against the float64 oracle on the
same float32-rounded images at the north star's 1e-5 (the reference's own production
precision, exp_mnist_resnet/save_kernel.py:19-24)."""
import numpy as np
import pytest
import torch

from oracle import nngp_oracle as O
from oracle import specs

import configs_util
from test_gpu_scale import _images, _samples

pytestmark = pytest.mark.gpu

DEV = "cuda"
B = 4096
RTOL = {("f64", "fast"): 1e-8, ("f64", "exact"): 1e-10, ("f32", "fast"): 1e-5}
_IMAGES = {}


def _data(cfg):
    if cfg not in _IMAGES:
        C, side = specs.GEOMETRY[cfg]
        _IMAGES[cfg] = _images(2 * B, C, side, 57)
    return _IMAGES[cfg]


@pytest.mark.parametrize("cfg", ["mnist_as_tf", "cifar10"])
@pytest.mark.parametrize("dt,numerics", [("f64", "fast"), ("f32", "fast"), ("f64", "exact")])
def test_full_scale_tiles_vs_oracle(cfg, dt, numerics):
    from cnn_gp import _native as Nat
    from cnn_gp.netplan import NetPlan
    tdt = torch.float64 if dt == "f64" else torch.float32
    item = 8 if dt == "f64" else 4
    C, side = specs.GEOMETRY[cfg]
    spec = specs.CONFIGS[cfg]()
    X = _data(cfg)
    Xr = X.astype(np.float32).astype(np.float64) if dt == "f32" else X   # what the GPU sees
    m = configs_util.model(cfg).to(DEV, tdt).set_exact_relu(numerics == "exact")
    net = m._net_plan(m._plan(side, side), item)
    assert net is not None
    st = Nat.load().cgp_net_supertile()
    Xd = torch.from_numpy(X).to(DEV, tdt)
    chunks = {}
    for same in (True, False):
        units = NetPlan.units(B, B, same)
        if len(net.stages) > 1:
            chunk = net.chunk_units(item, units, Xd.device)
            assert chunk < units, "the production chunking must cut this tile"
            stride_b = max(s.load_stride for s in net.stages[1:])
            if dt == "f64":
                assert chunk * stride_b * item > 1 << 32, "state offsets stay below 4 GB"
            chunks[same] = chunk
        else:
            assert numerics == "exact"               # the op-by-op ReLU runs one stage
            chunks[same] = None
    with torch.no_grad():
        Kd = m(Xd[:B]).double().cpu().numpy()                              # tile (0, 0)
        Ko = m(Xd[:B], Xd[B:], False, False).double().cpu().numpy()        # tile (0, 1)
    assert np.isfinite(Kd).all() and np.isfinite(Ko).all()
    assert np.array_equal(Kd, Kd.T)            # the kernel mirrors K[j, i] = K[i, j]
    rng = np.random.default_rng(3)
    pick = []                                   # (tile, i, j) local to the tile
    for same, K in ((True, Kd), (False, Ko)):
        ch = chunks[same] or 1 << 62
        for i, j in _samples(rng, ch, st, B, B, B, same, 32):
            pick.append((same, i, j))
    pick += [(True, k, k) for k in (0, 1, 2047, 4095)]
    tol = RTOL[(dt, numerics)]
    worst = 0.0
    for same, i, j in pick:
        if same and i == j:
            ref = O.kernel(spec, Xr[i:i + 1])[0, 0]
            got = Kd[i, i]
        elif same:
            lo, hi = min(i, j), max(i, j)
            ref = O.kernel(spec, Xr[lo:lo + 1], Xr[hi:hi + 1], False, False)[0, 0]
            got = Kd[lo, hi]
        else:
            ref = O.kernel(spec, Xr[i:i + 1], Xr[B + j:B + j + 1], False, False)[0, 0]
            got = Ko[i, j]
        err = abs(got - ref) / abs(ref)
        worst = max(worst, err)
        assert err < tol, (cfg, dt, numerics, same, i, j, got, ref, err)
    n_bounds = sum(len(range(1, -(-NetPlan.units(B, B, s) // c))) for s, c in chunks.items()
                   if c)
    assert len(pick) >= 64
    print(f"{cfg} {dt} {numerics}: {len(pick)} sampled entries ({2 * n_bounds} at chunk "
          f"boundaries, chunks {chunks}), worst rel err {worst:.2e}")
