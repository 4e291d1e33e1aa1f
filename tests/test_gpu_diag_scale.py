"""The prior variances of the test set at the reference's size (save_kernel.py:33-36:
Kv_diag / Kt_diag = ``model(z, z, True, True)`` over the 10 000 test images, the input of
the posterior variance), for the two ResNet configs, fp64 and fp32.

One call over all 10 000 MNIST-/CIFAR-like images (tools/fullscale.py's generator, seed 1,
the full-scale legs' Z) is checked on sampled images, the first and the last among them:
against ``oracle.kernel(..., same=True, diag=True)`` (reference kernels.py:18-57; 1e-8 in
fp64 — the closed-form ReLU's bound —, 1e-5 in fp32 against the fp64 oracle on the same
float32-rounded images), bit-equal to the same call on the single image (no dependence on
the batch), and within 1e-12 of the diagonal the Kxx path writes (the variance chain's
kdiag on a same tile)."""
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
M = 10000
CASES = [("mnist_as_tf", "f64", 1e-8), ("cifar10", "f64", 1e-8), ("mnist_as_tf", "f32", 1e-5),
         ("cifar10", "f32", 1e-5)]


@pytest.mark.parametrize("cfg,dt,rtol", CASES, ids=[f"{c}-{d}" for c, d, _ in CASES])
def test_prior_variances_of_the_test_set(cfg, dt, rtol):
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(
        os.path.abspath(__file__))), "tools"))
    from fullscale import mnist_like
    tdt = torch.float64 if dt == "f64" else torch.float32
    C, side = specs.GEOMETRY[cfg]
    spec = specs.CONFIGS[cfg]()
    m = configs_util.model(cfg).to(DEV, tdt)
    Z = mnist_like(M, C, side, 1).to(DEV, tdt)
    with torch.no_grad():
        kd = m(Z, Z, True, True)
        Kxx = m(Z[:64])
    assert kd.shape == (M,) and kd.dtype == tdt
    kh = kd.double().cpu().numpy()
    assert np.isfinite(kh).all() and (kh > 0).all()
    Zh = Z.double().cpu().numpy()
    rng = np.random.default_rng(3)
    pick = sorted({0, 1, 63, M - 1, *(int(v) for v in rng.integers(0, M, 20))})
    worst = 0.0
    for k in pick:
        ref = O.kernel(spec, Zh[k:k + 1], Zh[k:k + 1], True, True)[0]
        err = abs(kh[k] - ref) / abs(ref)
        worst = max(worst, err)
        assert err < rtol, (cfg, dt, k, kh[k], ref, err)
        with torch.no_grad():
            one = m(Z[k:k + 1], Z[k:k + 1], True, True).item()
        assert one == kh[k], ("batch dependence", k, one, kh[k])
    dg = torch.diagonal(Kxx).double().cpu().numpy()
    rel = np.abs(dg - kh[:64]) / np.abs(kh[:64])
    assert rel.max() < 1e-12 if dt == "f64" else rel.max() < 1e-6, rel.max()
    print(f"{cfg} {dt} Kt_diag over {M} images: {len(pick)} vs oracle, worst {worst:.2e}; "
          f"single-image calls bit-equal; vs the Kxx diagonal {rel.max():.1e}")
