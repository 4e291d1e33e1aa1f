"""Parity at the bench geometry: a 4096-image Kxx and a 4096 × 1024 Kxz built from
B = 1024 tiles (the bench's tile size, staged programs with chunked state for the ResNet,
the per-XCD work counters and the supertile walk at full size), sampled entries checked
against the CPU oracle.  The oracle evaluates one pair at a time (the ConvNet at ~2 k
pairs/s on one core), so 96 samples per matrix cost seconds.

Samples cover: diagonal-tile interior pairs (i < j, and their mirror j > i), the tile
diagonal itself (K[i, i] from the variance chain), off-diagonal tiles, pairs on both
sides of every state-chunk boundary of the staged program (units u = k·chunk − 1 and
k·chunk), supertile corners, and MNIST-like images (4-pixel zero border, ~60% zero
pixels, k/255 values: the f32_tiny path) next to uniform ones.

Tolerances: 1e-10 relative with the op-by-op ReLU (set_exact_relu(True)), 1e-8 with
the closed form (the reference's acos(ρ) near |ρ| = 1 carries ~1e-8 of its own noise)."""
import numpy as np
import pytest
import torch

from oracle import nngp_oracle as O
from oracle import specs

import configs_util

pytestmark = pytest.mark.gpu

DEV = "cuda"
N, NZ, B = 4096, 1024, 1024
RTOL = {"exact": 1e-10, "fast": 1e-8}


def _images(n, C, side, seed):
    """half uniform, half MNIST-like, interleaved"""
    rng = np.random.default_rng(seed)
    X = rng.random((n, C, side, side))
    m = np.floor(rng.random((n, C, side, side)) * 256) / 255.0
    m[rng.random(m.shape) < 0.6] = 0.0
    m[..., :4, :] = 0.0
    m[..., -4:, :] = 0.0
    m[..., :, :4] = 0.0
    m[..., :, -4:] = 0.0
    X[1::2] = m[1::2]
    return X


def _tri_decode(s, nb):
    """supertile s of the upper triangle (bi <= bj), row-major (netfuse.hip tri_decode)"""
    r = 0
    while (r + 1) * nb - (r + 1) * r // 2 <= s:
        r += 1
    return r, r + (s - (r * nb - r * (r - 1) // 2))


def _unit_pair(u, n1, n2, same, st):
    s, q = divmod(u, st * st)
    nbi, nbj = -(-n1 // st), -(-n2 // st)
    bi, bj = _tri_decode(s, nbi) if same else divmod(s, nbj)
    return bi * st + q // st, bj * st + q % st


def _samples(rng, chunk, st, same_tile_n, n1, n2, same, count):
    """(i, j) inside one tile: chunk-boundary units, supertile corners, random pairs"""
    from cnn_gp.netplan import NetPlan
    units = NetPlan.units(n1, n2, same)
    out = []
    for k in range(1, -(-units // chunk)):
        for u in (k * chunk - 1, k * chunk):
            i, j = _unit_pair(u, n1, n2, same, st)
            if i < n1 and j < n2:
                out.append((i, j))
    out += [(0, 0), (0, n2 - 1), (n1 - 1, 0), (n1 - 1, n2 - 1), (st - 1, st), (st, st - 1)]
    while len(out) < count:
        out.append((int(rng.integers(n1)), int(rng.integers(n2))))
    return out


@pytest.mark.parametrize("cfg", ["mnist_paper_convnet_gp", "mnist_as_tf", "cifar10"])
@pytest.mark.parametrize("numerics", ["fast", "exact"])
def test_bench_geometry_sampled_entries_vs_oracle(cfg, numerics, monkeypatch):
    from cnn_gp import gram, netplan
    from cnn_gp import _native as Nat
    C, side = specs.GEOMETRY[cfg]
    spec = specs.CONFIGS[cfg]()
    X = _images(N, C, side, 41)
    Z = _images(NZ, C, side, 42)
    m = configs_util.model(cfg).to(DEV, torch.float64).set_exact_relu(numerics == "exact")
    plan = m._plan(side, side)
    net = m._net_plan(plan, 8)
    assert net is not None
    st = Nat.load().cgp_net_supertile()
    chunk = None
    if len(net.stages) > 1:
        # ~10 state chunks per tile: every launch group starts mid-supertile-row
        stride = max(max(s.load_stride, s.store_stride) for s in net.stages)
        chunk = 100032
        monkeypatch.setattr(netplan, "CHUNK_BYTES", chunk * stride * 8)
    Xd, Zd = torch.from_numpy(X).to(DEV), torch.from_numpy(Z).to(DEV)
    kern = gram.model_kern(m)
    Kxx, tiles = gram.gram_tiles(kern, Xd, None, B)
    Kxz, _ = gram.gram_tiles(kern, Xd, Zd, B)
    assert len(tiles) == 10
    Kxx_h, Kxz_h = Kxx.cpu().numpy(), Kxz.cpu().numpy()
    assert not np.isnan(Kxz_h).any()
    iu = np.triu_indices(N)
    assert not np.isnan(Kxx_h[iu]).any()
    rng = np.random.default_rng(7)
    pick = []          # (matrix, global i, global j)
    ch = chunk or 1 << 62
    # diagonal tile (1, 1), off-diagonal Kxx tile (0, 2), Kxz tile (3, 0)
    for name, ti, tj, same in (("xx", 1, 1, True), ("xx", 0, 2, False), ("xz", 3, 0, False)):
        for i, j in _samples(rng, ch, st, B, B, B, same, 32):
            pick.append((name, ti * B + i, tj * B + j))
    pick += [("xx", k, k) for k in (0, 1, 1023, 1024, 4095)]          # diagonal entries
    tol = RTOL[numerics]
    worst = 0.0
    for name, i, j in pick:
        a = X[i:i + 1]
        if name == "xx" and i == j:
            ref = O.kernel(spec, a)[0, 0]
            got = Kxx_h[i, i]
        elif name == "xx":
            lo, hi = min(i, j), max(i, j)
            ref = O.kernel(spec, X[lo:lo + 1], X[hi:hi + 1], False, False)[0, 0]
            got = Kxx_h[lo, hi]                  # the upper triangle holds every pair
        else:
            ref = O.kernel(spec, a, Z[j:j + 1], False, False)[0, 0]
            got = Kxz_h[i, j]
        err = abs(got - ref) / abs(ref)
        worst = max(worst, err)
        assert err < tol, (cfg, numerics, name, i, j, got, ref, err)
    # diagonal tiles hold both triangles (the kernel mirrors K[j, i] = K[i, j])
    d = Kxx_h[B:2 * B, B:2 * B]
    assert np.array_equal(d, d.T)
    print(f"{cfg} {numerics}: {len(pick)} sampled entries, worst rel err {worst:.2e}")


@pytest.mark.parametrize("cfg", ["mnist_paper_convnet_gp", "mnist_as_tf", "cifar10"])
def test_f32_kernel_within_north_star_tolerance(cfg):
    """The reference's own pipeline (exp_mnist_resnet/save_kernel.py:19-24) runs the
    float32 model on float32 images and stores K as float32 (kernel_save_tools.py:21).
    The fp32 whole-network kernel on the same images stays within the north star's 1e-5
    relative of the fp64 kernel (itself within 1e-8 of the reference's fp64 goldens):
    a 512 x 384 Kxz and a 384-image Kxx (two-pair head stage, staged ResNet programs)."""
    C, side = specs.GEOMETRY[cfg]
    X = _images(512, C, side, 11)
    Z = _images(384, C, side, 12)
    out = {}
    for dt in (torch.float64, torch.float32):
        m = configs_util.model(cfg).to(DEV, dt)
        with torch.no_grad():
            x = torch.from_numpy(X).to(DEV, dt)
            z = torch.from_numpy(Z).to(DEV, dt)
            out[dt] = (m(x, z, False, False).double().cpu().numpy(),
                       m(z).double().cpu().numpy())
    for a, b in zip(out[torch.float32], out[torch.float64]):
        err = float(np.max(np.abs(a - b) / np.abs(b)))
        print(f"{cfg}: fp32 vs fp64 max rel err {err:.2e}")
        assert err < 1e-5
