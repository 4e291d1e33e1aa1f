"""Generate the golden vectors in tests/golden/*.npz by running the REFERENCE.

Run in the build container only (the reference is not on the GPU box):

    python tests/golden/make_golden.py

It imports /root/reference/cnn_gp (pure Python over torch) with two import-time shims
that SURVEY.md §8(c) records: a stub ``torchvision`` module (cnn_gp/__init__.py imports
data.py, which imports torchvision for DatasetFromConfig only; configs reference
``torchvision.datasets.*`` as a class attribute) and ``np.int = int`` (data.py:12 uses
the alias removed in numpy 1.24).  Nothing from the reference is copied: the files
written here hold inputs and the reference's outputs only.

Fixtures (all inputs are float32-representable, stored as float32):
  conv_ops.npz    Conv2d.propagate on random maps for many (k, stride, padding, dilation)
  relu_ops.npz    ReLU.propagate on valid covariance patches, every same/diag combination
  e2e_<cfg>.npz   model(X), model(X, Z), model(X, X, same=True, diag=True),
                  model(X[:6], Z, same=False, diag=True) for every config, fp64 and fp32
  tiles.npz       save_K tile assembly with a fake h5 file (NaN pattern, worker split)
  solve.npz       scipy posv on a reference Kxx with NaN lower triangle
  e2e_mixture.npz Mixture (3 branches, non-zero logits) + 3-term Sum networks at 28x28
                  (whole-network kernel shapes) and 10x10 (layer path), fp64 and fp32
"""
from __future__ import annotations

import itertools
import os
import sys
import types

import numpy as np

np.int = int  # data.py:12 (numpy >= 1.24 removed the alias)
_tv = types.ModuleType("torchvision")
_tv.datasets = types.SimpleNamespace(MNIST=None, CIFAR10=None)
_tv.transforms = types.SimpleNamespace(ToTensor=None, Compose=None)
sys.modules["torchvision"] = _tv
sys.path.insert(0, "/root/reference")

import importlib  # noqa: E402

import scipy.linalg  # noqa: E402
import torch  # noqa: E402
from torch.utils.data import TensorDataset  # noqa: E402

import cnn_gp  # noqa: E402
from cnn_gp.kernel_patch import ConvKP, NonlinKP  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))
CONFIGS = ["mnist_paper_convnet_gp", "mnist_paper_residual_cnn_gp", "mnist_as_tf", "cifar10"]


def mnist_like(n, c, side, rng):
    """4-px zero border, ~60% zero pixels, values k/255 (MNIST-like statistics)."""
    x = np.zeros((n, c, side, side), dtype=np.float32)
    inner = rng.integers(0, 256, size=(n, c, side - 8, side - 8)).astype(np.float32) / 255
    inner[rng.random(inner.shape) < 0.6] = 0
    x[:, :, 4:-4, 4:-4] = inner
    return x


def uniform(n, c, side, rng):
    return rng.random((n, c, side, side), dtype=np.float32)


def gen_conv_ops():
    rng = np.random.default_rng(1234)
    cases = []
    for k, s, pad, d, side in itertools.product([1, 2, 3, 4, 5, 7], [1, 2], ["same", 0, 1],
                                                 [1, 2], [28, 14, 7]):
        cases.append((k, s, pad, d, side))
    sel = [cases[i] for i in rng.choice(len(cases), size=48, replace=False)]
    # every geometry the configs use
    sel += [(7, 1, "same", 1, 28), (28, 1, 0, 1, 28), (4, 1, "same", 1, 28), (3, 1, "same", 1, 28),
            (3, 2, "same", 1, 28), (1, 2, "same", 1, 28), (3, 2, "same", 1, 14),
            (1, 2, "same", 1, 14), (7, 1, 0, 1, 7), (1, 1, 0, 1, 1), (8, 1, 0, 1, 8),
            (3, 1, "same", 1, 32), (3, 2, "same", 1, 32), (2, 1, "same", 2, 14),
            (6, 1, "same", 1, 14)]
    recs = {}
    for n, (k, s, pad, d, side) in enumerate(sel):
        maps = rng.random((3, side, side), dtype=np.float32)
        vw = float(rng.choice([1.0, 2.79 * k * k, 7.27 * k * k, 0.5]))
        vb = float(rng.choice([0.0, 7.86, 4.69]))
        try:
            mod = cnn_gp.Conv2d(k, stride=s, padding=pad, dilation=d, var_weight=vw,
                                var_bias=vb).double()
            t = torch.from_numpy(maps.astype(np.float64))
            kp = ConvKP(False, True, t[:, None], t[:, None], t[:, None])
            out = mod.propagate(kp).xy[:, 0].numpy()
        except RuntimeError:
            continue  # geometry invalid for this size (F.conv2d refuses it)
        recs[f"c{n}_in"] = maps
        recs[f"c{n}_out"] = out
        recs[f"c{n}_par"] = np.array([k, s, -1 if pad == "same" else pad, d, vw, vb])
    np.savez_compressed(os.path.join(OUT, "conv_ops.npz"), **recs)
    print("conv_ops:", len(recs) // 3, "cases")


def _valid_kp(n1, n2, hw, rng, dtype, zero_frac=0.2):
    """Covariances from random feature vectors, so |c| <= sqrt(v1 v2) holds."""
    f = 5
    a = rng.standard_normal((n1, hw, f))
    b = rng.standard_normal((n2, hw, f))
    mask1 = rng.random((n1, hw)) < zero_frac
    a[mask1] = 0.0
    xx = (a * a).sum(-1)
    yy = (b * b).sum(-1)
    xy = np.einsum("ipf,jpf->ijp", a, b)
    return xy.astype(dtype), xx.astype(dtype), yy.astype(dtype)


def gen_relu_ops():
    rng = np.random.default_rng(99)
    recs = {}
    side = 5
    hw = side * side
    for dtn, dt, tdt in (("f64", np.float64, torch.float64), ("f32", np.float32, torch.float32)):
        for same, diag in itertools.product([False, True], [False, True]):
            n1 = 4
            n2 = 4 if (same or diag) else 3
            xy, xx, yy = _valid_kp(n1, n2, hw, rng, dt)
            if same:
                # same tiles: yy is xx, and the pair maps are a Gram of one set
                yy = xx.copy()
                a = np.sqrt(np.maximum(xx, 0))[:, None] * np.sqrt(np.maximum(yy, 0))[None]
                xy = (0.7 * a).astype(dt)
            if diag:
                xy = xy[np.arange(n1), np.arange(n1)]
            key = f"{dtn}_s{int(same)}_d{int(diag)}"
            xyt = torch.from_numpy(xy.reshape(-1, side, side)[:, None].copy())
            kp = NonlinKP(ConvKP(same, diag, xyt, torch.from_numpy(xx.reshape(n1, 1, side, side)),
                                 torch.from_numpy(yy.reshape(n2, 1, side, side))))
            out = cnn_gp.ReLU().propagate(kp)
            recs[key + "_xy"] = xy.reshape(-1, hw)
            recs[key + "_xx"] = xx
            recs[key + "_yy"] = yy
            recs[key + "_oxy"] = out.xy.reshape(-1, hw).numpy()
            recs[key + "_oxx"] = out.xx.reshape(n1, hw).numpy()
            recs[key + "_oyy"] = out.yy.reshape(n2, hw).numpy()
            assert out.xy.dtype == tdt
    # known answers: v1=2, v2=3 and c in {0, +sqrt(6), -sqrt(6)}, plus zeros
    c = np.array([0.0, np.sqrt(6.0), -np.sqrt(6.0), 0.0])
    v1 = np.array([2.0, 2.0, 2.0, 0.0])
    v2 = np.array([3.0, 3.0, 3.0, 0.0])
    t = lambda a: torch.from_numpy(a.reshape(4, 1, 1, 1))  # noqa: E731
    kp = ConvKP(False, True, t(c), t(v1), t(v2))
    out = cnn_gp.ReLU().propagate(NonlinKP(kp))
    recs["known_c"], recs["known_v1"], recs["known_v2"] = c, v1, v2
    recs["known_out"] = out.xy.reshape(4).numpy()
    np.savez_compressed(os.path.join(OUT, "relu_ops.npz"), **recs)
    print("relu_ops:", len(recs), "arrays")


def gen_e2e():
    for name in CONFIGS:
        cfg = importlib.import_module(f"configs.{name}")
        chans = getattr(cfg, "in_channels", 1)
        side = 32 if name == "cifar10" else 28
        recs = {}
        seeds = [0] if name == "cifar10" else [0, 1]
        for seed, dist in itertools.product(seeds, ["uniform", "mnist"]):
            rng = np.random.default_rng(1000 + seed)
            gen = uniform if dist == "uniform" else mnist_like
            X = gen(8, chans, side, rng)
            Z = gen(6, chans, side, rng)
            key = f"s{seed}_{dist}"
            recs[key + "_X"], recs[key + "_Z"] = X, Z
            for dtn, tdt in (("f64", torch.float64), ("f32", torch.float32)):
                model = cfg.initial_model.to(tdt)
                Xt, Zt = torch.from_numpy(X).to(tdt), torch.from_numpy(Z).to(tdt)
                with torch.no_grad():
                    recs[f"{key}_{dtn}_Kxx"] = model(Xt).numpy()
                    recs[f"{key}_{dtn}_Kxz"] = model(Xt, Zt, False, False).numpy()
                    recs[f"{key}_{dtn}_Kxdiag"] = model(Xt, Xt, True, True).numpy()
                    recs[f"{key}_{dtn}_Kxzdiag"] = model(Xt[:6], Zt, False, True).numpy()
            cfg.initial_model.to(torch.float32)
        np.savez_compressed(os.path.join(OUT, f"e2e_{name}.npz"), **recs)
        print("e2e", name, len(recs), "arrays")


class FakeDataset:
    """numpy-backed stand-in for one h5py dataset (create_dataset + slice assignment)."""

    def __init__(self, shape, dtype, fillvalue, chunks, maxshape):
        self.a = np.full(shape, fillvalue, dtype=dtype)
        self.chunks, self.maxshape = chunks, maxshape

    def __setitem__(self, k, v):
        self.a[k] = v


class FakeFile:
    def __init__(self):
        self.d = {}

    def keys(self):
        return self.d.keys()

    def create_dataset(self, name, shape, dtype, fillvalue, chunks, maxshape):
        self.d[name] = FakeDataset(shape, dtype, fillvalue, chunks, maxshape)
        return self.d[name]


def gen_tiles():
    cfg = importlib.import_module("configs.mnist_paper_convnet_gp")
    model = cfg.initial_model.to(torch.float64)
    rng = np.random.default_rng(7)
    X = mnist_like(40, 1, 28, rng)
    Z = mnist_like(23, 1, 28, rng)
    dsx = TensorDataset(torch.from_numpy(X).double(), torch.zeros(40, dtype=torch.long))
    dsz = TensorDataset(torch.from_numpy(Z).double(), torch.zeros(23, dtype=torch.long))

    def kern(x, x2, same, diag):
        with torch.no_grad():
            return model(x, x2, same, diag).detach().cpu().numpy()

    recs = {"X": X, "Z": Z}
    for nw in (1, 3):
        for r in range(nw):
            f = FakeFile()
            cnn_gp.save_K(f, kern, "Kxx", dsx, None, False, 16, worker_rank=r, n_workers=nw,
                          print_interval=1e9)
            cnn_gp.save_K(f, kern, "Kxz", dsx, dsz, False, 16, worker_rank=r, n_workers=nw,
                          print_interval=1e9)
            recs[f"Kxx_nw{nw}_r{r}"] = f.d["Kxx"].a
            recs[f"Kxz_nw{nw}_r{r}"] = f.d["Kxz"].a
            if r == 0:
                recs[f"Kxx_chunks_nw{nw}"] = np.array(f.d["Kxx"].chunks)
    f = FakeFile()
    cnn_gp.save_K(f, kern, "Kx_diag", dsx, None, True, 16, print_interval=1e9)
    recs["Kx_diag"] = f.d["Kx_diag"].a
    recs["Kx_diag_chunks"] = np.array(f.d["Kx_diag"].chunks)
    np.savez_compressed(os.path.join(OUT, "tiles.npz"), **recs)
    print("tiles:", len(recs), "arrays")
    cfg.initial_model.to(torch.float32)


def gen_solve():
    """classify_gp.solve_system's call (classify_gp.py:24-26) on a reference Kxx whose
    strictly-lower triangle is NaN, as in the reference's HDF5 output."""
    cfg = importlib.import_module("configs.mnist_paper_convnet_gp")
    model = cfg.initial_model.to(torch.float64)
    rng = np.random.default_rng(11)
    n = 96
    X = mnist_like(n, 1, 28, rng)
    labels = rng.integers(0, 10, size=n)
    with torch.no_grad():
        K = model(torch.from_numpy(X).double()).numpy()
    Y = -np.ones((n, 10))
    Y[np.arange(n), labels] = 1.0
    Kn = K.copy()
    Kn[np.tril_indices(n, -1)] = np.nan
    jitter = 1e-6
    A = Kn.copy()
    A.flat[::n + 1] += jitter
    sol = scipy.linalg.solve(A, Y, overwrite_a=True, overwrite_b=False, check_finite=False,
                             assume_a="pos", lower=False)
    np.savez_compressed(os.path.join(OUT, "solve.npz"), X=X, K=K, Y=Y, labels=labels,
                        jitter=np.array(jitter), sol=sol)
    print("solve: n =", n)
    cfg.initial_model.to(torch.float32)


def mixture_nets(m):
    """The two Mixture networks of e2e_mixture.npz, built from module namespace ``m``
    (the reference's cnn_gp here; tests/test_gpu_parity.py builds the same ones from the
    build's package).  Logits are non-zero so every softmax weight differs."""
    logit = torch.tensor([0.3, -0.2, 0.1])
    big = m.Sequential(
        m.Conv2d(3, var_bias=0.3),
        m.Mixture([m.Sequential(),
                   m.Sequential(m.ReLU(), m.Conv2d(3, var_weight=2.0)),
                   m.Sequential(m.ReLU(), m.Conv2d(7))], logit.clone()),
        m.Sum([m.Sequential(), m.ReLU(),
               m.Sequential(m.ReLU(), m.Conv2d(1, var_bias=0.5))]),
        m.ReLU(), m.Conv2d(28, padding=0))
    small = m.Sequential(
        m.Conv2d(3, var_bias=0.3),
        m.Mixture([m.Sequential(),
                   m.Sequential(m.ReLU(), m.Conv2d(3, var_weight=2.0)),
                   m.Sequential(m.ReLU(), m.Conv2d(5))], torch.tensor([1.1, -0.7, 0.25])),
        m.ReLU(), m.Conv2d(10, padding=0))
    return {"big": (big, 28), "small": (small, 10)}


def gen_mixture():
    recs = {}
    rng = np.random.default_rng(77)
    for name, (model, side) in mixture_nets(cnn_gp).items():
        X = uniform(7, 1, side, rng)
        Z = mnist_like(5, 1, side, rng) if side == 28 else uniform(5, 1, side, rng)
        recs[f"{name}_X"], recs[f"{name}_Z"] = X, Z
        for dtn, tdt in (("f64", torch.float64), ("f32", torch.float32)):
            mod = model.to(tdt)
            Xt, Zt = torch.from_numpy(X).to(tdt), torch.from_numpy(Z).to(tdt)
            with torch.no_grad():
                recs[f"{name}_{dtn}_Kxx"] = mod(Xt).numpy()
                recs[f"{name}_{dtn}_Kxz"] = mod(Xt, Zt, False, False).numpy()
                recs[f"{name}_{dtn}_Kxdiag"] = mod(Xt, Xt, True, True).numpy()
    np.savez_compressed(os.path.join(OUT, "e2e_mixture.npz"), **recs)
    print("mixture:", len(recs), "arrays")


if __name__ == "__main__":
    torch.set_num_threads(8)
    which = sys.argv[1:] or ["conv", "relu", "e2e", "tiles", "solve", "mixture"]
    for w in which:
        {"conv": gen_conv_ops, "relu": gen_relu_ops, "e2e": gen_e2e, "tiles": gen_tiles,
         "solve": gen_solve, "mixture": gen_mixture}[w]()
