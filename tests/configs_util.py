"""Test helpers: build product models for the restated configs and convert a product
module tree into the oracle's spec format (so the oracle evaluates the same architecture)."""
import importlib

import cnn_gp


def model(name):
    mod = importlib.import_module(f"configs.{name}")
    importlib.reload(mod)       # fresh module tree (fusion flags, dtype) per test
    return mod.initial_model


def spec_of(m):
    if isinstance(m, cnn_gp.Conv2d):
        pad = m._padding_arg
        return ("conv", dict(kernel_size=m.kernel_size, stride=m.stride, padding=pad,
                             dilation=m.dilation, var_weight=m.var_weight,
                             var_bias=m.var_bias))
    if isinstance(m, cnn_gp.ReLU):
        return ("relu",)
    if isinstance(m, cnn_gp.Sequential):
        return ("seq", [spec_of(x) for x in m.mods])
    if isinstance(m, cnn_gp.Sum):
        return ("sum", [spec_of(x) for x in m.mods])
    if isinstance(m, cnn_gp.Mixture):
        return ("mix", [spec_of(x) for x in m.mods], [float(v) for v in m.logit.detach()])
    raise TypeError(type(m))


def mixture_nets():
    """The Mixture networks of tests/golden/e2e_mixture.npz built from the build's package
    — the same architectures tests/golden/make_golden.py:mixture_nets builds from the
    reference (keep the two in sync).  name -> (model, side)."""
    import torch
    m = cnn_gp
    big = m.Sequential(
        m.Conv2d(3, var_bias=0.3),
        m.Mixture([m.Sequential(),
                   m.Sequential(m.ReLU(), m.Conv2d(3, var_weight=2.0)),
                   m.Sequential(m.ReLU(), m.Conv2d(7))], torch.tensor([0.3, -0.2, 0.1])),
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
