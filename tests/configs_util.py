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
