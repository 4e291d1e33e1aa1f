"""Pin the CPU oracle to the reference's own outputs (tests/golden/*.npz, produced by
tests/golden/make_golden.py running /root/reference in the build container)."""
import os

import numpy as np
import pytest

from oracle import nngp_oracle as O
from oracle import specs

from conftest import GOLDEN


def load(name):
    return np.load(os.path.join(GOLDEN, name))


def conv_spec(par):
    k, s, pad, d, vw, vb = par
    return dict(kernel_size=int(k), stride=int(s), padding="same" if pad == -1 else int(pad),
                dilation=int(d), var_weight=float(vw), var_bias=float(vb))


def test_conv_ops_match_reference():
    z = load("conv_ops.npz")
    keys = sorted({k.rsplit("_", 1)[0] for k in z.files})
    assert len(keys) >= 50
    for k in keys:
        maps = z[k + "_in"].astype(np.float64)
        out = O.conv_maps(maps, conv_spec(z[k + "_par"]))
        ref = z[k + "_out"]
        assert out.shape == ref.shape, k
        np.testing.assert_allclose(out, ref, rtol=1e-13, atol=1e-13, err_msg=k)


@pytest.mark.parametrize("dt", ["f64", "f32"])
@pytest.mark.parametrize("same", [0, 1])
@pytest.mark.parametrize("diag", [0, 1])
def test_relu_ops_match_reference(dt, same, diag):
    z = load("relu_ops.npz")
    key = f"{dt}_s{same}_d{diag}"
    xy, xx, yy = z[key + "_xy"], z[key + "_xx"], z[key + "_yy"]
    n1, hw = xx.shape
    side = int(round(hw ** 0.5))
    kp = O.make_kp(same, diag, xy.reshape(-1, side, side), xx.reshape(n1, side, side),
                   yy.reshape(len(yy), side, side))
    out = O.relu(kp)
    tol = 1e-12 if dt == "f64" else 2e-6
    np.testing.assert_allclose(out["xy"].reshape(-1, hw), z[key + "_oxy"], rtol=tol, atol=tol)
    np.testing.assert_array_equal(out["xx"].reshape(n1, hw), z[key + "_oxx"])
    np.testing.assert_array_equal(out["yy"].reshape(len(yy), hw), z[key + "_oyy"])


def test_relu_known_answers():
    z = load("relu_ops.npz")
    c, v1, v2 = z["known_c"], z["known_v1"], z["known_v2"]
    kp = O.make_kp(False, True, c.reshape(4, 1, 1), v1.reshape(4, 1, 1), v2.reshape(4, 1, 1))
    out = O.relu(kp)["xy"].reshape(4)
    np.testing.assert_allclose(out, z["known_out"], rtol=1e-15, atol=0)
    # SURVEY.md §4 known answers
    assert abs(out[0] - np.sqrt(6.0) / (2 * np.pi)) < 1e-15
    assert abs(out[1] - np.sqrt(6.0) / 2) < 1e-8
    assert abs(out[3] - 1.7255613506e-20) / 1.7255613506e-20 < 1e-9


@pytest.mark.parametrize("cfg", ["mnist_paper_convnet_gp", "mnist_paper_residual_cnn_gp",
                                 "mnist_as_tf", "cifar10"])
def test_e2e_match_reference(cfg):
    z = load(f"e2e_{cfg}.npz")
    spec = specs.CONFIGS[cfg]()
    prefixes = sorted({k.rsplit("_", 1)[0] for k in z.files if k.endswith("_X")})
    assert prefixes
    for pre in prefixes:
        X, Z = z[pre + "_X"], z[pre + "_Z"]
        for dtn, dt, tol in (("f64", np.float64, 1e-11), ("f32", np.float32, 2e-5)):
            Xd, Zd = X.astype(dt), Z.astype(dt)
            cases = {
                "Kxx": O.kernel(spec, Xd),
                "Kxz": O.kernel(spec, Xd, Zd, False, False),
                "Kxdiag": O.kernel(spec, Xd, Xd, True, True),
                "Kxzdiag": O.kernel(spec, Xd[:6], Zd, False, True),
            }
            for name, got in cases.items():
                ref = z[f"{pre}_{dtn}_{name}"]
                np.testing.assert_allclose(got, ref, rtol=tol, atol=0,
                                           err_msg=f"{cfg} {pre} {dtn} {name}")


@pytest.mark.parametrize("net", ["big", "small"])
def test_mixture_matches_reference(net):
    """Mixture (kernels.py:220-225): softmax of the float32-created logit in the model's
    dtype, branch-weighted sum; 3-term Sum alongside"""
    import configs_util
    z = load("e2e_mixture.npz")
    model, _ = configs_util.mixture_nets()[net]
    spec = configs_util.spec_of(model)
    X, Z = z[net + "_X"], z[net + "_Z"]
    for dtn, dt, tol in (("f64", np.float64, 1e-11), ("f32", np.float32, 2e-5)):
        Xd, Zd = X.astype(dt), Z.astype(dt)
        cases = {"Kxx": O.kernel(spec, Xd), "Kxz": O.kernel(spec, Xd, Zd, False, False),
                 "Kxdiag": O.kernel(spec, Xd, Xd, True, True)}
        for name, got in cases.items():
            np.testing.assert_allclose(got, z[f"{net}_{dtn}_{name}"], rtol=tol, atol=0,
                                       err_msg=f"{net} {dtn} {name}")


@pytest.mark.parametrize("cfg", ["mnist_paper_convnet_gp", "mnist_as_tf"])
def test_torch_cpu_baseline_matches_reference(cfg):
    """bench.py's CPU baseline (oracle/torch_cpu.py) computes what the reference does"""
    import torch
    from oracle import torch_cpu
    z = load(f"e2e_{cfg}.npz")
    spec = specs.CONFIGS[cfg]()
    for pre in ("s0_uniform", "s0_mnist"):
        X, Z = torch.from_numpy(z[pre + "_X"]), torch.from_numpy(z[pre + "_Z"])
        for dtn, dt, tol in (("f64", torch.float64, 1e-12), ("f32", torch.float32, 2e-6)):
            got = {"Kxx": torch_cpu.kernel(spec, X.to(dt)),
                   "Kxz": torch_cpu.kernel(spec, X.to(dt), Z.to(dt), False, False),
                   "Kxdiag": torch_cpu.kernel(spec, X.to(dt), X.to(dt), True, True)}
            for name, t in got.items():
                np.testing.assert_allclose(t.numpy(), z[f"{pre}_{dtn}_{name}"], rtol=tol,
                                           atol=0, err_msg=f"{cfg} {pre} {dtn} {name}")


def test_tile_schedule_matches_reference():
    z = load("tiles.npz")
    X, Z = z["X"].astype(np.float64), z["Z"].astype(np.float64)
    spec = specs.mnist_paper_convnet_gp()
    for nw in (1, 3):
        for r in range(nw):
            got = O.gram_tiles(spec, X, None, 16, r, nw)
            ref = z[f"Kxx_nw{nw}_r{r}"]
            np.testing.assert_array_equal(np.isnan(got), np.isnan(ref))
            m = ~np.isnan(ref)
            np.testing.assert_allclose(got[m], ref[m], rtol=1e-6)
            got = O.gram_tiles(spec, X, Z, 16, r, nw)
            ref = z[f"Kxz_nw{nw}_r{r}"]
            np.testing.assert_array_equal(np.isnan(got), np.isnan(ref))
    # the documented 3-worker split
    assert O.tile_schedule(40, None, 16, 0, 3) == [(True, 0, 0), (False, 0, 16)]
    assert O.tile_schedule(40, None, 16, 1, 3) == [(False, 0, 32), (True, 16, 16)]
    assert O.tile_schedule(40, None, 16, 2, 3) == [(False, 16, 32), (True, 32, 32)]


def test_solve_matches_reference_call():
    z = load("solve.npz")
    K = z["K"].copy()
    K[np.tril_indices(len(K), -1)] = np.nan
    sol = O.solve_upper(K, z["Y"], float(z["jitter"]))
    np.testing.assert_allclose(sol, z["sol"], rtol=1e-10, atol=1e-10)
