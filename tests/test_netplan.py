"""Whole-network kernel lowering (cnn_gp/netplan.py) checked on CPU: the op list, run by a
numpy emulator of csrc/netfuse.hip (tests/net_emulator.py) over the planned LDS slots,
must reproduce the oracle — this pins slot classes, halos, in-place reuse and LINEAR
chains without a GPU."""
import numpy as np
import pytest
import torch

import cnn_gp
import configs_util
import net_emulator as E
from cnn_gp.netplan import NetPlan, Unsupported
from cnn_gp.program import Plan
from oracle import nngp_oracle as O
from oracle import specs


@pytest.mark.parametrize("cfg", ["mnist_paper_convnet_gp", "mnist_paper_residual_cnn_gp",
                                 "mnist_as_tf", "cifar10"])
def test_emulated_net_program_matches_oracle(cfg):
    C, side = specs.GEOMETRY[cfg]
    m = configs_util.model(cfg)
    net = NetPlan(Plan(m, side, side))
    rng = np.random.default_rng(5)
    X = rng.random((3, C, side, side))
    Z = rng.random((2, C, side, side))
    spec = configs_util.spec_of(m)
    np.testing.assert_allclose(E.kernel(net, X, X, True), O.kernel(spec, X), rtol=1e-13)
    np.testing.assert_allclose(E.kernel(net, X, Z, False), O.kernel(spec, X, Z, False),
                               rtol=1e-13)
    assert net.lds_elems * 8 <= 48 * 1024      # ≥ 3 workgroups per CU


def test_emulated_mixture_and_multiterm_sum():
    m = cnn_gp.Sequential(
        cnn_gp.Conv2d(3, var_bias=0.3),
        cnn_gp.Mixture([cnn_gp.Sequential(),
                        cnn_gp.Sequential(cnn_gp.ReLU(), cnn_gp.Conv2d(3, var_weight=2.0)),
                        cnn_gp.Sequential(cnn_gp.ReLU(), cnn_gp.Conv2d(7))],
                       torch.tensor([0.3, -0.2, 0.1])),
        cnn_gp.Sum([cnn_gp.Sequential(), cnn_gp.ReLU(),
                    cnn_gp.Sequential(cnn_gp.ReLU(), cnn_gp.Conv2d(1, var_bias=0.5))]),
        cnn_gp.ReLU(), cnn_gp.Conv2d(28, padding=0))
    net = NetPlan(Plan(m, 28, 28))
    kinds = [f["kind"] for f, _ in net.records]
    assert kinds.count(3) >= 3                 # LINEAR chain
    rng = np.random.default_rng(6)
    X = rng.random((3, 1, 28, 28))
    Z = rng.random((2, 1, 28, 28))
    ref = O.kernel(configs_util.spec_of(m), X, Z, False, False)
    np.testing.assert_allclose(E.kernel(net, X, Z, False), ref, rtol=1e-6)


def test_unsupported_programs_fall_back():
    with pytest.raises(Unsupported):           # geometry without an instantiation
        NetPlan(Plan(cnn_gp.Sequential(cnn_gp.Conv2d(3), cnn_gp.ReLU(),
                                       cnn_gp.Conv2d(10, padding=0)), 10, 10))
    with pytest.raises(Unsupported):           # output map is not 1x1
        NetPlan(Plan(cnn_gp.Sequential(cnn_gp.Conv2d(3)), 28, 28))
    with pytest.raises(Unsupported):           # dilation
        NetPlan(Plan(cnn_gp.Sequential(cnn_gp.Conv2d(3, dilation=2), cnn_gp.ReLU(),
                                       cnn_gp.Conv2d(28, padding=0)), 28, 28))


def test_slot_reuse_is_tight():
    """ResNet: two 28x28 slots suffice (block input + branch, branch convs in place)"""
    net = NetPlan(Plan(configs_util.model("mnist_as_tf"), 28, 28))
    ws = net.ws[(28, 28)]
    n28 = len({f["dst"] for f, _ in net.records if f["h"] == 28 and f["kind"] != 0
               or f["kind"] == 0 and f.get("geom", (0,) * 7)[2] == 28})
    assert n28 <= 3
    assert ws == 29                             # 28 + one shared zero column


@pytest.mark.parametrize("cfg,fused", [("mnist_paper_convnet_gp", True),
                                       ("mnist_paper_residual_cnn_gp", True),
                                       ("mnist_as_tf", False), ("cifar10", False)])
def test_conv_fused_into_final_reduction(cfg, fused, monkeypatch):
    """the separable conv whose map only the full-map reduction reads is marked SUM and the
    reduction FROM_SUM (one-pair stages only; the ResNets reduce in a 16-pair stage after a
    conv with an addend); CGP_NET_FUSE_REDUCE=0 keeps them apart, emulated results agree"""
    from cnn_gp import _native as N
    from cnn_gp import netplan
    C, side = specs.GEOMETRY[cfg]
    m = configs_util.model(cfg)
    net = NetPlan(Plan(m, side, side))
    codes = [f["code"] for f, _ in net.records if f["kind"] == N.CGP_NET_CONV]
    n_sum = sum(1 for c in codes if c & N.CGP_NET_CODE_SUM)
    n_from = sum(1 for c in codes if c & N.CGP_NET_CODE_FROM_SUM)
    assert (n_sum, n_from) == ((1, 1) if fused else (0, 0))
    if fused:
        k = next(k for k, (f, _) in enumerate(net.records)
                 if f["kind"] == N.CGP_NET_CONV and f["code"] & N.CGP_NET_CODE_SUM)
        assert net.records[k + 1][0]["code"] & N.CGP_NET_CODE_FROM_SUM
        monkeypatch.setattr(netplan, "FUSE_REDUCE", False)
        apart = NetPlan(Plan(m, side, side))
        assert not any(f["code"] & (N.CGP_NET_CODE_SUM | N.CGP_NET_CODE_FROM_SUM)
                       for f, _ in apart.records if f["kind"] == N.CGP_NET_CONV)
        rng = np.random.default_rng(8)
        X = rng.random((3, C, side, side))
        np.testing.assert_allclose(E.kernel(net, X, X, True), E.kernel(apart, X, X, True),
                                   rtol=1e-14)


def test_sum_contract_is_validated():
    """CGP_NET_CODE_SUM / FROM_SUM preconditions (include/cnngp.h): the lowered reference
    programs pass cgp_net_validate and the emulator's check; op lists that break them —
    a SUM the next op does not reduce, a FROM_SUM with no SUM before it, SUM on a direct
    (3-tap) conv or with a second output, SUM in a multi-pair stage — are rejected by
    both, so a misuse of the public ABI raises instead of reading stale partial sums."""
    import copy
    import ctypes
    from cnn_gp import _native as N
    lib = N.load()

    def lib_ok(st):
        arr = net._ops_array(st, None)
        return lib.cgp_net_validate(ctypes.byref(arr), st.n_ops, st.pairs) == 0

    def emu_ok(st):
        try:
            E.validate(st)
            return True
        except ValueError:
            return False

    for cfg in ("mnist_paper_convnet_gp", "mnist_paper_residual_cnn_gp", "mnist_as_tf",
                "cifar10"):
        C, side = specs.GEOMETRY[cfg]
        net = NetPlan(Plan(configs_util.model(cfg), side, side))
        for st in net.stages:
            assert lib_ok(st) and emu_ok(st), cfg
    net = NetPlan(Plan(configs_util.model("mnist_paper_convnet_gp"), 28, 28))
    st = net.stages[0]
    recs = [f for f, _ in st.records]
    k = next(i for i, f in enumerate(recs) if f["kind"] == 0 and f["code"] & N.CGP_NET_CODE_SUM)

    def broken(edit):
        b = copy.deepcopy(st)
        edit([f for f, _ in b.records])
        return b

    cases = [
        lambda r: r[k + 1].__setitem__("code", r[k + 1]["code"] & ~N.CGP_NET_CODE_FROM_SUM),
        lambda r: r[k].__setitem__("code", r[k]["code"] & ~N.CGP_NET_CODE_SUM),
        lambda r: r[k].__setitem__("dst2", r[k]["src"]),
        lambda r: r[k + 1].__setitem__("src", r[k + 1]["src"] + 1),
    ]
    for edit in cases:
        b = broken(edit)
        assert not lib_ok(b) and not emu_ok(b)
    # SUM on a direct 3x3 conv (mnist_as_tf's) and SUM in a 4-pair stage
    tf = NetPlan(Plan(configs_util.model("mnist_as_tf"), 28, 28))
    d = copy.deepcopy(tf.stages[0])
    r = [f for f, _ in d.records]
    j = next(i for i, f in enumerate(r) if f["kind"] == 0 and f["geom"][4] == 3)
    r[j]["code"] |= N.CGP_NET_CODE_SUM
    assert not lib_ok(d) and not emu_ok(d)
    m = copy.deepcopy(st)
    m.pairs = 4
    assert not lib_ok(m) and not emu_ok(m)


def test_chunk_units_asks_free_memory_only_for_large_state(monkeypatch):
    """the free-memory query (hipMemGetInfo, 0.1-0.5 ms) runs only when a launch group's
    state buffers could exceed SMALL_STATE_BYTES: a per-tile forward at batch 200 never
    asks, a full-scale B = 4096 tile does"""
    from cnn_gp import netplan
    calls = []

    def fake_info(dev):
        calls.append(dev)
        return (64 << 30, 288 << 30)
    monkeypatch.setattr(torch.cuda, "mem_get_info", fake_info)
    net = NetPlan(Plan(configs_util.model("mnist_as_tf"), 28, 28))
    small = 40000                                 # a B = 200 Kxz tile: 25² supertiles · 64
    assert net.chunk_units(8, small, "cuda:0") == small and not calls
    big = 4096 * 4096
    c = net.chunk_units(8, big, "cuda:0")
    assert calls and 64 <= c < big and c % 64 == 0
    per_unit = sum(st.load_stride for st in net.stages[1:]) * 8
    assert c * per_unit <= (64 << 30) * netplan.STATE_FREE_FRAC
