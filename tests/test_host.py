"""CPU-only tests: the C ABI library loads and exports what include/cnngp.h declares,
the program compiler/fuser, the tile schedule and HDF5 layout, and the host plumbing."""
import ctypes
import os
import re

import numpy as np
import pytest
import torch

import cnn_gp
from cnn_gp import _native as N
from cnn_gp.program import Plan
from cnn_gp.data import tile_schedule, worker_slice, read_idx, ProductIterator
from cnn_gp.kernel_save_tools import save_K, merge_nan_fill
from oracle import nngp_oracle as O
from oracle import specs

from conftest import ROOT, GOLDEN
import configs_util


HEADER = os.path.join(ROOT, "include", "cnngp.h")


def header_symbols():
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"\b(cgp_[a-z0-9_]+)\s*\(", txt)))


def test_library_exports_every_header_symbol():
    lib = N.load()
    syms = header_symbols()
    assert len(syms) >= 20
    for s in syms:
        assert hasattr(lib, s), s
    assert set(syms) == set(N.SIGNATURES), set(syms) ^ set(N.SIGNATURES)


def test_struct_layouts_match():
    lib = N.load()
    assert lib.cgp_conv_args_size() == ctypes.sizeof(N.ConvArgs)
    assert lib.cgp_relu_args_size() == ctypes.sizeof(N.ReluArgs)
    assert lib.cgp_abi_version() == N.CGP_ABI_VERSION


def test_library_selftest():
    lib = N.load()
    assert lib.cgp_selftest() == 0, lib.cgp_last_error()


def test_pred_var_rejects_bad_arguments_on_host():
    lib = N.load()
    assert lib.cgp_pred_var_f64(None, 4, 4, None, 2, 4, None, None, None) == 1001
    buf = (ctypes.c_double * 16)()
    p = ctypes.cast(buf, ctypes.c_void_p)
    assert lib.cgp_pred_var_f64(p, 4, 3, p, 2, 4, p, p, None) == 1001     # ldk < n
    assert lib.cgp_pred_var_f64(p, 4, 4, p, 2, 3, p, p, None) == 1001     # ldz < n
    assert lib.cgp_pred_var_f64(p, 4, 4, p, 0, 4, p, p, None) == 0        # m = 0: no work


def test_device_count_without_gpu_is_safe():
    assert N.load().cgp_device_count() >= 0


def test_invalid_arguments_rejected_on_host():
    """argument checks run before any launch (no GPU needed to exercise them)"""
    lib = N.load()
    a = N.ConvArgs()
    assert lib.cgp_conv_f64(ctypes.byref(a), None) == 1001
    assert b"NULL" in lib.cgp_last_error()
    a.in_, a.out = 16, 32
    a.nmaps, a.h, a.w, a.ho, a.wo = 4, 28, 28, 30, 28
    a.taps, a.offset, a.stride, a.dilation = 3, -1, 1, 1
    assert lib.cgp_conv_f64(ctypes.byref(a), None) == 1001
    assert b"inconsistent" in lib.cgp_last_error()
    r = N.ReluArgs()
    assert lib.cgp_relu_f64(ctypes.byref(r), None) == 1001
    assert lib.cgp_axpby_f64(1.0, None, 1.0, None, None, 10, None) == 1001
    assert lib.cgp_scale_batch_f64(2, None, None, None, 0.25, None) == 1001
    assert lib.cgp_scale_batch_f64(0, None, None, None, 0.25, None) == 0


def test_forward_without_gpu_fails_loudly():
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    m = cnn_gp.Sequential(cnn_gp.Conv2d(3), cnn_gp.ReLU(), cnn_gp.Conv2d(4, padding=0))
    with pytest.raises(RuntimeError, match="HIP device"):
        m(torch.rand(2, 1, 4, 4, dtype=torch.float64))


# ------------------------------------------------------------------------------------
# program compiler
# ------------------------------------------------------------------------------------
def _kinds(plan):
    return [(o.kind, o.pre, o.post, o.addend is not None) for o in plan.pair_ops]


def test_convnet_fuses_to_eight_kernels():
    m = configs_util.model("mnist_paper_convnet_gp")
    p = Plan(m, 28, 28)
    k = _kinds(p)
    assert len(k) == 8
    assert k[0] == ("conv", N.CGP_PRE_MOMENTS, N.CGP_POST_RELU, False)
    assert all(x == ("conv", 0, 1, False) for x in k[1:7])
    assert k[7] == ("conv", 0, 0, False)
    assert p.final_hw == (1, 1) and p.moments_fused


def test_resnet_fusion_counts():
    m = configs_util.model("mnist_as_tf")
    p = Plan(m, 28, 28)
    unfused = Plan(m, 28, 28, enable_fusion=False)
    assert len(unfused.pair_ops) == 36 + 31 + 15
    # identity block -> 2 kernels; projection block -> relu + conv1 + conv3(post) +
    # conv3(add), except the first, whose relu folds into the stem conv's epilogue
    assert len(p.pair_ops) == 1 + 3 * (4 + 4 * 2) - 1 + 2
    assert sum(o.kind == "relu" for o in p.pair_ops) == 2
    assert not any(o.kind == "add" for o in p.pair_ops)


def test_residual_cnn_gp_fusion():
    m = configs_util.model("mnist_paper_residual_cnn_gp")
    p = Plan(m, 28, 28)
    k = _kinds(p)
    # 8 x [conv4 + relu + add(identity)] -> 1 kernel each, then conv4+relu, final conv
    assert len(k) == 8 + 1 + 1
    assert not p.moments_fused   # v0 feeds both the first conv and the first shortcut
    assert sum(1 for x in k if x == ("conv", 0, 1, True)) == 8


def test_mixture_lowering_keeps_add():
    m = cnn_gp.Sequential(cnn_gp.Conv2d(3), cnn_gp.Mixture(
        [cnn_gp.Sequential(), cnn_gp.Sequential(cnn_gp.ReLU(), cnn_gp.Conv2d(3))],
        torch.tensor([0.3, -0.2])), cnn_gp.Conv2d(6, padding=0))
    p = Plan(m, 6, 6)
    adds = [o for o in p.pair_ops if o.kind == "add"]
    assert len(adds) == 1 and all(c is not None for c, _ in adds[0].terms)


def test_configs_match_oracle_specs():
    for name in ["mnist_paper_convnet_gp", "mnist_paper_residual_cnn_gp", "mnist_as_tf",
                 "cifar10"]:
        assert configs_util.spec_of(configs_util.model(name)) == specs.CONFIGS[name](), name


def test_nonsquare_output_error_mentions_size():
    m = cnn_gp.Sequential(cnn_gp.Conv2d(3))
    p = Plan(m, 5, 5)
    assert p.final_hw == (5, 5)


# ------------------------------------------------------------------------------------
# tiles / persistence
# ------------------------------------------------------------------------------------
def test_worker_slice_matches_reference_formula():
    for nb in range(0, 40):
        for nw in range(1, 9):
            tot = 0
            for r in range(nw):
                s, c = worker_slice(nb, r, nw)
                assert s == tot
                tot += c
            assert tot == nb
            assert [O.worker_slice(nb, r, nw) for r in range(nw)] == \
                [worker_slice(nb, r, nw) for r in range(nw)]


def test_tile_schedule_matches_oracle():
    for n, n2, b, nw in [(40, None, 16, 3), (40, 23, 16, 2), (7, None, 3, 4), (100, 64, 32, 5)]:
        for r in range(nw):
            ref = O.tile_schedule(n, n2, b, r, nw)
            got = [(s, i * b, j * b) for s, i, j in tile_schedule(n, n2, b, r, nw)]
            assert got == ref


class FakeDS:
    def __init__(self, shape, dtype, fillvalue, chunks, maxshape):
        self.a = np.full(shape, fillvalue, dtype=dtype)
        self.chunks, self.maxshape, self.shape = chunks, maxshape, shape

    def __setitem__(self, k, v):
        self.a[k] = v

    def __getitem__(self, k):
        return self.a[k]

    def __len__(self):
        return len(self.a)


class FakeFile:
    def __init__(self):
        self.d = {}

    def keys(self):
        return self.d.keys()

    def create_dataset(self, name, shape, dtype, fillvalue, chunks, maxshape):
        self.d[name] = FakeDS(shape, dtype, fillvalue, chunks, maxshape)
        return self.d[name]


def test_save_K_layout_matches_reference_files():
    """save_K with the oracle as `kern` reproduces the reference's tile files
    (NaN pattern, chunking, worker split) bit for bit in the NaN mask."""
    z = np.load(os.path.join(GOLDEN, "tiles.npz"))
    X, Z = z["X"].astype(np.float64), z["Z"].astype(np.float64)
    spec = specs.mnist_paper_convnet_gp()
    dsx = torch.utils.data.TensorDataset(torch.from_numpy(X), torch.zeros(len(X)))
    dsz = torch.utils.data.TensorDataset(torch.from_numpy(Z), torch.zeros(len(Z)))

    def kern(x, x2, same, diag):
        return O.kernel(spec, x.numpy(), x2.numpy(), same, diag)

    files = []
    for r in range(3):
        f = FakeFile()
        save_K(f, kern, "Kxx", dsx, None, False, 16, worker_rank=r, n_workers=3,
               print_interval=1e9)
        save_K(f, kern, "Kxz", dsx, dsz, False, 16, worker_rank=r, n_workers=3,
               print_interval=1e9)
        for name in ("Kxx", "Kxz"):
            ref = z[f"{name}_nw3_r{r}"]
            got = f.d[name].a
            np.testing.assert_array_equal(np.isnan(got), np.isnan(ref))
            m = ~np.isnan(ref)
            np.testing.assert_allclose(got[m], ref[m], rtol=1e-6)
        assert f.d["Kxx"].chunks == tuple(z["Kxx_chunks_nw3"])
        files.append(f)
    merged = merge_nan_fill(files[0].d["Kxx"].a.copy(), [f.d["Kxx"].a for f in files[1:]])
    ref1 = z["Kxx_nw1_r0"]
    np.testing.assert_array_equal(np.isnan(merged), np.isnan(ref1))
    f = FakeFile()
    save_K(f, kern, "Kx_diag", dsx, None, True, 16, print_interval=1e9)
    np.testing.assert_allclose(f.d["Kx_diag"].a, z["Kx_diag"], rtol=1e-6)
    assert f.d["Kx_diag"].chunks == tuple(z["Kx_diag_chunks"])
    # existing datasets are skipped, like the reference
    save_K(f, kern, "Kx_diag", dsx, None, True, 16, print_interval=1e9)


def test_product_iterator_batches():
    ds = torch.utils.data.TensorDataset(torch.arange(10.).reshape(10, 1), torch.arange(10))
    it = ProductIterator(4, ds, None, 0, 1)
    seen = [(s, i, j, len(a[0]), len(b[0])) for s, (i, a), (j, b) in it]
    assert seen == [(True, 0, 0, 4, 4), (False, 0, 4, 4, 4), (False, 0, 8, 4, 2),
                    (True, 4, 4, 4, 4), (False, 4, 8, 4, 2), (True, 8, 8, 2, 2)]


def test_idx_reader(tmp_path):
    imgs = (np.arange(2 * 3 * 4) % 256).astype(np.uint8).reshape(2, 3, 4)
    raw = bytes([0, 0, 0x08, 3]) + b"".join(int(d).to_bytes(4, "big") for d in imgs.shape)
    (tmp_path / "t.idx").write_bytes(raw + imgs.tobytes())
    np.testing.assert_array_equal(read_idx(str(tmp_path / "t.idx")), imgs)


def _cifar_fixture(root, fmt, rng):
    """5 train batches of 3 images + a test batch of 2, in the binary or python format"""
    import pickle
    batches = {}
    names = [f"data_batch_{k}" for k in range(1, 6)] + ["test_batch"]
    for k, name in enumerate(names):
        n = 2 if name == "test_batch" else 3
        x = rng.integers(0, 256, size=(n, 3072), dtype=np.uint8)
        y = rng.integers(0, 10, size=n).astype(np.uint8)
        batches[name] = (x, y)
        if fmt == "bin":
            d = root / "CIFAR10" / "cifar-10-batches-bin"
            d.mkdir(parents=True, exist_ok=True)
            (d / (name + ".bin")).write_bytes(np.concatenate([y[:, None], x], 1).tobytes())
        else:
            d = root / "CIFAR10" / "cifar-10-batches-py"
            d.mkdir(parents=True, exist_ok=True)
            with open(d / name, "wb") as f:
                pickle.dump({b"batch_label": name.encode(), b"labels": [int(v) for v in y],
                             b"data": x, b"filenames": [b"f"] * n}, f)
    return batches, names


@pytest.mark.parametrize("fmt", ["bin", "py"])
def test_cifar10_dataset_from_config(tmp_path, fmt):
    """DatasetFromConfig for CIFAR10 (data.py:143-158): ConcatDataset(train 5 batches,
    test batch), ToTensor's float32/255 in [3,32,32] R,G,B planes, Subsets by the
    config's ranges (configs/cifar10.py:4-6 pattern, scaled to the fixture)"""
    import types
    from cnn_gp.data import DatasetFromConfig
    rng = np.random.default_rng(3)
    batches, names = _cifar_fixture(tmp_path, fmt, rng)
    cfg = types.SimpleNamespace(dataset_name="CIFAR10", train_range=range(12),
                                validation_range=range(12, 15), test_range=range(15, 17),
                                transforms=[])
    ds = DatasetFromConfig(str(tmp_path), cfg)
    assert len(ds.data_full) == 17 and len(ds.train) == 12 and len(ds.test) == 2
    allx = np.concatenate([batches[n][0] for n in names]).reshape(-1, 3, 32, 32)
    ally = np.concatenate([batches[n][1] for n in names])
    X, Y = DatasetFromConfig.load_full(ds.test)
    assert X.dtype == torch.float32 and X.shape == (2, 3, 32, 32)
    np.testing.assert_array_equal(X.numpy(), allx[15:17].astype(np.float32) / 255)
    np.testing.assert_array_equal(Y.numpy(), ally[15:17])
    Xv, _ = DatasetFromConfig.load_full(ds.validation)
    np.testing.assert_array_equal(Xv.numpy(), allx[12:15].astype(np.float32) / 255)
    # config transforms run after ToTensor, per item
    cfg.transforms = [lambda t: t * 2]
    X2, _ = DatasetFromConfig.load_full(DatasetFromConfig(str(tmp_path), cfg).test)
    np.testing.assert_array_equal(X2.numpy(), 2 * X.numpy())


def test_cifar10_python_batches_refuse_foreign_globals(tmp_path):
    import pickle
    from cnn_gp.data import load_cifar10
    d = tmp_path / "cifar-10-batches-py"
    d.mkdir()
    for name in [f"data_batch_{k}" for k in range(1, 6)]:
        with open(d / name, "wb") as f:
            pickle.dump({b"data": np.zeros((1, 3072), np.uint8), b"labels": [0],
                         b"evil": os.system}, f)
    with pytest.raises(pickle.UnpicklingError):
        load_cifar10(str(tmp_path), True)


def test_print_timings_passthrough(capsys):
    from cnn_gp.data import print_timings
    assert list(print_timings([1, 2, 3], print_interval=0.0)) == [1, 2, 3]
    assert "3/3 it" in capsys.readouterr().out


def test_bench_balanced_split_covers_every_tile_once():
    """bench.py's multi-GPU split: every tile on exactly one rank, per-rank evaluated
    pairs within one off-diagonal tile of the mean, reference order within a rank"""
    import importlib.util
    import os
    from cnn_gp.data import tile_schedule
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(root, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    B = 1024
    # the block counts DESIGN §7 quotes for the driver's N = 1 / 2 / 4 / 8 runs
    assert [bench.blocks_for_world(4096, B, w) for w in (1, 2, 4, 8)] == [4, 6, 8, 12]
    for world in (1, 2, 3, 4, 8):
        nb = bench.blocks_for_world(4096, B, world)
        n = nb * B
        allt = tile_schedule(n, None, B, 0, 1)
        parts = bench.balanced_split(allt, B, n, world)
        assert len(parts) == world
        assert sorted(t for p in parts for t in p) == sorted(allt)
        for p in parts:
            assert p == sorted(p, key=allt.index)
        cost = lambda t: B * (B - 1) // 2 if t[0] else B * B  # noqa: E731
        loads = [sum(cost(t) for t in p) for p in parts]
        assert max(loads) - sum(loads) / world <= B * B
        # nb² divisible by the world size: every rank within a few pairs of the mean
        assert (nb * nb) % world == 0 or world == 1
        assert max(loads) <= sum(loads) / world * (1 + 1e-3), (world, loads)
        # weak scaling: per-rank work stays within 1/8 of the 1-GPU work at N = 2, 4, 8
        if world in (2, 4, 8):
            assert sum(loads) / world <= sum(loads_1) * 1.126, (world, loads)
        if world == 1:
            loads_1 = loads


# ------------------------------------------------------------------------------------
# compiled programs (csrc/net_programs.h, tools/gen_net_programs.py)
# ------------------------------------------------------------------------------------
def _stage_program_ids(name, dt):
    import importlib
    from cnn_gp import netplan
    cfg = importlib.import_module(f"configs.{name}")
    m = cfg.initial_model.to(dt)
    side = 32 if getattr(cfg, "in_channels", 1) == 3 else 28
    plan = m._plan(side, side)
    itemsize = torch.tensor([], dtype=dt).element_size()
    net = m._net_plan(plan, itemsize)
    dummy = torch.zeros(8, dtype=torch.float64)
    var = {v: (dummy, dummy) for v in net.need_var}
    ids = []
    for st in net.stages:
        arr = net._ops_array(st, var, dummy, dummy)
        flags = N.CGP_FLAG_NET_DUAL if st.dual else 0
        ids.append(N.load().cgp_net_program(ctypes.byref(arr), st.n_ops, st.pairs, flags,
                                            st.lds_elems, itemsize))
    return ids, net


@pytest.mark.parametrize("name", ["mnist_paper_convnet_gp", "mnist_paper_residual_cnn_gp",
                                  "mnist_as_tf", "cifar10"])
@pytest.mark.parametrize("dt", [torch.float64, torch.float32])
def test_reference_configs_have_compiled_programs(name, dt):
    """net_programs.h is in sync with NetPlan's lowering: every stage of every reference
    config finds its compiled program (a stale header would silently fall back to the
    interpreter; rerun tools/gen_net_programs.py)"""
    ids, _ = _stage_program_ids(name, dt)
    assert all(i > 0 for i in ids), ids
    assert len(set(ids)) == len(ids)


def test_program_match_ignores_weights_but_not_structure():
    """weights, biases and variance pointers are runtime fields; any structural field
    (here one LDS offset) makes the op list fall back to the interpreter"""
    import importlib
    cfg = importlib.import_module("configs.mnist_paper_convnet_gp")
    m = cfg.initial_model.double()
    net = m._net_plan(m._plan(28, 28), 8)
    st = net.stages[0]
    dummy = torch.zeros(8, dtype=torch.float64)
    var = {v: (dummy, dummy) for v in net.need_var}
    arr = net._ops_array(st, var)
    lib = N.load()
    np_ = st.pairs
    pid = lib.cgp_net_program(ctypes.byref(arr), st.n_ops, np_, 0, st.lds_elems, 8)
    assert pid > 0
    for o in arr:
        o.weight, o.bias = 3.5, 0.25
    assert lib.cgp_net_program(ctypes.byref(arr), st.n_ops, np_, 0, st.lds_elems, 8) == pid
    arr[3].dst += 1
    assert lib.cgp_net_program(ctypes.byref(arr), st.n_ops, np_, 0, st.lds_elems, 8) == 0
    arr[3].dst -= 1
    # other pair count, dual flag, footprint or item size: no program
    assert lib.cgp_net_program(ctypes.byref(arr), st.n_ops, 4 if np_ != 4 else 1, 0, st.lds_elems, 8) == 0
    assert lib.cgp_net_program(ctypes.byref(arr), st.n_ops, np_, N.CGP_FLAG_NET_DUAL,
                               st.lds_elems, 8) == 0
    assert lib.cgp_net_program(ctypes.byref(arr), st.n_ops, np_, 0, st.lds_elems + 2, 8) == 0
    assert lib.cgp_net_program(ctypes.byref(arr), st.n_ops - 1, np_, 0, st.lds_elems, 8) == 0


def test_tensor_rows_equals_dataloader_collation():
    """ProductIterator's sliced batches (data.tensor_rows) are exactly what the
    reference's DataLoader collation of the same Subset yields (data.py:36-96), for the
    dataset shapes DatasetFromConfig builds (Subset of a ConcatDataset, across the
    train/test boundary) and for index lists; other datasets fall back to the DataLoader."""
    from torch.utils.data import ConcatDataset, DataLoader, Subset, TensorDataset
    from cnn_gp.data import ProductIterator, tensor_rows
    g = torch.Generator().manual_seed(0)
    a = TensorDataset(torch.rand((50, 1, 4, 4), generator=g), torch.arange(50))
    b = TensorDataset(torch.rand((30, 1, 4, 4), generator=g), torch.arange(100, 130))
    cat = ConcatDataset([a, b])

    def ref(ds, lo, hi):
        return next(iter(DataLoader(Subset(ds, range(lo, hi)), batch_size=hi - lo)))
    cases = [(a, 0, 50), (a, 7, 19), (cat, 40, 60), (cat, 50, 80), (cat, 0, 80),
             (Subset(cat, range(45, 75)), 3, 17), (Subset(a, [3, 1, 4, 1, 5]), 1, 4)]
    for ds, lo, hi in cases:
        got, want = tensor_rows(ds, lo, hi), ref(ds, lo, hi)
        assert len(got) == len(want) == 2
        for x, y in zip(got, want):
            assert x.dtype == y.dtype and torch.equal(x, y)

    class Plain(torch.utils.data.Dataset):
        def __len__(self):
            return 5

        def __getitem__(self, k):
            return torch.full((1, 2, 2), float(k)), k
    assert tensor_rows(Plain(), 0, 5) is None
    for ds in (cat, Plain()):
        for same, (i, x), (j, x2) in ProductIterator(16, ds, None):
            want = ref(ds, i, min(i + 16, len(ds)))[0]
            assert torch.equal(x[0], want)


@pytest.mark.parametrize("name", ["mnist_paper_convnet_gp", "mnist_as_tf", "cifar10"])
@pytest.mark.parametrize("dt", [torch.float64, torch.float32])
def test_op_record_template_equals_records_built_per_call(name, dt):
    """NetPlan.prepare writes each forward's op records from a cached template plus the
    variance / state pointers (_ops_template): byte-identical to building every record
    field by field (_ops_array), and the same compiled program id"""
    ids, net = _stage_program_ids(name, dt)
    itemsize = torch.tensor([], dtype=dt).element_size()
    # distinct fake maps per value and side, distinct state buffers
    var = {v: (torch.empty(4 + 2 * k), torch.empty(5 + 2 * k))
           for k, v in enumerate(sorted(net.need_var))}
    states = [torch.empty(7 + k) for k in range(len(net.stages) + 1)]
    for sidx, st in enumerate(net.stages):
        flags = 0
        tmpl, slots, what, program = net._ops_template(sidx, st, flags, itemsize)
        ptrs = [var[w[0]][w[1]].data_ptr() if isinstance(w, tuple) else
                (states[sidx] if w == "in" else states[sidx + 1]).data_ptr() for w in what]
        buf = tmpl.copy()
        buf.view("<u8")[slots] = ptrs
        ref = net._ops_array(st, var, states[sidx], states[sidx + 1])
        assert bytes(buf) == bytes(ref)
        assert program == ids[sidx]


def test_diag_iterator_batches_equal_dataloader():
    from torch.utils.data import ConcatDataset, DataLoader, Subset, TensorDataset
    from cnn_gp.data import DiagIterator
    g = torch.Generator().manual_seed(1)
    a = TensorDataset(torch.rand((37, 1, 3, 3), generator=g), torch.arange(37))
    b = TensorDataset(torch.rand((20, 1, 3, 3), generator=g), torch.arange(20))
    X = Subset(ConcatDataset([a, b]), range(10, 50))
    Y = Subset(ConcatDataset([a, b]), range(0, 40))
    for X2 in (None, Y):
        got = list(DiagIterator(16, X, X2))
        ref = list(zip(DataLoader(X, batch_size=16), DataLoader(X2 if X2 is not None else X,
                                                                batch_size=16)))
        assert len(got) == len(ref) == 3
        for (same, (i, xy), (j, xy2)), (rx, ry) in zip(got, ref):
            assert same == (X2 is None) and i == j
            assert torch.equal(xy[0], rx[0]) and torch.equal(xy2[0], ry[0])
            assert torch.equal(xy[1], rx[1])


def test_empty_batches_return_empty_results():
    """An empty image batch on either side gives the empty [N1, N2] (or [N1] diag) result,
    as the reference's torch ops do (kernels.py:18-57 run on a zero-size batch; checked
    against the reference in the build container: shapes (0, 3), (3, 0), (0, 0), (0,),
    float64) — nothing is evaluated, so no device is needed."""
    import importlib
    m = importlib.import_module("configs.mnist_as_tf").initial_model.double()
    e = torch.zeros((0, 1, 28, 28), dtype=torch.float64)
    x = torch.rand((3, 1, 28, 28), dtype=torch.float64)
    for args, shape in [((e, x, False, False), (0, 3)), ((x, e, False, False), (3, 0)),
                        ((e,), (0, 0)), ((e, e, True, True), (0,))]:
        r = m(*args)
        assert tuple(r.shape) == shape and r.dtype == torch.float64 and r.device == e.device


def test_conv_geometry_refuses_a_non_constant_kernel():
    """the device kernels run the reference's constant box kernel (kernels.py:75-87): an
    edited buffer of any other shape or value raises instead of being read at one tap"""
    import torch
    import cnn_gp
    from cnn_gp.program import conv_geometry
    for k in (3, 4):
        c = cnn_gp.Conv2d(k, var_weight=2.0)
        geo = conv_geometry(c)
        assert geo.weight == float(torch.tensor(2.0 / k ** 2, dtype=torch.float32))
        c.kernel.mul_(2)                          # still a constant box: accepted
        assert conv_geometry(c).weight == 2 * geo.weight
        bad = cnn_gp.Conv2d(k)
        bad.kernel[0, 0, -1, -1] += 1.0
        with pytest.raises(NotImplementedError):
            conv_geometry(bad)
    even = cnn_gp.Conv2d(4)
    even.kernel[0, 0, 0, 0] = 1.0                 # the zero row of an even 'same' kernel
    with pytest.raises(NotImplementedError):
        conv_geometry(even)


def test_tensor_rows_exact_classes_and_mixed_concat():
    """a TensorDataset subclass with its own __getitem__ goes through the DataLoader (its
    transform applies); a ConcatDataset mixing a TensorDataset with another dataset type
    yields the DataLoader's batches, never None"""
    from torch.utils.data import ConcatDataset, DataLoader, Dataset, TensorDataset
    from cnn_gp.data import DiagIterator, tensor_rows

    class Doubled(TensorDataset):
        def __getitem__(self, i):
            x, y = super().__getitem__(i)
            return 2 * x, y

    class Plain(Dataset):
        def __init__(self, x, y):
            self.x, self.y = x, y

        def __len__(self):
            return len(self.x)

        def __getitem__(self, i):
            return self.x[i], self.y[i]

    x = torch.arange(24, dtype=torch.float64).reshape(6, 1, 2, 2)
    y = torch.arange(6)
    assert tensor_rows(Doubled(x, y), 0, 3) is None
    d = Doubled(x, y)
    got = [b for _, (_, b), _ in DiagIterator(4, d)]
    want = list(DataLoader(d, batch_size=4))
    assert all(torch.equal(a[0], b[0]) and torch.equal(a[1], b[1]) for a, b in zip(got, want))
    mixed = ConcatDataset([TensorDataset(x[:3], y[:3]), Plain(x[3:], y[3:])])
    got = [b for _, (_, b), _ in DiagIterator(2, mixed)]
    assert len(got) == 3 and all(b is not None for b in got)
    assert torch.equal(torch.cat([b[0] for b in got]), x)


@pytest.mark.parametrize("overlap", [2, 3, 5])
def test_save_K_overlap_writes_the_serial_files(overlap):
    """tiles in flight on helper threads (save_K's default overlap = 2): the same dataset
    as the serial reference loop, tiles written in the reference's order, and the first
    failing tile's FloatingPointError raised with nothing written after it"""
    import threading
    rng = np.random.default_rng(3)
    X = torch.from_numpy(rng.random((37, 1, 4, 4)))
    ds = torch.utils.data.TensorDataset(X, torch.zeros(len(X)))
    threads = set()

    def kern(x, x2, same, diag):
        threads.add(threading.get_ident())
        k = (x.reshape(len(x), -1) @ x2.reshape(len(x2), -1).T).numpy()
        return np.diag(k).copy() if diag else k

    ref, got = FakeFile(), FakeFile()
    save_K(ref, kern, "Kxx", ds, None, False, 8, print_interval=1e9, overlap=1)
    save_K(got, kern, "Kxx", ds, None, False, 8, print_interval=1e9, overlap=overlap)
    np.testing.assert_array_equal(got.d["Kxx"].a, ref.d["Kxx"].a)
    assert len(threads) > 1
    writes = []

    class Rec(FakeFile):
        def create_dataset(self, *a, **k):
            ds_ = super().create_dataset(*a, **k)
            orig = ds_.__class__.__setitem__

            class W(ds_.__class__):
                def __setitem__(self, key, v):
                    writes.append((key[1].start, key[2].start))
                    orig(self, key, v)
            ds_.__class__ = W
            return ds_

    def bad(x, x2, same, diag):
        k = kern(x, x2, same, diag)
        if x[0, 0, 0, 0] == X[16, 0, 0, 0]:          # the tiles of row block 2
            k[0, 0] = np.nan
        return k

    with pytest.raises(FloatingPointError, match="16,16"):
        save_K(Rec(), bad, "Kxx", ds, None, False, 8, print_interval=1e9, overlap=overlap)
    order = [(0, 0), (0, 8), (0, 16), (0, 24), (0, 32), (8, 8), (8, 16), (8, 24), (8, 32)]
    assert writes == order


def test_save_K_overlap_kern_error_surfaces_in_order():
    """an exception inside a kern call on a helper thread reaches the caller at that tile's
    turn; earlier tiles are written, later ones are not"""
    rng = np.random.default_rng(5)
    X = torch.from_numpy(rng.random((30, 1, 3, 3)))
    ds = torch.utils.data.TensorDataset(X, torch.zeros(len(X)))
    written = []

    class F(FakeFile):
        def create_dataset(self, *a, **k):
            d = super().create_dataset(*a, **k)

            class W(d.__class__):
                def __setitem__(self, key, v):
                    written.append((key[1].start, key[2].start))
                    super().__setitem__(key, v)
            d.__class__ = W
            return d

    def kern(x, x2, same, diag):
        if x[0, 0, 0, 0] == X[10, 0, 0, 0] and x2[0, 0, 0, 0] == X[20, 0, 0, 0]:
            raise ValueError("tile (10, 20) fails")
        return (x.reshape(len(x), -1) @ x2.reshape(len(x2), -1).T).numpy()

    with pytest.raises(ValueError, match="tile \\(10, 20\\)"):
        save_K(F(), kern, "Kxx", ds, None, False, 10, print_interval=1e9, overlap=4)
    assert written == [(0, 0), (0, 10), (0, 20), (10, 10)]


def test_save_K_pin_leaves_datasets_alone_without_a_gpu():
    """save_K(pin=True) on a host without a GPU: every dataset kind is handed on as it is
    (the page-locked copy is only made when a device will read the batches)"""
    from torch.utils.data import ConcatDataset, Subset, TensorDataset
    from cnn_gp.kernel_save_tools import _pinned
    X = torch.rand((6, 1, 4, 4))
    base = TensorDataset(X, torch.zeros(6))
    for ds in (base, Subset(base, range(1, 5)), ConcatDataset([base, base]), [X[i] for i in range(6)]):
        if torch.cuda.is_available():
            pytest.skip("a GPU is visible")
        assert _pinned(ds) is ds
