"""The multi-GPU assembly path and the HDF5 tile writer with the DEVICE model as ``kern``.

* World size 2, one process per rank (gloo ranks sharing the one GPU of the test box —
  RCCL needs one rank per GPU; 8-GPU RCCL runs are the driver's): every rank evaluates its
  tiles with the HIP kernel into a flat device buffer (``gram_local``), rank 0 gathers them
  (``gather_gram``, one collective, staged through host memory under gloo) and the result
  must be BIT-equal to the single-process device matrix, NaN lower triangle included.
  Both worker splits (the reference's by tile count, data.py:11-19; the build's by
  evaluated pairs).  Reference: exp_mnist_resnet/run.bash:28-43 + merge_h5_files.py:24-30.
* ``save_K`` (kernel_save_tools.py:26-58) driven by save_kernel.py:21-24's ``kern`` on the
  device model, for 1 and 3 workers, then ``merge_nan_fill``: NaN mask and float32 values
  against the reference's own files (tests/golden/tiles.npz).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

import configs_util
from conftest import GOLDEN

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _images(n, seed):
    g = torch.Generator().manual_seed(seed)
    return torch.rand((n, 1, 28, 28), generator=g, dtype=torch.float64)


def _rank_main(rank, world, port, q):
    import sys
    from conftest import PKG, ROOT
    sys.path[:0] = [PKG, ROOT]
    import torch.distributed as dist
    from cnn_gp import gram
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    res = {}
    try:
        torch.cuda.set_device(0)
        m = configs_util.model("mnist_paper_convnet_gp").to("cuda", torch.float64)
        X = _images(300, 3).cuda()
        Z = _images(130, 4).cuda()
        B = 64
        kern = gram.model_kern(m)
        for split in ("balanced", "reference"):
            for name, X2 in (("Kxx", None), ("Kxz", Z)):
                n2 = None if X2 is None else len(X2)
                if split == "balanced":
                    full = gram.gram_matrix(m, X, X2, batch_size=B)
                else:
                    buf, tiles = gram.gram_local(kern, X, X2, B, rank, world, split=split)
                    assert buf.device.type == "cuda"
                    assert buf.numel() == sum(a * b for *_, a, b in tiles)
                    full = gram.gather_gram(buf, len(X), n2, B, split=split)
                if rank != 0:
                    assert full is None
                    continue
                assert full.device.type == "cuda"
                single, _ = gram.gram_tiles(kern, X, X2, B)
                nan_a, nan_b = torch.isnan(full), torch.isnan(single)
                res[(split, name)] = (bool(torch.equal(nan_a, nan_b)),
                                      bool(torch.equal(full[~nan_a], single[~nan_b])),
                                      int(nan_a.sum()))
        dist.barrier()
    finally:
        dist.destroy_process_group()
    if rank == 0:
        q.put(res)


def test_world2_gather_on_device_bit_equal_to_single_process():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        res = q.get(timeout=240)
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    for p in procs:
        assert p.exitcode == 0
    assert len(res) == 4, res
    for key, (nan_same, vals_equal, n_nan) in res.items():
        assert nan_same and vals_equal, key
        # Kxx: the strictly-lower off-diagonal 64-tiles stay NaN (reference layout)
        if key[1] == "Kxx":
            nb = -(-300 // 64)
            full_tiles_lower = sum(min(64, 300 - 64 * i) * min(64, 300 - 64 * j)
                                   for i in range(nb) for j in range(i))
            assert n_nan == full_tiles_lower, key
        else:
            assert n_nan == 0


class _FakeDS:
    def __init__(self, shape, dtype, fillvalue, chunks, maxshape):
        self.a = np.full(shape, fillvalue, dtype=dtype)
        self.chunks, self.maxshape, self.shape = chunks, maxshape, shape

    def __setitem__(self, k, v):
        self.a[k] = v

    def __getitem__(self, k):
        return self.a[k]

    def __len__(self):
        return len(self.a)


class _FakeFile:
    """the h5py.File surface save_K uses: keys(), create_dataset(...), slice assignment"""

    def __init__(self):
        self.d = {}

    def keys(self):
        return self.d.keys()

    def create_dataset(self, name, shape, dtype, fillvalue, chunks, maxshape):
        self.d[name] = _FakeDS(shape, dtype, fillvalue, chunks, maxshape)
        return self.d[name]


@pytest.mark.parametrize("n_workers", [1, 3])
def test_save_K_with_device_kern_matches_reference_files(n_workers):
    from cnn_gp import merge_nan_fill, save_K
    z = np.load(os.path.join(GOLDEN, "tiles.npz"))
    X, Z = z["X"].astype(np.float64), z["Z"].astype(np.float64)
    dsx = torch.utils.data.TensorDataset(torch.from_numpy(X), torch.zeros(len(X)))
    dsz = torch.utils.data.TensorDataset(torch.from_numpy(Z), torch.zeros(len(Z)))
    model = configs_util.model("mnist_paper_convnet_gp").double().cuda()
    calls = []

    def kern(x, x2, same, diag):                       # save_kernel.py:21-24
        with torch.no_grad():
            k = model(x.cuda(), x2.cuda(), same, diag)
            calls.append(k.device.type)
            return k.detach().cpu().numpy()

    files = []
    for r in range(n_workers):
        f = _FakeFile()
        save_K(f, kern, "Kxx", dsx, None, False, 16, worker_rank=r, n_workers=n_workers,
               print_interval=1e9)
        save_K(f, kern, "Kxz", dsx, dsz, False, 16, worker_rank=r, n_workers=n_workers,
               print_interval=1e9)
        for name in ("Kxx", "Kxz"):
            ref = z[f"{name}_nw{n_workers}_r{r}"]
            got = f.d[name].a
            assert got.dtype == np.float32
            np.testing.assert_array_equal(np.isnan(got), np.isnan(ref))
            m = ~np.isnan(ref)
            np.testing.assert_allclose(got[m], ref[m], rtol=1e-6, atol=0)
        assert f.d["Kxx"].chunks == tuple(z[f"Kxx_chunks_nw{n_workers}"])
        files.append(f)
    assert calls and set(calls) == {"cuda"}
    for name in ("Kxx", "Kxz"):
        merged = merge_nan_fill(files[0].d[name].a.copy(), [f.d[name].a for f in files[1:]])
        ref1 = z[f"{name}_nw1_r0"]
        np.testing.assert_array_equal(np.isnan(merged), np.isnan(ref1))
        m = ~np.isnan(ref1)
        np.testing.assert_allclose(merged[m], ref1[m], rtol=1e-6, atol=0)
    f = _FakeFile()
    save_K(f, kern, "Kx_diag", dsx, None, True, 16, print_interval=1e9)
    np.testing.assert_allclose(f.d["Kx_diag"].a, z["Kx_diag"], rtol=1e-6, atol=0)
    assert f.d["Kx_diag"].chunks == tuple(z["Kx_diag_chunks"])


def _pipeline_rank(rank, world, port, q, backend="gloo"):
    """cnn_gp.pipeline.classify_distributed with the HIP model, rocSOLVER and the device
    score product: world 1 in-process (rank None) or one rank of a world — gloo ranks
    share GPU 0, nccl (RCCL) ranks run one per GPU"""
    import sys
    from conftest import PKG, ROOT
    sys.path[:0] = [PKG, ROOT]
    import torch.distributed as dist
    import cnn_gp
    from cnn_gp import gram
    from cnn_gp.pipeline import classify_distributed
    if world > 1:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
    dev = rank if backend == "nccl" else 0
    torch.cuda.set_device(dev)
    if world > 1:
        from datetime import timedelta
        kw = {"device_id": torch.device("cuda", dev)} if backend == "nccl" else {}
        dist.init_process_group(backend, rank=rank, world_size=world,
                                timeout=timedelta(seconds=120), **kw)
    try:
        m = configs_util.model("mnist_as_tf").to("cuda", torch.float64)
        X = _images(200, 5).cuda()
        Z = _images(70, 6).cuda()
        g = torch.Generator().manual_seed(7)
        Y = cnn_gp.one_hot_pm1(torch.randint(0, 10, (200,), generator=g), 10)

        def solve(K, Yd):
            return cnn_gp.solve_system(K, Yd, overwrite_a=True)

        with torch.no_grad():
            res = classify_distributed(gram.model_kern(m), X, Z, Y, solve, cnn_gp.scores,
                                       batch_size=48, gather_kxz=True, jitter=1e-6)
        out = None
        if (rank or 0) == 0:
            # numpy: pickled by value (a torch tensor on an mp queue travels as a shared
            # memory handle, which dies with this process)
            out = {k: res[k].cpu().numpy() for k in ("alpha", "pred", "scores", "Kxz")}
            out["peak_gather_solve"] = res["peak_bytes_gather_solve"]
            out["plan_kxx"] = res["plan_kxx"]
        if world > 1:
            dist.barrier()
    finally:
        if world > 1:
            dist.destroy_process_group()
    if q is None:
        return out
    if rank == 0:
        q.put(out)


def _world2_pipeline(backend):
    single = _pipeline_rank(None, 1, None, None)
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_pipeline_rank, args=(r, world, port, q, backend))
             for r in range(world)]
    for p in procs:
        p.start()
    try:
        res = q.get(timeout=240)
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    for p in procs:
        assert p.exitcode == 0
    assert len(res["plan_kxx"]) == 2
    assert np.array_equal(res["alpha"], single["alpha"])
    assert np.array_equal(res["pred"], single["pred"])
    assert np.array_equal(res["Kxz"], single["Kxz"])
    np.testing.assert_allclose(res["scores"], single["scores"], rtol=1e-12, atol=1e-12)
    print(f"{backend}: rank-0 device peak in the gather + solve: "
          f"{res['peak_gather_solve'] / 1e6:.1f} MB (Kxx {200 * 200 * 8 / 1e6:.2f} MB)")


def test_world2_pipeline_on_device_matches_single_process():
    """Row strips of Kxx gathered point-to-point, solve on rank 0 while rank 1 builds its
    Kxz rows, α broadcast, scores gathered: α and the predicted labels bit-equal to the
    one-process run, Kxz (gathered on request) bit-equal too (two gloo ranks sharing the
    GPU)"""
    _world2_pipeline("gloo")


@pytest.mark.skipif(torch.cuda.device_count() < 2, reason="RCCL ranks need two GPUs")
def test_world2_nccl_pipeline_matches_single_process():
    """The same over RCCL, one rank per GPU: batch_isend_irecv of the Kxx strips, the
    device all_reduce of the phase times, the broadcast of the solve status and of α"""
    _world2_pipeline("nccl")
