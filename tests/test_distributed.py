"""Multi-process Gram assembly on CPU (gloo, world size 2 and 3): each rank evaluates its
reference-split tiles with the oracle as ``kern``; rank 0 gathers and must reproduce the
single-process matrix, including the NaN lower triangle of Kxx."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import nngp_oracle as O
from oracle import specs


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, X, Z, B, q):
    import sys
    from conftest import PKG, ROOT
    sys.path[:0] = [PKG, ROOT]
    from cnn_gp.gram import gram_tiles, gather_gram
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    spec = specs.mnist_paper_convnet_gp()

    def kern(x, x2, same):
        return torch.from_numpy(O.kernel(spec, x.numpy(), x2.numpy(), same, False))

    try:
        res = {}
        for name, X2 in (("Kxx", None), ("Kxz", Z)):
            local, _ = gram_tiles(kern, X, X2, B, rank, world)
            full = gather_gram(local, len(X), None if X2 is None else len(X2), B)
            if rank == 0:
                res[name] = full.numpy()
        if rank == 0:
            q.put(res)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_gather_matches_single_process(world):
    rng = np.random.default_rng(0)
    X = torch.from_numpy(rng.random((11, 1, 28, 28)))
    Z = torch.from_numpy(rng.random((7, 1, 28, 28)))
    B = 4
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, X, Z, B, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    spec = specs.mnist_paper_convnet_gp()
    ref_xx = O.gram_tiles(spec, X.numpy(), None, B)[0]
    ref_xz = O.gram_tiles(spec, X.numpy(), Z.numpy(), B)[0]
    for got, ref in ((res["Kxx"], ref_xx), (res["Kxz"], ref_xz)):
        np.testing.assert_array_equal(np.isnan(got), np.isnan(ref))
        m = ~np.isnan(ref)
        np.testing.assert_allclose(got[m], ref[m], rtol=1e-6)   # ref file is float32


def test_single_process_gram_tiles_matches_oracle():
    import sys
    from conftest import PKG
    sys.path.insert(0, PKG)
    from cnn_gp.gram import gram_tiles
    rng = np.random.default_rng(1)
    X = torch.from_numpy(rng.random((9, 1, 28, 28)))
    spec = specs.mnist_paper_convnet_gp()

    def kern(x, x2, same):
        return torch.from_numpy(O.kernel(spec, x.numpy(), x2.numpy(), same, False))

    out, tiles = gram_tiles(kern, X, None, 4)
    assert [t[:3] for t in tiles] == [(True, 0, 0), (False, 0, 4), (False, 0, 8),
                                      (True, 4, 4), (False, 4, 8), (True, 8, 8)]
    full = O.kernel(spec, X.numpy())
    iu = np.triu_indices(9)
    np.testing.assert_allclose(out.numpy()[iu], full[iu], rtol=1e-12)
    # strictly-lower off-diagonal tiles stay NaN (reference layout)
    assert np.isnan(out.numpy()[4:, :4]).all()
