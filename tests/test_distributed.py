"""Multi-process Gram assembly on CPU (gloo, world size 2 and 3): each rank evaluates its
tiles with the oracle as ``kern`` (test infrastructure standing in for the device model;
the GPU variant is tests/test_gpu_multi.py); rank 0 gathers and must reproduce the
single-process matrix, including the NaN lower triangle of Kxx.  Both worker splits: the
reference's contiguous split by tile count (data.py:11-19) and the build's split by
evaluated pairs."""
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
    from cnn_gp.gram import gram_tiles, gram_local, gather_gram
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    spec = specs.mnist_paper_convnet_gp()

    def kern(x, x2, same):
        return torch.from_numpy(O.kernel(spec, x.numpy(), x2.numpy(), same, False))

    try:
        res = {}
        for name, X2 in (("Kxx", None), ("Kxz", Z)):
            n2 = None if X2 is None else len(X2)
            # legacy: a full matrix per rank, reference split
            local, _ = gram_tiles(kern, X, X2, B, rank, world, device="cpu",
                                  split="reference")
            full = gather_gram(local, len(X), n2, B, split="reference")
            # a matrix needs its split named; one filled by another plan is refused
            with pytest.raises(ValueError):
                gather_gram(local, len(X), n2, B)
            if world == 3 and rank == 2 and X2 is None:   # its plans differ (4, 4)
                with pytest.raises(ValueError, match="not finite"):
                    gather_gram(local, len(X), n2, B, split="balanced")
            # packed: only this rank's tiles, balanced split
            buf, tiles = gram_local(kern, X, X2, B, rank, world, device="cpu")
            assert buf.numel() == sum(a * b for *_, a, b in tiles)
            full2 = gather_gram(buf, len(X), n2, B)
            if rank == 0:
                res[name] = full.numpy()
                res[name + "_packed"] = full2.numpy()
            else:
                assert full is None and full2 is None
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
    for key, ref in (("Kxx", ref_xx), ("Kxz", ref_xz)):
        for got in (res[key], res[key + "_packed"]):
            np.testing.assert_array_equal(np.isnan(got), np.isnan(ref))
            m = ~np.isnan(ref)
            np.testing.assert_allclose(got[m], ref[m], rtol=1e-6)   # ref file is float32
        np.testing.assert_array_equal(res[key], res[key + "_packed"])


def test_single_process_gram_tiles_matches_oracle():
    from cnn_gp.gram import gram_tiles
    rng = np.random.default_rng(1)
    X = torch.from_numpy(rng.random((9, 1, 28, 28)))
    spec = specs.mnist_paper_convnet_gp()

    def kern(x, x2, same):
        return torch.from_numpy(O.kernel(spec, x.numpy(), x2.numpy(), same, False))

    out, tiles = gram_tiles(kern, X, None, 4, device="cpu")
    assert [t[:3] for t in tiles] == [(True, 0, 0), (False, 0, 4), (False, 0, 8),
                                      (True, 4, 4), (False, 4, 8), (True, 8, 8)]
    full = O.kernel(spec, X.numpy())
    iu = np.triu_indices(9)
    np.testing.assert_allclose(out.numpy()[iu], full[iu], rtol=1e-12)
    # strictly-lower off-diagonal tiles stay NaN (reference layout)
    assert np.isnan(out.numpy()[4:, :4]).all()


@pytest.mark.parametrize("N,N2,B,world", [(60000, None, 4096, 8), (10000, 60000, 4096, 8),
                                         (10000, 60000, 1024, 8), (4096, None, 1024, 3),
                                         (11, 7, 4, 3), (1, None, 4, 2), (9, None, 4, 8)])
def test_balanced_split_partitions_and_balances(N, N2, B, world):
    """every tile exactly once, each rank's share contiguous in the reference order, and
    the evaluated pairs per rank within one tile of the mean"""
    from cnn_gp.gram import tile_cost, tile_plan
    every = tile_plan(N, N2, B, 0, 1)
    parts = [tile_plan(N, N2, B, r, world) for r in range(world)]
    flat = [t for p in parts for t in p]
    assert flat == every                                  # contiguous, in order, complete
    loads = [sum(tile_cost(t) for t in p) for p in parts]
    biggest = max(tile_cost(t) for t in every)
    mean = sum(loads) / world
    assert max(loads) - mean <= biggest and mean - min(loads) <= biggest
    ref = [tile_plan(N, N2, B, r, world, split="reference") for r in range(world)]
    assert [t for p in ref for t in p] == every
    if (N, N2, B) == (10000, 60000, 4096):
        # the case the reference split leaves ≈20% apart
        rl = [sum(tile_cost(t) for t in p) for p in ref]
        assert max(rl) / min(rl) > 1.19 and max(loads) / min(loads) < max(rl) / min(rl)
