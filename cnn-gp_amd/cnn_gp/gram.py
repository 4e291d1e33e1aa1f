"""Device-resident Gram matrices and their multi-GPU assembly.

``save_K`` (kernel_save_tools.py) mirrors the reference's per-tile HDF5 writer.  For the
GP solve the build keeps the matrix on the device instead: ``gram_tiles`` evaluates this
worker's tiles (the reference's tile order and contiguous balanced worker split,
cnn_gp/data.py:11-96) straight into a NaN-filled device matrix, and ``gather_gram``
assembles every worker's tiles on rank 0 with ONE collective (torch.distributed ``gather``
— RCCL over xGMI with the nccl backend, gloo on CPU), replacing the reference's per-worker
HDF5 files + NaN merge (exp_mnist_resnet/run.bash:28-43, merge_h5_files.py:24-30).

Kxx keeps the reference's layout: upper-triangular tiles filled, strictly-lower tiles NaN
(solve_system reads only the upper triangle).  Kxz (X2 given): every tile; with the
contiguous split each rank owns a band of row blocks of X against all of Z.
"""
from __future__ import annotations

from typing import Callable, Optional

import torch
import torch.distributed as dist

from .data import tile_schedule

__all__ = ("gram_tiles", "gather_gram", "gram_matrix", "model_kern")


def _rows(X, lo, hi):
    """Images lo:hi of X — a tensor, a TensorDataset-like (first tensor) or a Dataset."""
    if isinstance(X, torch.Tensor):
        return X[lo:hi]
    if hasattr(X, "tensors"):
        return X.tensors[0][lo:hi]
    return torch.stack([X[k][0] for k in range(lo, hi)])


def model_kern(model, device=None, dtype=None) -> Callable:
    """kern(x, x2, same) -> device tensor: the model evaluated on the device."""
    def kern(x, x2, same):
        dev = device if device is not None else torch.device("cuda", torch.cuda.current_device())
        xd = x.to(dev, dtype or x.dtype)
        with torch.no_grad():
            if same:
                return model(xd)
            return model(xd, x2.to(dev, dtype or x2.dtype), False, False)
    return kern


def gram_tiles(kern: Callable, X, X2=None, batch_size: int = 1024, worker_rank: int = 0,
               n_workers: int = 1, out: Optional[torch.Tensor] = None, device=None,
               dtype=torch.float64):
    """Evaluate this worker's tiles into ``out`` ([N, N2], NaN where not computed).

    Returns (out, tiles) where tiles is the list of (same, i0, j0, n_i, n_j) written."""
    N = len(X)
    N2 = N if X2 is None else len(X2)
    src2 = X if X2 is None else X2
    if out is None:
        out = torch.full((N, N2), float("nan"), dtype=dtype, device=device)
    done = []
    for same, bi, bj in tile_schedule(N, None if X2 is None else N2, batch_size, worker_rank,
                                      n_workers):
        i0, j0 = bi * batch_size, bj * batch_size
        x = _rows(X, i0, min(i0 + batch_size, N))
        x2 = x if same else _rows(src2, j0, min(j0 + batch_size, N2))
        k = kern(x, x2, same)
        out[i0:i0 + k.shape[0], j0:j0 + k.shape[1]].copy_(k)
        done.append((same, i0, j0, k.shape[0], k.shape[1]))
    return out, done


def gather_gram(local: torch.Tensor, N: int, N2: Optional[int], batch_size: int,
                group=None, dst: int = 0):
    """Assemble every rank's tiles on rank ``dst`` with one gather.

    ``local`` is this rank's [N, N2] matrix from ``gram_tiles`` (tiles filled, the rest
    arbitrary).  Each rank packs its tiles into one flat buffer padded to the largest
    rank's size; rank ``dst`` receives all buffers and unpacks them by the (shared,
    deterministic) tile schedule.  Returns the full matrix on ``dst``, None elsewhere."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    n2 = N if N2 is None else N2

    def sched(r):
        out = []
        for same, bi, bj in tile_schedule(N, N2, batch_size, r, world):
            i0, j0 = bi * batch_size, bj * batch_size
            out.append((i0, j0, min(batch_size, N - i0), min(batch_size, n2 - j0)))
        return out

    sizes = [sum(a * b for _, _, a, b in sched(r)) for r in range(world)]
    cap = max(max(sizes), 1)
    buf = torch.empty(cap, dtype=local.dtype, device=local.device)
    off = 0
    for i0, j0, a, b in sched(rank):
        buf[off:off + a * b].view(a, b).copy_(local[i0:i0 + a, j0:j0 + b])
        off += a * b
    gathered = [torch.empty_like(buf) for _ in range(world)] if rank == dst else None
    dist.gather(buf, gathered, dst=dst, group=group)
    if rank != dst:
        return None
    full = torch.full((N, n2), float("nan"), dtype=local.dtype, device=local.device)
    for r in range(world):
        off = 0
        for i0, j0, a, b in sched(r):
            full[i0:i0 + a, j0:j0 + b].copy_(gathered[r][off:off + a * b].view(a, b))
            off += a * b
    return full


def gram_matrix(model, X, X2=None, batch_size: int = 1024, device=None,
                dtype=torch.float64, group=None):
    """Full Gram matrix of ``model`` on X (× X2) — single GPU, or sharded over the
    torch.distributed group (one process per GPU) and gathered on rank 0."""
    kern = model_kern(model, device)
    N = len(X)
    N2 = None if X2 is None else len(X2)
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        rank, world = dist.get_rank(group), dist.get_world_size(group)
        local, _ = gram_tiles(kern, X, X2, batch_size, rank, world, device=device, dtype=dtype)
        return gather_gram(local, N, N2, batch_size, group)
    out, _ = gram_tiles(kern, X, X2, batch_size, device=device, dtype=dtype)
    return out
