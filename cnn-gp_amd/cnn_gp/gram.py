"""Device-resident Gram matrices and their multi-GPU assembly.

``save_K`` (kernel_save_tools.py) mirrors the reference's per-tile HDF5 writer.  For the
GP solve the build keeps the matrix on the device instead:

* ``gram_tiles`` evaluates a worker's tiles (the reference's tile order,
  cnn_gp/data.py:22-29) straight into a NaN-filled device matrix (single process);
* ``gram_local`` evaluates a rank's tiles into ONE flat device buffer, tile after tile,
  so a rank holds only its share (1/world of the tiles, not an N×N2 matrix);
* ``gather_gram`` assembles every rank's buffer on rank ``dst`` with ONE collective
  (torch.distributed ``gather`` — RCCL over xGMI with the nccl backend; gloo stages
  through host memory), replacing the reference's per-worker HDF5 files + NaN merge
  (exp_mnist_resnet/run.bash:28-43, merge_h5_files.py:24-30).

Kxx keeps the reference's layout: upper-triangular tiles filled, strictly-lower tiles NaN
(solve_system reads only the upper triangle).  Kxz (X2 given): every tile, row blocks of X
against all of Z.

Worker split.  ``split="reference"`` is the reference's contiguous split by tile count
(data.py:11-19) — what the HDF5 worker files of run.bash use.  ``split="balanced"`` (the
default here) keeps each rank's tiles contiguous in the same order but cuts the list
where the cumulative *evaluated pairs* reach r/world of the total: the kernel evaluates
only i < j on a diagonal tile (half an off-diagonal one) and ragged edge tiles are
smaller, so equal tile counts are unequal work (at 10 000 × 60 000 with B = 4096, 45
tiles over 8 ranks is 6 vs 5 tiles, ≈20% apart).
"""
from __future__ import annotations

from typing import Callable, List, Optional, Tuple

import torch
import torch.distributed as dist

from .data import _ceil_div, _tile_order, tile_schedule

__all__ = ("gram_tiles", "gram_local", "gather_gram", "gram_matrix", "model_kern",
           "tile_plan", "tile_cost")

Tile = Tuple[bool, int, int, int, int]       # (same, i0, j0, rows, cols)


def _rows(X, lo, hi):
    """Images lo:hi of X — a tensor, a TensorDataset-like (first tensor) or a Dataset."""
    if isinstance(X, torch.Tensor):
        return X[lo:hi]
    if hasattr(X, "tensors"):
        return X.tensors[0][lo:hi]
    return torch.stack([X[k][0] for k in range(lo, hi)])


def _default_device(device):
    if device is not None:
        return torch.device(device)
    if not torch.cuda.is_available():
        raise RuntimeError("cnn_gp.gram needs a HIP device (there is no CPU path)")
    return torch.device("cuda", torch.cuda.current_device())


def model_kern(model, device=None, dtype=None) -> Callable:
    """kern(x, x2, same) -> device tensor: the model evaluated on the device."""
    def kern(x, x2, same):
        dev = _default_device(device)
        xd = x.to(dev, dtype or x.dtype)
        with torch.no_grad():
            if same:
                return model(xd)
            return model(xd, x2.to(dev, dtype or x2.dtype), False, False)
    return kern


def tile_cost(t: Tile) -> int:
    """Pairs the device kernel evaluates for a tile: i < j only on a diagonal tile."""
    same, _, _, a, b = t
    return a * (a - 1) // 2 if same else a * b


def tile_plan(N: int, N2: Optional[int], batch_size: int, rank: int = 0, world: int = 1,
              split: str = "balanced") -> List[Tile]:
    """This rank's tiles as (same, i0, j0, rows, cols), in the reference's tile order."""
    if not 0 <= rank < world:
        raise ValueError(f"rank {rank} not in [0, {world})")
    n2 = N if N2 is None else N2

    def sized(same, bi, bj):
        i0, j0 = bi * batch_size, bj * batch_size
        return (same, i0, j0, min(batch_size, N - i0), min(batch_size, n2 - j0))

    if split == "reference":
        return [sized(*t) for t in tile_schedule(N, N2, batch_size, rank, world)]
    if split != "balanced":
        raise ValueError(f"split {split!r}: 'reference' or 'balanced'")
    bx = _ceil_div(N, batch_size)
    bx2 = bx if N2 is None else _ceil_div(n2, batch_size)
    tiles = [sized(*t) for t in _tile_order(bx, bx2, N2 is None)]
    # tile k goes to the rank whose share [r, r+1)·total/world holds the midpoint of its
    # cost interval: monotone in k, so every share is contiguous (cost at least 1, so a
    # one-image diagonal tile still has an owner)
    owner, acc = [], 0
    costs = [max(1, tile_cost(t)) for t in tiles]
    total = sum(costs)
    for c in costs:
        owner.append(min(world - 1, (2 * acc + c) * world // (2 * total)))
        acc += c
    return [t for t, o in zip(tiles, owner) if o == rank]


def _eval_tile(kern, X, src2, t: Tile):
    same, i0, j0, a, b = t
    x = _rows(X, i0, i0 + a)
    x2 = x if same else _rows(src2, j0, j0 + b)
    k = kern(x, x2, same)
    if tuple(k.shape) != (a, b):
        raise RuntimeError(f"kern returned {tuple(k.shape)} for a {a}x{b} tile")
    return k


def gram_tiles(kern: Callable, X, X2=None, batch_size: int = 1024, worker_rank: int = 0,
               n_workers: int = 1, out: Optional[torch.Tensor] = None, device=None,
               dtype=torch.float64, split: str = "balanced"):
    """Evaluate this worker's tiles into ``out`` ([N, N2], NaN where not computed; a new
    device matrix when None).  Returns (out, tiles) with tiles the (same, i0, j0, rows,
    cols) written.  For one process; ranks of a group use ``gram_local``.  ``split`` has
    the same default as ``gram_local`` / ``gather_gram`` (with one worker both splits are
    every tile)."""
    N = len(X)
    N2 = N if X2 is None else len(X2)
    src2 = X if X2 is None else X2
    if out is None:
        out = torch.full((N, N2), float("nan"), dtype=dtype, device=_default_device(device))
    done = tile_plan(N, None if X2 is None else N2, batch_size, worker_rank, n_workers, split)
    for t in done:
        _, i0, j0, a, b = t
        out[i0:i0 + a, j0:j0 + b].copy_(_eval_tile(kern, X, src2, t))
    return out, done


def gram_local(kern: Callable, X, X2=None, batch_size: int = 1024, rank: int = 0,
               world: int = 1, device=None, dtype=torch.float64, split: str = "balanced",
               capacity: Optional[int] = None):
    """This rank's tiles packed into one flat device buffer (tile after tile, each
    row-major), sized ``capacity`` (default: just its own tiles).  Returns (buf, tiles)."""
    N = len(X)
    N2 = None if X2 is None else len(X2)
    src2 = X if X2 is None else X2
    tiles = tile_plan(N, N2, batch_size, rank, world, split)
    need = sum(a * b for _, _, _, a, b in tiles)
    cap = need if capacity is None else capacity
    if cap < need:
        raise ValueError(f"capacity {cap} < {need} elements of rank {rank}'s tiles")
    buf = torch.empty(max(cap, 1), dtype=dtype, device=_default_device(device))
    off = 0
    for t in tiles:
        _, _, _, a, b = t
        buf[off:off + a * b].view(a, b).copy_(_eval_tile(kern, X, src2, t))
        off += a * b
    return buf, tiles


def _capacity(N, N2, batch_size, world, split):
    return max(1, max(sum(a * b for _, _, _, a, b in tile_plan(N, N2, batch_size, r, world,
                                                                  split))
                      for r in range(world)))


def gather_gram(local: torch.Tensor, N: int, N2: Optional[int], batch_size: int,
                group=None, dst: int = 0, split: Optional[str] = None):
    """Assemble every rank's tiles on rank ``dst`` with one gather.

    ``local`` is this rank's flat buffer from ``gram_local`` (split default "balanced",
    as there), or an [N, N2] matrix holding its tiles — packed first, which needs the
    ``split`` the matrix was filled with named explicitly, and every packed tile must be
    finite (a tile of another split's plan would still hold the NaN fill).  Every rank's buffer is
    padded to the largest share; rank ``dst`` unpacks them by the shared, deterministic
    tile plan into a NaN-filled [N, N2] matrix on ``local``'s device and returns it; the
    other ranks return None.  With a gloo group, device buffers travel through host
    memory (gloo's gather takes CPU tensors)."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    n2 = N if N2 is None else N2
    if local.dim() != 2 and split is None:
        split = "balanced"                     # gram_local's default
    plans = [tile_plan(N, N2, batch_size, r, world, split) for r in range(world)]
    cap = max(1, max(sum(a * b for _, _, _, a, b in p) for p in plans))
    if local.dim() == 2:
        if split is None:
            raise ValueError("gather_gram of an [N, N2] matrix: pass the split its tiles "
                             "were evaluated with (gram_tiles(..., split=...))")
        packed = torch.empty(cap, dtype=local.dtype, device=local.device)
        off = 0
        for _, i0, j0, a, b in plans[rank]:
            packed[off:off + a * b].view(a, b).copy_(local[i0:i0 + a, j0:j0 + b])
            off += a * b
        if not bool(torch.isfinite(packed[:off]).all()):
            raise ValueError(f"rank {rank}: a tile of the {split!r} plan is not finite in the "
                             "matrix given — it was filled with another split")
        local = packed
    if local.numel() < cap:
        grown = torch.empty(cap, dtype=local.dtype, device=local.device)
        grown[:local.numel()].copy_(local)
        local = grown
    send = local[:cap]
    staged = local.device.type == "cuda" and dist.get_backend(group) == "gloo"
    if staged:
        send = send.cpu()
    gathered = [torch.empty_like(send) for _ in range(world)] if rank == dst else None
    dist.gather(send, gathered, group=group, group_dst=dst)   # dst: a rank of `group`
    if rank != dst:
        return None
    full = torch.full((N, n2), float("nan"), dtype=local.dtype, device=local.device)
    for r in range(world):
        src = gathered[r].to(local.device) if staged else gathered[r]
        off = 0
        for _, i0, j0, a, b in plans[r]:
            full[i0:i0 + a, j0:j0 + b].copy_(src[off:off + a * b].view(a, b))
            off += a * b
        gathered[r] = None
    return full


def gram_matrix(model, X, X2=None, batch_size: int = 1024, device=None,
                dtype=torch.float64, group=None, split: str = "balanced"):
    """Full Gram matrix of ``model`` on X (× X2) on the device — single GPU, or sharded
    over the torch.distributed group (one process per GPU: each rank evaluates its tiles
    into a flat buffer, rank 0 gathers them; other ranks return None)."""
    kern = model_kern(model, device)
    N = len(X)
    N2 = None if X2 is None else len(X2)
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        rank, world = dist.get_rank(group), dist.get_world_size(group)
        cap = _capacity(N, N2, batch_size, world, split)
        local, _ = gram_local(kern, X, X2, batch_size, rank, world, device=device,
                              dtype=dtype, split=split, capacity=cap)
        return gather_gram(local, N, N2, batch_size, group, split=split)
    out, _ = gram_tiles(kern, X, X2, batch_size, device=device, dtype=dtype)
    return out
