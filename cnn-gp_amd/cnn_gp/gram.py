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

__all__ = ("gram_tiles", "gram_local", "gather_gram", "gram_matrix", "model_kern", "ModelKern",
           "tile_plan", "tile_cost")

Tile = Tuple[bool, int, int, int, int]       # (same, i0, j0, rows, cols)


def _rows(X, lo, hi):
    """Images lo:hi of X — a tensor, a TensorDataset-like (first tensor) or a Dataset."""
    if isinstance(X, torch.Tensor):
        return X[lo:hi]
    if hasattr(X, "tensors"):
        return X.tensors[0][lo:hi]
    return torch.stack([X[k][0] for k in range(lo, hi)])


def row_slice(X, lo, hi):
    """Images lo:hi of X as an image set of the same kind (tensor, TensorDataset-like or
    Dataset), for building a strip from only the rows it reads."""
    if isinstance(X, torch.Tensor):
        return X[lo:hi]
    if hasattr(X, "tensors"):
        from torch.utils.data import TensorDataset
        return TensorDataset(*(t[lo:hi] for t in X.tensors))
    from torch.utils.data import Subset
    return Subset(X, range(lo, hi))


def _default_device(device):
    if device is not None:
        return torch.device(device)
    if not torch.cuda.is_available():
        raise RuntimeError("cnn_gp.gram needs a HIP device (there is no CPU path)")
    return torch.device("cuda", torch.cuda.current_device())


class ModelKern:
    """kern(x, x2, same) -> device tensor: the model evaluated on the device, one forward
    per tile (the reference's call, save_kernel.py → kernel_save_tools.py:36-45).

    ``bind(X, X2)`` is the whole-build form the builders below take when they are given a
    ModelKern: every image's variance maps are computed once for the build
    (NNGPKernel.image_variances) instead of once per tile and side, and each tile is
    written straight into its place in the output (NNGPKernel.tile_from_variances).  The
    maps live as long as the bound object, i.e. one build."""

    def __init__(self, model, device=None, dtype=None):
        self.model, self.device, self.dtype = model, device, dtype

    def __call__(self, x, x2, same):
        dev = _default_device(self.device)
        xd = x.to(dev, self.dtype or x.dtype)
        with torch.no_grad():
            if same:
                return self.model(xd)
            return self.model(xd, x2.to(dev, self.dtype or x2.dtype), False, False)

    def bind(self, X, X2=None) -> Optional["BoundKern"]:
        """The build's variance maps of X (and X2), or None when the model has no
        whole-network program for them (the builders then call the kern per tile)."""
        if not hasattr(self.model, "image_variances"):
            return None
        dev = _default_device(self.device)

        def images(S):
            if isinstance(S, torch.Tensor):
                t = S
            elif hasattr(S, "tensors"):
                t = S.tensors[0]
            else:
                return None
            return t.to(dev, self.dtype or t.dtype).contiguous()
        xd = images(X)
        if xd is None:
            return None
        with torch.no_grad():
            vx = self.model.image_variances(xd)
            if vx is None:
                return None
            if X2 is None:
                return BoundKern(self.model, vx, vx)
            yd = images(X2)
            vy = None if yd is None else self.model.image_variances(yd.to(xd.dtype))
        return None if vy is None else BoundKern(self.model, vx, vy)


class BoundKern:
    """ModelKern.bind's result: tiles of one build from its precomputed variance maps."""

    def __init__(self, model, vx, vy):
        self.model, self.vx, self.vy = model, vx, vy

    def tile(self, t: Tile, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Tile t = (same, i0, j0, rows, cols); written into ``out`` when it is a
        row-major view of the images' dtype, else returned (and copied by the caller)."""
        same, i0, j0, a, b = t
        direct = out is not None and out.dtype == self.vx.images.dtype and \
            out.device == self.vx.images.device and out.dim() == 2 and \
            out.stride(1) == 1 and tuple(out.shape) == (a, b)
        with torch.no_grad():
            k = self.model.tile_from_variances(self.vx, i0, i0 + a, self.vx if same else self.vy,
                                               j0, j0 + b, same, out=out if direct else None)
        if out is not None and not direct:
            out.copy_(k)
        return k


def model_kern(model, device=None, dtype=None) -> ModelKern:
    """kern(x, x2, same) -> device tensor: the model evaluated on the device (a ModelKern:
    the builders below evaluate its tiles from one build's variance maps)."""
    return ModelKern(model, device, dtype)


def _fill_tiles(kern, X, src2, X2, tiles, view):
    """Evaluate ``tiles`` into view(t) (a [rows, cols] slice of the output each): from one
    bound build when kern is a ModelKern with a whole-network program, else one kern call
    per tile copied into place."""
    if not tiles:                 # an empty strip: nothing to bind
        return
    bound = kern.bind(X, X2) if isinstance(kern, ModelKern) else None
    for t in tiles:
        if bound is not None:
            bound.tile(t, view(t))
        else:
            view(t).copy_(_eval_tile(kern, X, src2, t))


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
    _fill_tiles(kern, X, src2, X2, done, lambda t: out[t[1]:t[1] + t[3], t[2]:t[2] + t[4]])
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
    offs, off = {}, 0
    for t in tiles:
        offs[t] = off
        off += t[3] * t[4]
    _fill_tiles(kern, X, src2, X2, tiles,
                lambda t: buf[offs[t]:offs[t] + t[3] * t[4]].view(t[3], t[4]))
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
    staged = _p2p_staged(group, local.device)
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


# ------------------------------------------------------------------------------------------
# Row strips: the full-scale layout (one contiguous block of rows per rank)
# ------------------------------------------------------------------------------------------
# A rank owns rows [r0, r1) of the matrix and evaluates every tile of them: for Kxx the
# upper triangle of those rows (j >= i: its square [r0, r1)² as diagonal + upper tiles, then
# the rectangle [r0, r1) × [r1, N)); for Kxz all of [r0, r1) × [0, N2) — the north star's
# "row-blocks of X against all Z".  Rows i0:i1 of a row-major [N, N2] matrix are one
# contiguous range, so rank 0 receives each rank's strip straight into its place in the
# full matrix (one point-to-point receive per rank, all in flight together over xGMI): no
# staging buffer, no unpack, and rank 0 evaluates its own strip in place — its peak is the
# matrix itself (1.0× Kxx, against 2.1× for gather_gram's padded receive list).
#
# Strip boundaries come from the evaluated pairs: row i of Kxx costs N − 1 − i pairs (the
# kernel evaluates i < j; K[i, i] is the variance chain's), a Kxz row costs N2, so the split
# balances to one alignment unit of rows (8 = the kernel's supertile edge), not to one tile.
# ``weights`` gives ranks unequal shares (e.g. a smaller Kxz share for the rank that
# solves while the others build Kxz).

def _row_cost_prefix(N: int, N2: Optional[int], r: int) -> int:
    """evaluated pairs in rows [0, r)"""
    if N2 is None:
        return r * (N - 1) - r * (r - 1) // 2
    return r * N2


def strip_plan(N: int, N2: Optional[int], world: int, weights=None,
               align: int = 8) -> List[Tuple[int, int]]:
    """[(r0, r1)] per rank: contiguous row ranges covering [0, N) whose evaluated pairs
    follow ``weights`` (default equal), boundaries on multiples of ``align``."""
    if world < 1:
        raise ValueError("world must be >= 1")
    w = [1.0] * world if weights is None else [float(v) for v in weights]
    if len(w) != world or min(w) < 0 or sum(w) <= 0:
        raise ValueError(f"weights {weights!r} for world {world}")
    total = _row_cost_prefix(N, N2, N)
    cuts, acc = [0], 0.0
    for k in range(world - 1):
        acc += w[k]
        target = total * acc / sum(w)
        lo, hi = cuts[-1], N                   # smallest r with prefix(r) >= target
        while lo < hi:
            mid = (lo + hi) // 2
            if _row_cost_prefix(N, N2, mid) >= target:
                hi = mid
            else:
                lo = mid + 1
        r = lo
        if align > 1 and 0 < r < N:            # nearest aligned row
            down = r // align * align
            up = min(N, down + align)
            r = down if target - _row_cost_prefix(N, N2, down) <= \
                _row_cost_prefix(N, N2, up) - target else up
        cuts.append(max(cuts[-1], min(N, r)))
    cuts.append(N)
    return [(cuts[k], cuts[k + 1]) for k in range(world)]


def strip_cost(N: int, N2: Optional[int], rows: Tuple[int, int]) -> int:
    """pairs the kernel evaluates for the strip ``rows``"""
    return _row_cost_prefix(N, N2, rows[1]) - _row_cost_prefix(N, N2, rows[0])


def strip_tiles(N: int, N2: Optional[int], rows: Tuple[int, int],
                batch_size: int) -> List[Tile]:
    """The tiles (same, i0, j0, a, b) of a strip, global coordinates.  Kxx: the square
    [r0, r1)² in the reference's upper-tile order (data.py:22-29) with B-tiles anchored at
    r0, then the rectangle [r0, r1) × [r1, N) in row blocks of B × B.  Kxz: [r0, r1) × [0, N2)
    in B × B tiles.  For one strip covering [0, N) this is exactly tile_plan's list."""
    r0, r1 = rows
    B = batch_size
    out: List[Tile] = []
    if r1 <= r0:
        return out
    if N2 is not None:
        for i0 in range(r0, r1, B):
            for j0 in range(0, N2, B):
                out.append((False, i0, j0, min(B, r1 - i0), min(B, N2 - j0)))
        return out
    for i0 in range(r0, r1, B):
        a = min(B, r1 - i0)
        out.append((True, i0, i0, a, a))
        for j0 in range(i0 + B, r1, B):
            out.append((False, i0, j0, a, min(B, r1 - j0)))
        for j0 in range(r1, N, B):
            out.append((False, i0, j0, a, min(B, N - j0)))
    return out


def gram_strip(kern: Callable, X, X2=None, batch_size: int = 4096,
               rows: Tuple[int, int] = (0, 0), out: Optional[torch.Tensor] = None,
               device=None, dtype=torch.float64):
    """Evaluate the strip ``rows`` of Kxx (X2 None) or Kxz into ``out`` ([r1 − r0, N2] —
    e.g. a row range of the full matrix; a new NaN-filled device block when None).  Entries
    the strip does not evaluate (Kxx's strictly-lower part) stay as ``out`` had them.
    Returns (out, tiles, pairs evaluated)."""
    N = len(X)
    N2 = None if X2 is None else len(X2)
    n2 = N if N2 is None else N2
    src2 = X if X2 is None else X2
    r0, r1 = rows
    if out is None:
        out = torch.full((r1 - r0, n2), float("nan"), dtype=dtype,
                         device=_default_device(device))
    if tuple(out.shape) != (r1 - r0, n2):
        raise ValueError(f"out {tuple(out.shape)} for strip rows {rows} of width {n2}")
    tiles = strip_tiles(N, N2, rows, batch_size)
    _fill_tiles(kern, X, src2, X2, tiles,
                lambda t: out[t[1] - r0:t[1] - r0 + t[3], t[2]:t[2] + t[4]])
    return out, tiles, sum(tile_cost(t) for t in tiles)


def group_moves_device(group) -> bool:
    """True when the group has RCCL for device tensors: backend "nccl", or a mixed group
    such as "cpu:gloo,cuda:nccl" (dist.get_backend returns the whole string then)."""
    return "nccl" in str(dist.get_backend(group))


def _p2p_staged(group, tensor_device) -> bool:
    """gloo moves CPU tensors only: without RCCL in the group, device buffers travel
    through host memory"""
    return tensor_device.type == "cuda" and not group_moves_device(group)


def gather_strips(strip: Optional[torch.Tensor], plan: List[Tuple[int, int]], n2: int,
                  full: Optional[torch.Tensor] = None, group=None, dst: int = 0):
    """Assemble every rank's strip on rank ``dst``: rank r sends its [r1 − r0, n2] block,
    ``dst`` receives it straight into ``full[r0:r1]`` (a contiguous range of the row-major
    matrix).  ``full`` on ``dst``: the [N, n2] matrix whose own rows already hold dst's
    strip (gram_strip(out=full[r0:r1])).  All receives are posted together
    (batch_isend_irecv: one link per peer over xGMI with RCCL); under gloo, device data is
    staged through host memory one strip at a time.  Returns ``full`` on dst, None
    elsewhere."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    if len(plan) != world:
        raise ValueError(f"plan has {len(plan)} strips for world {world}")
    if rank == dst:
        if full is None or full.dim() != 2 or full.shape[1] != n2 or \
                full.shape[0] != plan[-1][1] or not full.is_contiguous():
            raise ValueError("dst needs the contiguous [N, n2] matrix holding its own strip")
        peers = [(r, plan[r]) for r in range(world) if r != dst and plan[r][1] > plan[r][0]]
        if _p2p_staged(group, full.device):
            for r, (a, b) in peers:
                buf = torch.empty((b - a, n2), dtype=full.dtype)
                dist.recv(buf, dist.get_global_rank(group, r) if group else r, group=group)
                full[a:b].copy_(buf)
        elif peers:
            ops = [dist.P2POp(dist.irecv, full[a:b], dist.get_global_rank(group, r)
                              if group else r, group) for r, (a, b) in peers]
            for req in dist.batch_isend_irecv(ops):
                req.wait()
        return full
    a, b = plan[rank]
    if b > a:
        if strip is None or tuple(strip.shape) != (b - a, n2):
            raise ValueError(f"rank {rank}: strip must be [{b - a}, {n2}]")
        peer = dist.get_global_rank(group, dst) if group else dst
        if _p2p_staged(group, strip.device):
            dist.send(strip.contiguous().cpu(), peer, group=group)
        else:
            for req in dist.batch_isend_irecv([dist.P2POp(dist.isend, strip.contiguous(),
                                                          peer, group)]):
                req.wait()
    return None
