"""The exp_mnist_resnet pipeline over one process per GPU, in device memory.

Reference: exp_mnist_resnet/run.bash:28-43 launches one save_kernel.py process per GPU
(each writes its share of the Kxx / Kxvx tiles to its own HDF5 file), merge_h5_files.py
NaN-merges the files, and classify_gp.py:61-77 loads Kxx, solves Kxx⁻¹Y and predicts
argmax(Kxz @ A).  Here:

1. every rank evaluates its row strip of Kxx (gram.strip_plan: balanced by evaluated
   pairs to 8 rows; gram.gram_strip), rank ``dst`` straight into the full matrix;
2. the strips are received into the full matrix on ``dst`` (gram.gather_strips: one
   point-to-point receive per rank, all posted together — RCCL over xGMI);
3. ``dst`` solves (rocSOLVER, classify_gp.py:17-27) WHILE the other ranks evaluate their
   row strips of Kxz; ``dst`` takes a smaller Kxz share sized so that its solve plus its
   strip ends with the others' strips (the solve time is estimated from n³/3 at
   ``solve_tflops``, the kernel rate from the Kxx phase);
4. α = Kxx⁻¹Y is broadcast, each rank multiplies its own Kxz rows by it, and only the
   [m, classes] scores travel back to ``dst`` (Kxz itself is gathered only
   when asked, e.g. for the HDF5 drop-in output or the posterior variance).

With world size 1 the same function runs the four steps in order on one device.  The
kernel, the solve and the score product are parameters, so the CPU tests drive this
exact code with the oracle on gloo ranks.
"""
from __future__ import annotations

import socket
import time
from typing import Callable, Optional

import numpy as np
import torch
import torch.distributed as dist

from .gram import (gather_strips, gram_strip, group_moves_device, row_slice, strip_cost,
                   strip_plan)
from .solve import check_alpha, diag_add, mirror_upper

__all__ = ("classify_distributed", "kxz_weights", "widening_matrix", "widen_in_place")


def widening_matrix(n: int, n2: int, dtype=torch.float32, out_dtype=torch.float64,
                    device=None):
    """An [n, n2] ``dtype`` matrix stored in the back half of an [n, n2] ``out_dtype``
    buffer (out_dtype twice as wide), so widen_in_place can turn it into the wide matrix
    without a second copy: classify_gp.py:45-48 widens the float32 K to float64 for the
    solve, and rank 0 then holds 1.0× the float64 matrix instead of 1.5×.
    Returns (buf, narrow view)."""
    a, b = torch.empty((), dtype=dtype).element_size(), \
        torch.empty((), dtype=out_dtype).element_size()
    if b != 2 * a:
        raise ValueError(f"{out_dtype} is not twice as wide as {dtype}")
    buf = torch.empty((n, n2), dtype=out_dtype, device=device)
    return buf, buf.view(-1).view(dtype)[n * n2:].view(n, n2)


def widen_in_place(buf: torch.Tensor, narrow: torch.Tensor,
                   cast: Optional[Callable] = None, tail_rows: int = 64) -> torch.Tensor:
    """Convert widening_matrix's narrow rows into buf, front to back.  Row block [i0, i1)
    is cast in one call when its wide destination ends before its narrow source starts
    (2·i1 ≤ n + i0; rows ≥ i1 are never touched) — half the rows, then a quarter, … — and
    the last ``tail_rows`` rows go through a small temporary.  ``cast(src, dst)`` converts
    one non-overlapping block (default dst.copy_(src); the device path passes
    solve.cast_into, the HIP cgp_cast_f32_f64).  Returns buf."""
    cast = cast or (lambda s, d: d.copy_(s))
    if tail_rows < 1:
        raise ValueError(f"tail_rows {tail_rows}: at least one row (the halving must end)")
    n = buf.shape[0]
    i0 = 0
    while i0 < n:
        i1 = (n + i0) // 2
        if i1 - i0 < tail_rows:
            cast(narrow[i0:].clone(), buf[i0:])
            break
        cast(narrow[i0:i1], buf[i0:i1])
        i0 = i1
    return buf


SOLVE_TFLOPS = 45.0     # the blocked Cholesky at n = 50-60 k in the full-scale runs (47-49)


def kxz_weights(world: int, n: int, m: int, kernel_pairs_per_s: float,
                solve_tflops: float = SOLVE_TFLOPS, dst: int = 0):
    """Kxz row shares: rank ``dst`` also solves, so its share s0 satisfies
    solve + s0·T = (1 − s0)/(world − 1)·T, T = m·n / rate (the whole Kxz on one GPU),
    clipped to [0, 1/world].  None (equal shares) at world size 1."""
    if world <= 1:
        return None
    T = m * n / max(kernel_pairs_per_s, 1.0)
    S = n ** 3 / 3.0 / (solve_tflops * 1e12)
    s0 = (T / (world - 1) - S) / (T + T / (world - 1))
    s0 = min(max(s0, 0.0), 1.0 / world)
    w = [(1.0 - s0) / (world - 1)] * world
    w[dst] = s0
    return w


def _bcast(t: torch.Tensor, src: int, group):
    if t.device.type == "cuda" and not group_moves_device(group):
        h = t.cpu()
        dist.broadcast(h, src, group=group)
        t.copy_(h)
    else:
        dist.broadcast(t, src, group=group)
    return t


def _ctl_device(dev, group):
    """where the group's small control tensors live: the host when a gloo backend serves
    host tensors ("gloo", or a mixed "cpu:gloo,cuda:nccl" group), the device under a pure
    RCCL group (RCCL moves device tensors only)"""
    return torch.device("cpu") if "gloo" in str(dist.get_backend(group)) else dev


def _max_over_ranks(v: float, dev, group) -> float:
    """max of a host scalar over the group"""
    t = torch.tensor([v], dtype=torch.float64, device=_ctl_device(dev, group))
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t)


def device_key(dev) -> str:
    """The physical device a rank computes on: host name plus the GPU's PCI location and
    UUID (the same for two processes that see one GPU under different visible-device
    lists), or the host name for a CPU device."""
    dev = torch.device(dev)
    host = socket.gethostname()
    if dev.type != "cuda":
        return f"{host}:cpu"
    p = torch.cuda.get_device_properties(dev)
    return f"{host}:{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}:{p.uuid}"


def co_resident_ranks(dev, group, dst: int) -> list:
    """The ranks of ``group`` other than ``dst`` whose device is dst's device (all_gather
    of device_key): none in the one-process-per-GPU layout; every rank in a rehearsal
    whose ranks share one GPU."""
    keys = [None] * dist.get_world_size(group)
    dist.all_gather_object(keys, device_key(dev), group=group)
    return [r for r, k in enumerate(keys) if r != dst and k == keys[dst]]


_SOLVE_OK, _SOLVE_FAILED, _SOLVE_WRONG_ALPHA = 0, 1, 2


def _sync(dev):
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)


def classify_distributed(kern: Callable, X, Z, Y: torch.Tensor, solve: Callable,
                         scores: Callable, batch_size: int = 4096, group=None, dst: int = 0,
                         device=None, dtype=torch.float64, out_dtype=torch.float64,
                         gather_kxz: bool = False, kxz_share=None,
                         solve_tflops: float = SOLVE_TFLOPS,
                         widen: Optional[Callable] = None, log: Optional[Callable] = None,
                         warm: Optional[Callable] = None, cast: Optional[Callable] = None,
                         rank_times: Optional[dict] = None,
                         pre_solve: Optional[Callable] = None, jitter: float = 0.0,
                         check: bool = True, check_tol: Optional[float] = None,
                         guard_shared_device: bool = True):
    """Kxx of X, α = solve(Kxx, Y), scores = Kxz @ α for Z against X, over the process
    group (or one process).

    kern(x, x2, same) -> [a, b] tile (gram.model_kern); solve(K, Y) -> α (may factor K in
    place, e.g. solve_system(..., overwrite_a=True)); scores(Kz, α) -> [rows, classes].
    ``dtype``: the kernel's output dtype (K is stored in it; float32 as the reference's
    save_kernel.py stores it); ``out_dtype``: the dtype solve and scores receive (float64:
    classify_gp.py:45-48 widens K) — ``widen(t)`` converts (default ``t.to(out_dtype)``;
    it may release its input).  When out_dtype is twice as wide as dtype (float32 → float64),
    dst's K lives in the back half of the wide matrix and is widened in place
    (widen_in_place with ``cast(src, dst)``, default a torch copy).  ``warm()`` (optional) runs on ``dst`` before the Kxx build
    and may return a thread to join before the solve (solve.warm_up_solver: the solver
    libraries load while the kernels run).  Returns on ``dst`` a dict with alpha, scores, pred, K (the
    matrix solve saw), Kxz (when gather_kxz), dst's own Kxz rows (``kxz_rows``,
    ``Kxz_rows``), timings, the plans and the device memory peaks (overall, and from the
    end of the Kxx build: the gather, the solve and the Kxz phase); None on the other
    ranks.  ``rank_times`` (optional dict) is filled on EVERY rank with that rank's own
    phase times and pairs (kxx_s, gather_kxx_s, kxz_s, predict_s, kxx_pairs, kxz_pairs).
    ``pre_solve(K)`` (optional) runs on ``dst`` with the assembled matrix just before the
    solve, outside ``solve_s`` (its time is ``pre_solve_s``): a caller's look at K before a
    solve that factors it in place (e.g. tools/fullscale.py's residual rows).

    ``jitter`` is added to the diagonal of the (widened) Kxx before the solve, as
    classify_gp.py:66-67 does (load_kern, then diag_add); ``solve`` must solve the system
    it is handed, exactly.  With ``check`` (default) the system is mirrored into Kxx's
    strictly-lower triangle first (solve.mirror_upper: the NaN tiles of the reference's
    layout) and α is verified against all of it (solve.check_alpha: backward error ≤
    ``check_tol``, default 16·√n·eps) — ``solve`` may factor the upper triangle in place
    but must leave the strictly-lower one alone (solve_system and scipy's posv do).  A
    failed check — or any exception in the widening, the pre_solve hook or the solve — is
    sent to every rank before α, and every rank raises (LinAlgError for a not
    positive-definite Kxx or a failed check, RuntimeError otherwise on the ranks that did
    not solve).  α never leaves ``dst`` unchecked.

    ``guard_shared_device``: ranks whose device is dst's device (co_resident_ranks: only in
    a rehearsal whose ranks share a GPU) wait until dst's solve has returned before they
    start their Kxz strips, and the Kxz rows are then split evenly.  Factorisations running
    beside other processes' work on one GPU have returned wrong factors with info = 0
    (round 5, profiles/r5/r5z_*); with one process per GPU nobody waits.

    Each rank binds only the images its strips read: a Kxx strip [r0, r1) touches rows
    and columns >= r0 (X[r0:]), a Kxz strip [z0, z1) the images Z[z0:z1] against all of
    X — the tiles and their order are those of the full sets (gram.strip_tiles anchors
    them at r0)."""
    conv = widen or (lambda t: t.to(out_dtype))
    dev = torch.device(device) if device is not None else (
        torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available()
        else torch.device("cpu"))
    multi = dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1
    world = dist.get_world_size(group) if multi else 1
    rank = dist.get_rank(group) if multi else 0
    n, m = len(X), len(Z)
    say = log if (log is not None and rank == dst) else (lambda *_: None)
    res = {"world": world}

    # 1. Kxx strips (dst evaluates its rows in place in the full matrix)
    plan_x = strip_plan(n, None, world)
    res["plan_kxx"] = plan_x
    if multi:
        dist.barrier(group)
    _sync(dev)
    t0 = time.perf_counter()
    warming = warm() if (warm is not None and rank == dst) else None
    r0, r1 = plan_x[rank]
    K = Kwide = None
    in_place = dtype != out_dtype and \
        2 * torch.empty((), dtype=dtype).element_size() == \
        torch.empty((), dtype=out_dtype).element_size()
    if rank == dst:
        if in_place:
            Kwide, K = widening_matrix(n, n, dtype, out_dtype, dev)
            K.fill_(float("nan"))
        else:
            K = torch.full((n, n), float("nan"), dtype=dtype, device=dev)
        rows_out = K[r0:r1]
    else:
        strip = torch.full((r1 - r0, n), float("nan"), dtype=dtype, device=dev)
        rows_out = strip
    # the strip's upper part [r0, r1) x [r0, n) from the images X[r0:] (strip_tiles in
    # local coordinates: the same tiles as over all of X, shifted by r0)
    _, _, px = gram_strip(kern, row_slice(X, r0, n), None, batch_size, (0, r1 - r0),
                          out=rows_out[:, r0:], dtype=dtype)
    _sync(dev)
    t_kxx = time.perf_counter() - t0
    if warming is not None:           # done long before on a full-size build; its 1.2 GB
        warming.join()                # identity must not count in the next phase's peak
        warming = None
        if dev.type == "cuda":        # nor stay reserved on the warm-up thread's stream
            torch.cuda.empty_cache()
    if dev.type == "cuda":
        res["peak_bytes_kxx_build"] = int(torch.cuda.max_memory_allocated(dev))
        torch.cuda.reset_peak_memory_stats(dev)      # next: the gather and the solve
    el = _max_over_ranks(t_kxx, dev, group) if multi else t_kxx
    res["kxx_s"] = round(el, 3)
    res["kxx_s_rank"] = round(t_kxx, 3)
    res["kxx_pairs_rank"] = px
    say(f"  Kxx strips built in {el:.1f} s")

    # 2. strips to dst
    t1 = time.perf_counter()
    if multi:
        K = gather_strips(K if rank == dst else strip, plan_x, n, full=K, group=group, dst=dst)
        strip = None
    _sync(dev)
    res["gather_kxx_s"] = round(time.perf_counter() - t1, 3)

    # 3. solve on dst, Kxz strips everywhere (dst's share sized to end with the others)
    share = co_resident_ranks(dev, group, dst) if (multi and guard_shared_device) else []
    res["co_resident_ranks"] = share
    rate = strip_cost(n, None, (0, n)) / world / max(el, 1e-9)
    if kxz_share is not None:
        w = kxz_share
    elif share:                     # dst's solve runs alone: no overlap to size for
        w = None
    else:
        w = kxz_weights(world, n, m, rate, solve_tflops, dst)
    plan_z = strip_plan(m, n, world, weights=w)
    res["plan_kxz"] = plan_z
    z0, z1 = plan_z[rank]
    alpha = None
    failure = None
    status = _SOLVE_OK
    if rank == dst:
        t2 = None
        Kd = None
        try:
            if pre_solve is not None:
                tp = time.perf_counter()
                pre_solve(K)
                _sync(dev)
                res["pre_solve_s"] = round(time.perf_counter() - tp, 4)
            t2 = time.perf_counter()
            if K.dtype == out_dtype:
                Kd = K
            elif Kwide is not None:
                Kd = widen_in_place(Kwide, K, cast)
            else:
                Kd = conv(K)
            del K, Kwide
            if jitter:
                diag_add(Kd, jitter)
            _sync(dev)
            res["widen_s"] = round(time.perf_counter() - t2, 3)
            dK = mirror_upper(Kd) if check else None        # before solve factors Kd
            Yd = Y.to(dev, out_dtype)
            alpha = solve(Kd, Yd)
            if check:
                try:
                    res["alpha_backward_error"] = check_alpha(Kd, dK, alpha, Yd, check_tol)
                except np.linalg.LinAlgError:
                    status = _SOLVE_WRONG_ALPHA
                    raise
        except Exception as e:      # e.g. LinAlgError (not PD): the other ranks must not
            failure = e             # wait for an α that never comes (see step 4)
            alpha = None
            if status == _SOLVE_OK:
                status = _SOLVE_FAILED
        _sync(dev)
        res["solve_s"] = round(time.perf_counter() - t2, 3) if t2 is not None else None
        if res["solve_s"] is not None:
            say(f"  solve {res['solve_s']:.2f} s")
        res["K"] = Kd
        if failure is not None and not multi:
            raise failure
    if share and (rank == dst or rank in share):
        # co-resident ranks start their Kxz strips only after dst's solve has returned
        flag = torch.tensor([status], dtype=torch.int64, device=_ctl_device(dev, group))
        gr = (lambda r: dist.get_global_rank(group, r)) if group is not None else (lambda r: r)
        if rank == dst:
            for r in share:
                dist.send(flag, gr(r), group=group)
        else:
            dist.recv(flag, gr(dst), group=group)
    if dev.type == "cuda":
        res["peak_bytes_gather_solve"] = int(torch.cuda.max_memory_allocated(dev))
        torch.cuda.reset_peak_memory_stats(dev)      # next: the Kxz strips
    t3 = time.perf_counter()
    Kz_full = None
    if gather_kxz and rank == dst:
        Kz_full = torch.full((m, n), float("nan"), dtype=dtype, device=dev)
        Kz, _, pz = gram_strip(kern, row_slice(Z, z0, z1), X, batch_size, (0, z1 - z0),
                               out=Kz_full[z0:z1], dtype=dtype)
    else:
        Kz, _, pz = gram_strip(kern, row_slice(Z, z0, z1), X, batch_size, (0, z1 - z0),
                               device=dev, dtype=dtype)
    _sync(dev)
    res["kxz_s_rank"] = round(time.perf_counter() - t3, 3)
    res["kxz_pairs_rank"] = pz
    done = time.perf_counter() - t0

    # 4. α to every rank, local scores, scores to dst.  The solve's outcome travels first, so
    # a failed solve (or an α that fails its check) raises on every rank instead of leaving
    # them in the broadcast
    ncls = Y.shape[1] if Y.dim() > 1 else 1
    if multi:
        ok = torch.tensor([status], dtype=torch.int64, device=_ctl_device(dev, group))
        dist.broadcast(ok, dst, group=group)
        code = int(ok)
        if code != _SOLVE_OK and failure is None:
            if code == _SOLVE_WRONG_ALPHA:
                raise np.linalg.LinAlgError(
                    f"classify_distributed: the solution on rank {dst} failed its residual "
                    f"check (a wrong factorisation); no α was broadcast")
            raise RuntimeError(f"classify_distributed: the solve failed on rank {dst}")
    if failure is not None:
        raise failure
    if multi:
        if rank != dst:
            alpha = torch.empty((n, ncls), dtype=out_dtype, device=dev)
        alpha = _bcast(alpha.reshape(n, ncls).contiguous(), dst, group)
    alpha = alpha.reshape(n, ncls)
    t4 = time.perf_counter()
    sc = scores(Kz if Kz.dtype == out_dtype else conv(Kz), alpha) if z1 > z0 else \
        torch.empty((0, ncls), dtype=out_dtype, device=dev)
    full_sc = None
    if rank == dst:
        full_sc = torch.empty((m, ncls), dtype=out_dtype, device=dev)
        full_sc[z0:z1].copy_(sc)
    if multi:
        full_sc = gather_strips(sc if rank != dst else None, plan_z, ncls, full=full_sc,
                                group=group, dst=dst)
        if gather_kxz:
            Kz_full = gather_strips(Kz if rank != dst else None, plan_z, n, full=Kz_full,
                                    group=group, dst=dst)
    elif gather_kxz:
        Kz_full = Kz
    _sync(dev)
    res["predict_s"] = round(time.perf_counter() - t4, 3)
    if multi:
        done = _max_over_ranks(done, dev, group)
    res["kxx_to_kxz_s"] = round(done, 3)
    res["total_s"] = round(time.perf_counter() - t0, 3)
    if rank_times is not None:
        rank_times.update(rank=rank, kxx_s=res["kxx_s_rank"], kxx_pairs=px,
                          gather_kxx_s=res["gather_kxx_s"], kxz_s=res["kxz_s_rank"],
                          kxz_pairs=pz, kxz_rows=[z0, z1], kxx_rows=[r0, r1],
                          predict_s=res["predict_s"])
    if rank != dst:
        return None
    res.update(alpha=alpha, scores=full_sc, pred=full_sc.argmax(1), Kxz=Kz_full,
               kxz_share=w, kxz_rows=(z0, z1), Kxz_rows=Kz)
    if dev.type == "cuda":
        res["peak_bytes_kxz"] = int(torch.cuda.max_memory_allocated(dev))
    return res
