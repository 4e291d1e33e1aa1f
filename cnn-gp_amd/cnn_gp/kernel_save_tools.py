"""HDF5 tile persistence with the reference's exact layout (kernel_save_tools.py:7-58).

Datasets are float32, shape (1, N, N2) (diag: (1, N)), NaN-filled, chunked
(1, min(B, N), min(B, N2)), maxshape (None, N, N2): a worker writes only its tiles, the
rest stay NaN (Kxx's strictly-lower off-diagonal tiles stay NaN forever), and files of
several workers merge by filling NaNs (exp_mnist_resnet/merge_h5_files.py).  ``f`` is
anything with ``keys()``, ``create_dataset(...)`` and slice assignment (an h5py.File,
or the in-memory stand-in used by the tests).
"""
from __future__ import annotations

import collections
import threading
from concurrent.futures import ThreadPoolExecutor

import numpy as np

from .data import DiagIterator, ProductIterator, print_timings

__all__ = ("create_h5py_dataset", "save_K", "merge_nan_fill")


def create_h5py_dataset(f, batch_size, name, diag, N, N2):
    if diag:
        chunks, shape, maxshape = (1, min(batch_size, N)), (1, N), (None, N)
    else:
        chunks = (1, min(batch_size, N), min(batch_size, N2))
        shape, maxshape = (1, N, N2), (None, N, N2)
    return f.create_dataset(name, shape=shape, dtype=np.float32, fillvalue=np.nan,
                            chunks=chunks, maxshape=maxshape)


def save_K(f, kern, name, X, X2, diag, batch_size, worker_rank=0, n_workers=1,
           print_interval=2., overlap=4, pin=True):
    """Evaluate this worker's tiles with ``kern(x, x2, same, diag) -> np.ndarray`` and
    write them into dataset ``name`` (created if absent; skipped if it exists).

    ``overlap`` (default 4): up to that many tiles are in flight at once, each kern call
    on a helper thread with a HIP stream of its own (torch's current stream is per
    thread), so one tile's host work — the caller's pageable H2D copies, forward's launch
    calls, the synchronous copy back, the finiteness check and the dataset write — runs
    while the GPU evaluates another, and small tiles' kernels fill each other's tails
    (save_kernel.py:21-24's kern synchronises per tile, which left the GPU idle for 30-43%
    of a B = 200 build, bench.py ``dropin``).  The helper threads persist across save_K
    calls.  Measured at B = 200 on one MI355X
    (tools/dropin_overlap_probe.py, profiles/r6/r6c_overlap_*.log): ConvNet GP 0.46 ms per
    tile serial, 0.32 at overlap 3; mnist_as_tf 0.89 → 0.58-0.66.  Tiles
    are still checked and written in the reference's order, every tile's values are the
    same bits (a tile depends on its own images only), and an exception of a kern call
    or of the finiteness check surfaces in that order.  ``overlap=1`` calls kern on the
    calling thread, one tile at a time, as kernel_save_tools.py:49-58 does.

    ``pin`` (default True, with a GPU visible): a TensorDataset's host tensors (also under
    a Subset / ConcatDataset) are copied once into page-locked memory for this call, so
    the batches kern receives are views of pinned memory and the caller's ``x.cuda()`` is
    one DMA instead of a staged pageable copy (bench.py ``dropin``, ConvNet GP, N = 4096,
    B = 200: 0.323 → 0.282 ms per tile, 0.89 → 1.02 of the bound build;
    profiles/r6/r6u_dropin_pin{0,1}_full.json).  Same values, same dtype; the caller's
    dataset is not modified."""
    if name in f.keys():
        print("Skipping {} (group exists)".format(name))
        return
    if pin:
        X, X2 = _pinned(X), (None if X2 is None else _pinned(X2))
    N = len(X)
    N2 = N if X2 is None else len(X2)
    out = create_h5py_dataset(f, batch_size, name, diag, N, N2)
    if diag:
        it = DiagIterator(batch_size, X, X2)       # diagonals are cheap: not split
    else:
        it = ProductIterator(batch_size, X, X2, worker_rank=worker_rank, n_workers=n_workers)
    it = print_timings(it, desc=f"{name} (worker {worker_rank}/{n_workers})",
                       print_interval=print_interval)

    def write(i, j, x, x2, k):
        if not np.all(np.isfinite(k)):
            raise FloatingPointError(f"About to write a nan or inf for {i},{j} in {name}")
        if diag:
            out[0, i:i + len(x)] = k
        else:
            out[0, i:i + len(x), j:j + len(x2)] = k

    if overlap <= 1:
        for same, (i, (x, _y)), (j, (x2, _y2)) in it:
            write(i, j, x, x2, kern(x, x2, same, diag))
        return
    call = _on_own_stream(kern)
    pending = collections.deque()
    pool = _pool(int(overlap))
    try:
        for same, (i, (x, _y)), (j, (x2, _y2)) in it:
            pending.append((i, j, x, x2, pool.submit(call, x, x2, same, diag)))
            if len(pending) >= overlap:
                i_, j_, a_, b_, fut = pending.popleft()
                write(i_, j_, a_, b_, fut.result())
        while pending:
            i_, j_, a_, b_, fut = pending.popleft()
            write(i_, j_, a_, b_, fut.result())
    finally:
        for *_, fut in pending:            # an error above: nothing more is written
            fut.cancel()
        for *_, fut in pending:            # and no call is left running behind the caller
            if not fut.cancelled():
                try:
                    fut.result()
                except Exception:          # noqa: BLE001 - the first error is the one raised
                    pass


# Helper threads live as long as the process (one pool per overlap): a thread keeps its
# HIP stream, and with it the model's tile recipes (netplan.TileRecipe, one per tile shape
# and stream), from one save_K to the next — save_kernel.py calls save_K five times.
_POOLS = {}
_POOLS_LOCK = threading.Lock()
_TLS = threading.local()                      # each helper thread's stream per device


def _pool(n: int) -> ThreadPoolExecutor:
    with _POOLS_LOCK:
        p = _POOLS.get(n)
        if p is None:
            p = _POOLS[n] = ThreadPoolExecutor(max_workers=n, thread_name_prefix="cgp-save-K")
        return p


def _on_own_stream(kern):
    """kern wrapped to run under a HIP stream of the calling thread's own (created on the
    thread's first call, on the caller's device) when a GPU is visible; plain kern
    otherwise.  (Handing kern its batches in freshly pinned memory measured slower: the
    pinned allocations stall the device.)"""
    import torch
    if not torch.cuda.is_available():
        return kern
    dev = torch.cuda.current_device()          # the caller's device, not device 0

    def call(x, x2, same, diag):
        streams = getattr(_TLS, "streams", None)
        if streams is None:
            streams = _TLS.streams = {}
        s = streams.get(dev)
        if s is None:
            torch.cuda.set_device(dev)
            s = streams[dev] = torch.cuda.Stream(dev)
        with torch.cuda.stream(s):
            k = kern(x, x2, same, diag)
        return k

    return call


def _pinned(ds):
    """ds with its host tensors in page-locked memory (a new dataset object of the same
    exact class), or ds itself: no GPU, other dataset kinds, tensors already on a device
    or pinned.  Only the classes data.tensor_rows slices (the exact ones: a subclass may
    override __getitem__)."""
    import torch
    from torch.utils.data import ConcatDataset, Subset, TensorDataset
    if not torch.cuda.is_available():
        return ds
    kind = type(ds)
    if kind is TensorDataset:
        ts = ds.tensors
        if not all(t.device.type == "cpu" for t in ts) or all(t.is_pinned() for t in ts):
            return ds
        try:
            return TensorDataset(*(t if t.is_pinned() else t.pin_memory() for t in ts))
        except RuntimeError:          # no page-locked memory to spare: the pageable rows
            return ds
    if kind is Subset:
        inner = _pinned(ds.dataset)
        return ds if inner is ds.dataset else Subset(inner, ds.indices)
    if kind is ConcatDataset:
        parts = [_pinned(d) for d in ds.datasets]
        if all(a is b for a, b in zip(parts, ds.datasets)):
            return ds
        return ConcatDataset(parts)
    return ds


def merge_nan_fill(dest, sources):
    """exp_mnist_resnet/merge_h5_files.py:24-30 on array-likes: fill dest's NaNs from
    each source in turn (dest[i] is read, patched and written back per leading index)."""
    for src in sources:
        for i in range(len(dest)):
            d = np.array(dest[i, ...])
            s = np.asarray(src[i, ...])
            hole = np.isnan(d)
            d[hole] = s[hole]
            dest[i, ...] = d
    return dest
