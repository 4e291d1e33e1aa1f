"""HDF5 tile persistence with the reference's exact layout (kernel_save_tools.py:7-58).

Datasets are float32, shape (1, N, N2) (diag: (1, N)), NaN-filled, chunked
(1, min(B, N), min(B, N2)), maxshape (None, N, N2): a worker writes only its tiles, the
rest stay NaN (Kxx's strictly-lower off-diagonal tiles stay NaN forever), and files of
several workers merge by filling NaNs (exp_mnist_resnet/merge_h5_files.py).  ``f`` is
anything with ``keys()``, ``create_dataset(...)`` and slice assignment (an h5py.File,
or the in-memory stand-in used by the tests).
"""
from __future__ import annotations

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
           print_interval=2.):
    """Evaluate this worker's tiles with ``kern(x, x2, same, diag) -> np.ndarray`` and
    write them into dataset ``name`` (created if absent; skipped if it exists)."""
    if name in f.keys():
        print("Skipping {} (group exists)".format(name))
        return
    N = len(X)
    N2 = N if X2 is None else len(X2)
    out = create_h5py_dataset(f, batch_size, name, diag, N, N2)
    if diag:
        it = DiagIterator(batch_size, X, X2)       # diagonals are cheap: not split
    else:
        it = ProductIterator(batch_size, X, X2, worker_rank=worker_rank, n_workers=n_workers)
    it = print_timings(it, desc=f"{name} (worker {worker_rank}/{n_workers})",
                       print_interval=print_interval)
    for same, (i, (x, _y)), (j, (x2, _y2)) in it:
        k = kern(x, x2, same, diag)
        if not np.all(np.isfinite(k)):
            raise FloatingPointError(f"About to write a nan or inf for {i},{j} in {name}")
        if diag:
            out[0, i:i + len(x)] = k
        else:
            out[0, i:i + len(x), j:j + len(x2)] = k


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
