"""Tile schedule, worker split and dataset plumbing (reference: cnn_gp/data.py).

The Gram matrix is evaluated in B×B tiles.  ``ProductIterator`` yields the reference's
tile order — for Kxx the upper triangle row by row, diagonal tile first (data.py:22-29),
for Kxz every tile — and gives worker ``r`` of ``n`` a contiguous, balanced slice of it
(data.py:11-19, 54-60).  Multi-GPU Gram assembly (gram.py) uses the same split, so a
rank's tiles are exactly the reference worker's.

Differences from the reference, all bug fixes that keep the documented behaviour:
``np.int`` (removed in numpy 1.24, data.py:12) is not used; ``DiagIterator`` with a
second dataset unpacks ``enumerate(zip(...))`` correctly (data.py:124 raises).
``DatasetFromConfig`` reads MNIST from local IDX files (no network download).
"""
from __future__ import annotations

import gzip
import itertools
import os
import time

import numpy as np
import torch
from torch.utils.data import ConcatDataset, DataLoader, Subset, TensorDataset

__all__ = ("DatasetFromConfig", "ProductIterator", "DiagIterator", "print_timings",
           "tile_schedule", "worker_slice", "tensor_rows")


def worker_slice(n_batches: int, worker_rank: int, n_workers: int):
    """(start, count) of this worker's contiguous share (data.py:11-19): every worker
    gets n_batches // n_workers, the first n_batches % n_workers one more."""
    if not 0 <= worker_rank < n_workers:
        raise ValueError(f"worker_rank {worker_rank} not in [0, {n_workers})")
    base, extra = divmod(n_batches, n_workers)
    start = worker_rank * base + min(worker_rank, extra)
    return start, base + (1 if worker_rank < extra else 0)


def _tile_order(bx: int, bx2: int, same: bool):
    for i in range(bx):
        if same:
            yield True, i, i
        for j in range(i + 1 if same else 0, bx2):
            yield False, i, j


def _ceil_div(a, b):
    return -(-a // b)


def tile_schedule(n_x: int, n_x2, batch_size: int, worker_rank: int = 0, n_workers: int = 1):
    """This worker's tiles as (same, i_block, j_block) in the reference's order."""
    bx = _ceil_div(n_x, batch_size)
    if n_x2 is None:
        same, bx2 = True, bx
        n_batches = max(1, bx * (bx + 1) // 2)
    else:
        same, bx2 = False, _ceil_div(n_x2, batch_size)
        n_batches = bx * bx2
    start, count = worker_slice(n_batches, worker_rank, n_workers)
    return list(itertools.islice(_tile_order(bx, bx2, same), start, start + count))


def tensor_rows(dataset, lo: int, hi: int):
    """Items lo:hi of ``dataset`` as the DataLoader collates them ([images, labels], each
    stacked along a new first dimension), sliced straight out of the backing tensors when
    the dataset is a TensorDataset or a Subset / ConcatDataset of them (what
    DatasetFromConfig builds and what save_K is handed); None for any other dataset
    (the caller then collates item by item).  Collating a 200-image batch item by item
    costs ~1-3 ms of host time per tile, several times the kernel's own time at the
    reference's batch_size 200 (bench.py ``dropin``).  The exact classes only: a subclass
    may override ``__getitem__`` (e.g. a transform), which slicing would bypass."""
    kind = type(dataset)
    if kind is TensorDataset:
        return [t[lo:hi] for t in dataset.tensors]
    if kind is Subset:
        idx = dataset.indices[lo:hi]
        if isinstance(idx, range) and idx.step == 1:
            return tensor_rows(dataset.dataset, idx.start, idx.stop)
        if type(dataset.dataset) is TensorDataset:
            ix = torch.as_tensor(list(idx), dtype=torch.int64)
            return [t[ix] for t in dataset.dataset.tensors]
        return None
    if kind is ConcatDataset:
        parts, start = [], 0
        for d, end in zip(dataset.datasets, dataset.cumulative_sizes):
            a, b = max(lo, start), min(hi, end)
            if a < b:
                p = tensor_rows(d, a - start, b - start)
                if p is None:
                    return None
                parts.append(p)
            start = end
        if not parts:
            return None
        return parts[0] if len(parts) == 1 else [torch.cat(c) for c in zip(*parts)]
    return None


class ProductIterator:
    """Iterates this worker's Gram tiles, yielding
    ``(same, (i0, x_batch), (j0, x2_batch))`` with the batches as the DataLoader
    collates them (data.py:36-96)."""

    def __init__(self, batch_size, X, X2=None, worker_rank=0, n_workers=1):
        self.same = X2 is None
        self.X = X
        self.X2 = X if X2 is None else X2
        self.batch_size = batch_size
        self.worker_rank = worker_rank
        self.tiles = tile_schedule(len(X), None if X2 is None else len(X2), batch_size,
                                   worker_rank, n_workers)
        self._it = iter(self.tiles)
        self._cache_i = (None, None)

    def __len__(self):
        return len(self.tiles)

    def __iter__(self):
        return self

    def _batch(self, dataset, b):
        lo = b * self.batch_size
        hi = min(lo + self.batch_size, len(dataset))
        fast = tensor_rows(dataset, lo, hi)
        if fast is not None:
            return fast
        sub = Subset(dataset, range(lo, hi))
        return next(iter(DataLoader(sub, batch_size=self.batch_size)))

    def __next__(self):
        same, i, j = next(self._it)
        if self._cache_i[0] != i:
            self._cache_i = (i, self._batch(self.X, i))
        xb = self._cache_i[1]
        x2b = xb if (self.same and i == j) else self._batch(self.X2, j)
        return same, (i * self.batch_size, xb), (j * self.batch_size, x2b)


class DiagIterator:
    """Batches for the kernel diagonal (data.py:99-126); never split across workers."""

    def __init__(self, batch_size, X, X2=None):
        self.batch_size = batch_size
        dl = self._batches(X, batch_size)
        if X2 is None:
            self.same = True
            self.it = iter(enumerate(dl))
            self.length = len(dl)
        else:
            dl2 = self._batches(X2, batch_size)
            self.same = False
            self.it = iter(enumerate(zip(dl, dl2)))
            self.length = min(len(dl), len(dl2))

    @staticmethod
    def _batches(X, batch_size):
        """The DataLoader's batches of X — sliced from the backing tensors when X is a
        TensorDataset / Subset / ConcatDataset of them (tensor_rows), else the DataLoader"""
        n = len(X)
        out = [tensor_rows(X, lo, min(lo + batch_size, n)) for lo in range(0, n, batch_size)]
        if any(b is None for b in out):      # e.g. a ConcatDataset with one other part
            return DataLoader(X, batch_size=batch_size)
        return out

    def __iter__(self):
        return self

    def __len__(self):
        return self.length

    def __next__(self):
        if self.same:
            i, xy = next(self.it)
            xy2 = xy
        else:
            i, (xy, xy2) = next(self.it)
        ib = i * self.batch_size
        return self.same, (ib, xy), (ib, xy2)


def _hhmmss(s):
    m, s = divmod(int(s), 60)
    h, m = divmod(m, 60)
    return f"{m:02d}:{s:02d}" if h == 0 else f"{h:02d}:{m:02d}:{s:02d}"


def print_timings(iterator, desc="time", print_interval=2.):
    """Progress lines (it/s, elapsed<eta) at most every print_interval s (data.py:174-196)."""
    start = time.perf_counter()
    total = len(iterator)
    last = -print_interval
    for i, value in enumerate(iterator):
        yield value
        elapsed = time.perf_counter() - start
        rate = (i + 1) / elapsed if elapsed > 0 else float("inf")
        if elapsed > last + print_interval:
            eta = total / rate if rate > 0 else 0.0
            print(f"{desc}: {i + 1}/{total} it, {rate:.02f} it/s,"
                  f"[{_hhmmss(elapsed)}<{_hhmmss(eta)}]")
            last = elapsed


# ------------------------------------------------------------------------------------
# datasets (data.py:129-162) — local files only
# ------------------------------------------------------------------------------------
class _Transformed(torch.utils.data.Dataset):
    """Applies a list of callables to each item's image (torchvision Compose order)."""

    def __init__(self, base, transforms):
        self.base, self.transforms = base, transforms

    def __len__(self):
        return len(self.base)

    def __getitem__(self, k):
        x, y = self.base[k]
        for t in self.transforms:
            x = t(x)
        return x, y


# ------------------------------------------------------------------------------------
# ------------------------------------------------------------------------------------
_MNIST_FILES = {
    True: ("train-images-idx3-ubyte", "train-labels-idx1-ubyte"),
    False: ("t10k-images-idx3-ubyte", "t10k-labels-idx1-ubyte"),
}


def _open_maybe_gz(base):
    for path, opener in ((base, open), (base + ".gz", gzip.open)):
        if os.path.exists(path):
            return opener(path, "rb")
    raise FileNotFoundError(base + "[.gz]")


def read_idx(path_base) -> np.ndarray:
    """Parse an IDX file (MNIST's format: magic 0x0000 <type> <ndim>, big-endian dims)."""
    with _open_maybe_gz(path_base) as f:
        raw = f.read()
    if len(raw) < 4 or raw[0] != 0 or raw[1] != 0:
        raise ValueError(f"{path_base}: not an IDX file")
    dtypes = {0x08: np.uint8, 0x09: np.int8, 0x0B: ">i2", 0x0C: ">i4", 0x0D: ">f4",
              0x0E: ">f8"}
    dt = np.dtype(dtypes[raw[2]])
    ndim = raw[3]
    dims = [int.from_bytes(raw[4 + 4 * k:8 + 4 * k], "big") for k in range(ndim)]
    off = 4 + 4 * ndim
    return np.frombuffer(raw, dtype=dt, count=int(np.prod(dims)), offset=off).reshape(dims)


def load_mnist(root: str, train: bool):
    """MNIST as torchvision's ToTensor() sees it: float32 in [0, 1], [N, 1, 28, 28],
    plus int64 labels.  Looks in root/, root/raw/ and root/MNIST/raw/."""
    img_name, lbl_name = _MNIST_FILES[train]
    for d in (root, os.path.join(root, "raw"), os.path.join(root, "MNIST", "raw")):
        try:
            imgs = read_idx(os.path.join(d, img_name))
            lbls = read_idx(os.path.join(d, lbl_name))
        except FileNotFoundError:
            continue
        x = torch.from_numpy(imgs.astype(np.float32) / 255.0).unsqueeze(1)
        return TensorDataset(x, torch.from_numpy(lbls.astype(np.int64)))
    raise FileNotFoundError(
        f"MNIST IDX files ({img_name}, {lbl_name}) not found under {root} "
        "(this build never downloads; place the files there)")


_CIFAR_BIN = ("cifar-10-batches-bin",
              tuple(f"data_batch_{k}.bin" for k in range(1, 6)), ("test_batch.bin",))
_CIFAR_PY = ("cifar-10-batches-py",
             tuple(f"data_batch_{k}" for k in range(1, 6)), ("test_batch",))


def _cifar_bin(path):
    """One CIFAR-10 binary batch: records of 1 label byte + 3072 pixel bytes (the R, G
    and B 32x32 planes, row-major)."""
    raw = np.fromfile(path, dtype=np.uint8)
    if raw.size % 3073:
        raise ValueError(f"{path}: not a CIFAR-10 binary batch ({raw.size} bytes)")
    rec = raw.reshape(-1, 3073)
    return rec[:, 1:].reshape(-1, 3, 32, 32), rec[:, 0].astype(np.int64)


class _ArrayOnlyUnpickler:
    """Unpickler for the CIFAR-10 python batches that resolves only numpy's array
    reconstruction (the batches hold a dict of bytes keys, a uint8 array and a label
    list); any other global in the file is refused."""
    _ALLOWED = {("numpy.core.multiarray", "_reconstruct"), ("numpy._core.multiarray",
                                                              "_reconstruct"),
                ("numpy", "ndarray"), ("numpy", "dtype")}

    @classmethod
    def load(cls, f):
        import pickle

        class U(pickle.Unpickler):
            def find_class(self, module, name):
                if (module, name) not in cls._ALLOWED:
                    raise pickle.UnpicklingError(f"refusing {module}.{name}")
                return super().find_class(module, name)
        return U(f, encoding="bytes").load()


def _cifar_py(path):
    with open(path, "rb") as f:
        d = _ArrayOnlyUnpickler.load(f)
    x = np.asarray(d[b"data"], dtype=np.uint8).reshape(-1, 3, 32, 32)
    return x, np.asarray(d[b"labels"], dtype=np.int64)


def load_cifar10(root: str, train: bool):
    """CIFAR-10 as torchvision's CIFAR10 + ToTensor() sees it: float32 in [0, 1],
    [N, 3, 32, 32] (channel planes R, G, B), int64 labels; train = the 5 data batches in
    order (50 000), test = test_batch (10 000).  Reads the binary distribution
    (cifar-10-batches-bin) or the python one torchvision downloads (cifar-10-batches-py)
    under root/; never downloads."""
    for sub, trn, tst, reader in (_CIFAR_BIN + (_cifar_bin,), _CIFAR_PY + (_cifar_py,)):
        files = [os.path.join(root, sub, f) for f in (trn if train else tst)]
        if all(os.path.exists(f) for f in files):
            parts = [reader(f) for f in files]
            x = np.concatenate([p[0] for p in parts])
            y = np.concatenate([p[1] for p in parts])
            return TensorDataset(torch.from_numpy(x.astype(np.float32) / 255.0),
                                 torch.from_numpy(y))
    raise FileNotFoundError(
        f"CIFAR-10 batches not found under {root} (cifar-10-batches-bin/ or "
        "cifar-10-batches-py/; this build never downloads)")


_LOADERS = {"MNIST": load_mnist, "CIFAR10": load_cifar10}


class DatasetFromConfig:
    """train/validation/test Subsets of ConcatDataset([train, test]) by the config's
    ranges (data.py:134-158).  Reads local files of config.dataset_name: "MNIST" (IDX)
    or "CIFAR10" (binary or python batches), from datasets_path/<dataset_name>/ like
    the reference.  Extra config.transforms are applied per item like torchvision's
    Compose after ToTensor."""

    def __init__(self, datasets_path, config):
        self.config = config
        name = getattr(config, "dataset_name", "MNIST")
        root = os.path.join(datasets_path, name)
        if name not in _LOADERS:
            raise NotImplementedError(f"dataset {name!r}: local MNIST and CIFAR10 are "
                                      "supported")
        train_full = _LOADERS[name](root, True)
        test_full = _LOADERS[name](root, False)
        transforms = list(getattr(config, "transforms", []) or [])
        if transforms:
            train_full, test_full = (_Transformed(d, transforms)
                                     for d in (train_full, test_full))
        self.data_full = ConcatDataset([train_full, test_full])
        self.train = Subset(self.data_full, config.train_range)
        self.validation = Subset(self.data_full, config.validation_range)
        self.test = Subset(self.data_full, config.test_range)

    @staticmethod
    def load_full(dataset):
        """(images, labels) of a whole dataset in one batch (data.py:160-162)."""
        return next(iter(DataLoader(dataset, batch_size=len(dataset))))
