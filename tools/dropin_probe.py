"""Where the per-tile drop-in path (bench.py ``dropin``: save_kernel.py's loop through
save_K) spends its host time: the loop under cProfile, plus the per-tile split between
the kern call's pieces (H2D, forward launch, D2H + sync) timed with perf_counter.

    python tools/dropin_probe.py [--config mnist_paper_convnet_gp] [--n 2048] [--tile 200]
"""
import argparse
import contextlib
import cProfile
import importlib
import io
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cnn-gp_amd"), ROOT]

import torch  # noqa: E402
from torch.utils.data import TensorDataset  # noqa: E402

from cnn_gp.data import ProductIterator  # noqa: E402
from cnn_gp.kernel_save_tools import save_K  # noqa: E402


class MemH5:
    def __init__(self):
        self.d = {}

    def keys(self):
        return self.d.keys()

    def create_dataset(self, name, shape, dtype, fillvalue, chunks, maxshape):
        import numpy as np
        self.d[name] = np.full(shape, fillvalue, dtype=dtype)
        return self.d[name]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="mnist_paper_convnet_gp")
    ap.add_argument("--n", type=int, default=2048)
    ap.add_argument("--tile", type=int, default=200)
    ap.add_argument("--pin", action="store_true", help="the dataset tensor in pinned memory")
    ap.add_argument("--dtype", default="f32", choices=["f64", "f32"])
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    cfg = importlib.import_module(f"configs.{args.config}")
    model = cfg.initial_model.to(dev)
    C = getattr(cfg, "in_channels", 1)
    side = 32 if C == 3 else 28
    X = torch.rand((args.n, C, side, side), generator=torch.Generator().manual_seed(0))
    if args.dtype == "f64":
        X, model = X.double(), model.double()
    if args.pin:
        X = X.pin_memory()
    ds = TensorDataset(X, torch.zeros(args.n, dtype=torch.int64))

    def kern(x, x2, same, diag):
        with torch.no_grad():
            return model(x.cuda(dev), x2.cuda(dev), same, diag).detach().cpu().numpy()

    with contextlib.redirect_stdout(sys.stderr):
        save_K(MemH5(), kern, "Kxx", ds, None, False, args.tile)     # warm
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        save_K(MemH5(), kern, "Kxx", ds, None, False, args.tile, print_interval=1e9)
        el = time.perf_counter() - t0
    tiles = len(ProductIterator(args.tile, ds, None))
    print(f"save_K loop: {el * 1e3:.1f} ms, {tiles} tiles, {el / tiles * 1e3:.3f} ms/tile, "
          f"{args.n * (args.n - 1) / 2 / el / 1e6:.1f} M pairs/s")

    # per-piece split over the same tiles
    parts = {"batches": 0.0, "h2d": 0.0, "forward_host": 0.0, "kernel_wait": 0.0,
             "d2h": 0.0, "isfinite+write": 0.0}
    out = MemH5().create_dataset("K", (1, args.n, args.n), "float32", float("nan"), None, None)
    import numpy as np
    it = iter(ProductIterator(args.tile, ds, None))
    for _ in range(tiles):
        t = time.perf_counter()
        same, (i, (x, _)), (j, (x2, _)) = next(it)
        t1 = time.perf_counter()
        xd, x2d = x.cuda(dev), x2.cuda(dev)
        t2 = time.perf_counter()
        with torch.no_grad():
            k = model(xd, x2d, same, False)
        t3 = time.perf_counter()
        torch.cuda.synchronize()
        t4 = time.perf_counter()
        kh = k.cpu().numpy()
        t5 = time.perf_counter()
        assert np.all(np.isfinite(kh))
        out[0, i:i + len(x), j:j + len(x2)] = kh
        t6 = time.perf_counter()
        for key, a, b in (("batches", t, t1), ("h2d", t1, t2), ("forward_host", t2, t3),
                          ("kernel_wait", t3, t4), ("d2h", t4, t5), ("isfinite+write", t5, t6)):
            parts[key] += b - a
    print("per tile (ms): " + ", ".join(f"{k} {v / tiles * 1e3:.3f}" for k, v in parts.items()))

    pr = cProfile.Profile()
    with contextlib.redirect_stdout(sys.stderr):
        pr.enable()      # serial (overlap 1): the calling thread runs every kern call
        save_K(MemH5(), kern, "Kxx", ds, None, False, args.tile, print_interval=1e9,
               overlap=1)
        torch.cuda.synchronize()
        pr.disable()
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(40)
    print(s.getvalue())


if __name__ == "__main__":
    main()
