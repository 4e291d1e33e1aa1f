"""How save_K's tile overlap behaves on the device (kernel_save_tools.save_K ``overlap``):
save_kernel.py:21-24's kern timed per call in every thread — H2D (pageable x.cuda()),
forward's launches, the wait in .cpu() — for overlap 1, 2, 3, with the dataset pageable
or pinned and the tile recipes on or off; prints ms per tile and, for overlap > 1, how
much of one thread's H2D / launch work ran while another thread waited on the GPU.

    python tools/dropin_overlap_probe.py [--config mnist_paper_convnet_gp] [--tile 200]
"""
import argparse
import contextlib
import gc
import importlib
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cnn-gp_amd"), ROOT, os.path.join(ROOT, "tools")]

import torch  # noqa: E402
from torch.utils.data import TensorDataset  # noqa: E402

from cnn_gp import netplan  # noqa: E402
from cnn_gp.kernel_save_tools import save_K  # noqa: E402
from dropin_probe import MemH5  # noqa: E402


def overlap_share(ev):
    """share of the host phases (H2D + launches) of each call that ran while another
    thread's call sat in its GPU wait"""
    waits = [(e[3], e[4], e[0]) for e in ev]
    tot = hid = 0.0
    for th, t0, t1, t2, t3 in ev:
        tot += t2 - t0
        for a, b, th2 in waits:
            if th2 != th:
                hid += max(0.0, min(t2, b) - max(t0, a))
    return hid / tot if tot else 0.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="mnist_paper_convnet_gp")
    ap.add_argument("--n", type=int, default=2048)
    ap.add_argument("--tile", default="200", help="tile sizes, run in turn (e.g. 200,1024)")
    ap.add_argument("--overlaps", default="1,2,3")
    ap.add_argument("--pins", default="0,1")
    ap.add_argument("--recipes", default="1,0")
    ap.add_argument("--reps", type=int, default=1)
    ap.add_argument("--gc", default="1", help="1: Python's collector on (default), 0: off, "
                    "0,1: both, around the timed save_K")
    ap.add_argument("--model-f64", action="store_true",
                    help="float64 weight buffers with the float32 images")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    cfg = importlib.import_module(f"configs.{args.config}")
    model = cfg.initial_model.to(dev, torch.float64 if args.model_f64 else torch.float32)
    C = getattr(cfg, "in_channels", 1)
    side = 32 if C == 3 else 28
    X0 = torch.rand((args.n, C, side, side), generator=torch.Generator().manual_seed(0))
    ev = []

    def kern(x, x2, same, diag):
        with torch.no_grad():
            t0 = time.perf_counter()
            a, b = x.cuda(dev), x2.cuda(dev)
            t1 = time.perf_counter()
            k = model(a, b, same, diag)
            t2 = time.perf_counter()
            out = k.detach().cpu().numpy()
            ev.append((threading.get_ident(), t0, t1, t2, time.perf_counter()))
            return out

    for pin in [bool(int(v)) for v in args.pins.split(",")]:
        X = X0                              # save_K(pin=...) pins its own copy
        ds = TensorDataset(X, torch.zeros(args.n, dtype=torch.int64))
        for recipes in [bool(int(v)) for v in args.recipes.split(",")]:
            netplan.RECIPE_MAX_BYTES = (512 << 20) if recipes else 0
            for tile, ov, gco in [(int(b), int(v), int(g)) for b in args.tile.split(",")
                                  for v in args.overlaps.split(",")
                                  for g in args.gc.split(",") for _ in range(args.reps)]:
                with contextlib.redirect_stdout(sys.stderr):
                    save_K(MemH5(), kern, "Kxx", ds, None, False, tile, overlap=ov,
                           print_interval=1e9, pin=pin)
                    torch.cuda.synchronize()
                    ev.clear()
                    if not gco:
                        gc.disable()
                    t = time.perf_counter()
                    save_K(MemH5(), kern, "Kxx", ds, None, False, tile, overlap=ov,
                           print_interval=1e9, pin=pin)
                    el = time.perf_counter() - t
                    gc.enable()
                n = len(ev)
                h2d = sum(e[2] - e[1] for e in ev) / n * 1e3
                launch = sum(e[3] - e[2] for e in ev) / n * 1e3
                print(f"B={tile} pin={int(pin)} recipes={int(recipes)} gc={gco} overlap={ov}: "
                      f"{el / n * 1e3:.3f} ms/tile ({args.n * (args.n - 1) / 2 / el / 1e6:.1f} "
                      f"M pairs/s); per call h2d {h2d:.3f} "
                      f"launch {launch:.3f} wait {sum(e[4] - e[3] for e in ev) / n * 1e3:.3f} "
                      f"(ms); host phases hidden behind another thread's wait "
                      f"{overlap_share(ev):.2f}", flush=True)


if __name__ == "__main__":
    main()
