"""Uninitialised / out-of-bounds reads show up as NaN: the caching allocator's free blocks
are filled with NaN (or zeros, the control) before a build, so every buffer the build
allocates without writing first starts as NaN.  A kernel that reads such memory — even
multiplied by a zero weight, 0·NaN = NaN — puts NaN or different values into K.  Builds
rank 0's full-scale Kxx strip (tools/fullscale.py's images, world size ``--world``) and a
solve of its leading block, after each fill, and compares.

    python tools/poison_probe.py [--config cifar10] [--n 16384] [--world 4] [--gb 64]
"""
import argparse
import importlib
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cnn-gp_amd"), ROOT, os.path.join(ROOT, "tools")]

import cnn_gp  # noqa: E402
from cnn_gp.gram import gram_strip, model_kern, row_slice, strip_plan  # noqa: E402
from fullscale import mnist_like  # noqa: E402


def fill_free(dev, value, gb):
    """allocate ~gb GB of blocks (large: 1 GB .. 2 MB, small: 4 KB .. 512 KB) filled with
    value, then free them: they stay in the caching allocator's pools"""
    torch.cuda.empty_cache()
    held = []
    left = int(gb * 2 ** 30)
    for size in [2 ** 30] * 16 + [2 ** 28] * 16 + [2 ** 24] * 64 + [2 ** 21] * 256:
        if left <= 0:
            break
        try:
            held.append(torch.full((size // 8,), value, dtype=torch.float64, device=dev))
            left -= size
        except torch.OutOfMemoryError:
            break
    for size in [2 ** 19, 2 ** 16, 2 ** 12] * 400:
        held.append(torch.full((size // 8,), value, dtype=torch.float64, device=dev))
    torch.cuda.synchronize()
    del held


def build(cfg_name, n, world, dev):
    cfg = importlib.import_module(f"configs.{cfg_name}")
    model = cfg.initial_model.to(dev, torch.float64)
    C = getattr(cfg, "in_channels", 1)
    side = 32 if C == 3 else 28
    X = mnist_like(n, C, side, 0).to(dev, torch.float64)
    r0, r1 = strip_plan(n, None, world)[0]
    K = torch.full((r1, n), float("nan"), dtype=torch.float64, device=dev)
    with torch.no_grad():
        gram_strip(model_kern(model), row_slice(X, r0, n), None, 4096, (0, r1),
                   out=K[:, r0:], dtype=torch.float64)
    L = min(2048, r1)
    lead = K[:L, :L].contiguous()
    Y = torch.ones((L, 10), dtype=torch.float64, device=dev)
    try:
        cnn_gp.solve_system(lead.clone(), Y, overwrite_a=True)
        solved = "solve ok"
    except Exception as e:  # noqa: BLE001
        solved = f"solve: {e}"
    torch.cuda.synchronize()
    return K.cpu(), solved


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="cifar10,mnist_as_tf,mnist_paper_convnet_gp")
    ap.add_argument("--n", type=int, default=16384)
    ap.add_argument("--world", type=int, default=4)
    ap.add_argument("--gb", type=float, default=48)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    bad = 0
    for name in args.configs.split(","):
        fill_free(dev, 0.0, args.gb)
        K0, s0 = build(name, args.n, args.world, dev)
        fill_free(dev, float("nan"), args.gb)
        K1, s1 = build(name, args.n, args.world, dev)
        up = torch.triu(torch.ones(K0.shape, dtype=torch.bool), diagonal=0)
        nan0 = int(torch.isnan(K0[up]).sum())
        nan1 = int(torch.isnan(K1[up]).sum())
        diff = ~((K0 == K1) | (torch.isnan(K0) & torch.isnan(K1)))
        nd = int(diff[up].sum())
        msg = (f"{name}: strip {tuple(K0.shape)}, zero-filled: NaN {nan0}, {s0}; NaN-filled: "
               f"NaN {nan1}, {s1}; entries differing {nd}")
        if nd:
            idx = torch.nonzero(diff & up)[:6].tolist()
            msg += " first " + str([(i, j, float(K0[i, j]), float(K1[i, j])) for i, j in idx])
        bad += bool(nd or nan0 or nan1)
        print(msg, flush=True)
    print(f"poison_probe: {'FAIL' if bad else 'ok'}", flush=True)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
