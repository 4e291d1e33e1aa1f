"""Conv2d.propagate alone (cgp_conv, no fused epilogue) on one B = 1024 tile's pair maps
at ConvNet-GP's conv7 28->28 shape — bench.py's conv_stencil_roofline launch, three times,
for rocprofv3 PMC passes (tools/gpu_pmc_r2.sh).

    python tools/stencil_once.py [--config mnist_paper_convnet_gp] [--tile 1024]
"""
import argparse
import importlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cnn-gp_amd"), ROOT]

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="mnist_paper_convnet_gp")
    ap.add_argument("--tile", type=int, default=1024)
    args = ap.parse_args()
    cfg = importlib.import_module(f"configs.{args.config}")
    m = cfg.initial_model.to("cuda", torch.float64)
    x = torch.rand((args.tile, 1, 28, 28), dtype=torch.float64, device="cuda")
    r = bench.conv_stencil_roofline(m, x, args.tile, reps=2)
    print(r["kernel"], r["avg_ms"], "ms", r["achieved"], "GB/s", flush=True)


if __name__ == "__main__":
    main()
