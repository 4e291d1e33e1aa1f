"""Conditioning of the synthetic full-scale Kxx (tools/fullscale.py's MNIST-/CIFAR-like
images): the leading blocks' extreme eigenvalues, numpy's Cholesky of them, and a bitwise
repeat of the HIP build (the kernel is deterministic).

    python tools/cond_probe.py [--config cifar10] [--n 16384] [--k 256]
"""
import argparse
import importlib
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cnn-gp_amd"), ROOT, os.path.join(ROOT, "tools")]

from fullscale import mnist_like  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cifar10")
    ap.add_argument("--n", type=int, default=16384)
    ap.add_argument("--k", type=int, default=256)
    args = ap.parse_args()
    cfg = importlib.import_module(f"configs.{args.config}")
    C = getattr(cfg, "in_channels", 1)
    side = 32 if C == 3 else 28
    X = mnist_like(args.n, C, side, 0)[:args.k].to("cuda")
    m = cfg.initial_model.to("cuda", torch.float64)
    with torch.no_grad():
        K1 = m(X).cpu().numpy()
        K2 = m(X).cpu().numpy()
    print("bitwise repeat:", np.array_equal(K1, K2))
    for k in (16, 66, 67, 128, args.k):
        if k > args.k:
            continue
        A = K1[:k, :k]
        A = np.triu(A) + np.triu(A, 1).T
        w = np.linalg.eigvalsh(A)
        try:
            np.linalg.cholesky(A)
            ch = "ok"
        except np.linalg.LinAlgError as e:
            ch = f"fails ({e})"
        print(f"k={k}: eig min {w[0]:.3e} max {w[-1]:.3e} cond {w[-1] / max(abs(w[0]), 1e-300):.2e}"
              f" cholesky {ch}")
    d = np.diag(K1)
    off = K1[np.triu_indices(args.k, 1)]
    print(f"diag {d.min():.6e}..{d.max():.6e}; off-diag {off.min():.6e}..{off.max():.6e}; "
          f"max corr {np.max(off / np.sqrt(np.outer(d, d))[np.triu_indices(args.k, 1)]):.12f}")


if __name__ == "__main__":
    main()
