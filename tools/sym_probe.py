"""Is K(x_a, x_b) bit-equal to K(x_b, x_a) on the device?  The kernel computes i < j on
diagonal tiles and mirrors, so an entry below the diagonal is the (j, i) evaluation; this
probe measures how far the two orientations differ for single pairs and for a tile.

    python tools/sym_probe.py
"""
import importlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cnn-gp_amd"), ROOT, os.path.join(ROOT, "tools")]

import torch  # noqa: E402

from fullscale import mnist_like  # noqa: E402


def main():
    for name in ("mnist_paper_convnet_gp", "mnist_as_tf"):
        m = importlib.import_module(f"configs.{name}").initial_model.to("cuda", torch.float64)
        X = mnist_like(64, 1, 28, 0).cuda()
        with torch.no_grad():
            A = m(X[:32], X[32:], False, False)
            Bt = m(X[32:], X[:32], False, False).T
            K = m(X)
        d = ((A - Bt).abs() / A.abs()).max().item()
        neq = int((A != Bt).sum())
        dk = ((K[:32, 32:] - A).abs() / A.abs()).max().item()
        print(f"{name}: K(a,b) vs K(b,a): {neq}/{A.numel()} differ, max rel {d:.2e}; "
              f"Kxx tile vs Kxz: max rel {dk:.2e}")


if __name__ == "__main__":
    main()
