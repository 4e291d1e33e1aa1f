"""Histogram of the ReLU map's x = (1 - |rho|)/2 per ReLU layer (test infrastructure: the
CPU oracle's recursion on sampled pairs; DESIGN.md §4.1 "range-adaptive ReLU polynomial").
The fp64 closed form picks its polynomial degree from the largest x a wave holds, so this
is the evidence for the sub-interval split points (tools/fit_relu_poly.py ADAPT).

    python tests/relu_x_hist.py mnist_as_tf mnist      # or: rand
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import nngp_oracle as O  # noqa: E402
from oracle import specs  # noqa: E402


def images(n, C, side, kind, rng):
    if kind == "rand":
        return rng.random((n, C, side, side))
    X = np.floor(rng.random((n, C, side, side)) * 256) / 255.0
    X[rng.random(X.shape) < 0.6] = 0.0
    X[..., :4, :] = 0
    X[..., -4:, :] = 0
    X[..., :, :4] = 0
    X[..., :, -4:] = 0
    return X


def main(cfg="mnist_as_tf", kind="mnist", n=24):
    C, side = specs.GEOMETRY[cfg]
    X = images(n, C, side, kind, np.random.default_rng(0))
    stats = []
    orig = O.relu

    def relu(kp):
        xx, yy, xy = kp["xx"], kp["yy"], kp["xy"]
        n1, n2 = xx.shape[0], yy.shape[0]
        H, W = xy.shape[-2:]
        c = xy.reshape(n1, n2, H, W)
        t = xx[:, None] * yy[None] + O.F32_TINY
        x = (1 - np.clip(np.abs(c) / np.sqrt(t), 0, 1)) / 2
        xm = x[np.triu_indices(n1, 1)]
        stats.append((H, xm.reshape(len(xm), -1)))
        return orig(kp)

    O.relu = relu
    try:
        O.kernel(specs.CONFIGS[cfg](), X, X, False, False)
    finally:
        O.relu = orig
    for L, (H, xm) in enumerate(stats):
        mx = xm.max(1)
        q = np.quantile(xm, [0.5, 0.9, 0.99])
        print(f"ReLU {L + 1:2d} {H:2d}x{H:<2d} x median {q[0]:.4f} p90 {q[1]:.4f} p99 {q[2]:.4f} "
              f"max {xm.max():.4f} | per-pair max: median {np.median(mx):.4f} "
              f"p90 {np.quantile(mx, 0.9):.4f}")


if __name__ == "__main__":
    main(*sys.argv[1:3])
