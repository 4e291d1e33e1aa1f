"""Per-op cost of the whole-network kernel: synthetic chains of one op type at one map
size (N repeats + a final full-window conv), timed per pair with HIP events.

    python tools/netops.py [--tile 512] [--repeat 16]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cnn-gp_amd"), ROOT]

import torch  # noqa: E402

import cnn_gp as G  # noqa: E402
from cnn_gp import _native as N  # noqa: E402


def chain(kind, side, n):
    mods = []
    for _ in range(n):
        if kind == "conv3+relu":
            mods += [G.Conv2d(3, var_bias=0.1), G.ReLU()]
        elif kind == "conv3":
            mods += [G.Conv2d(3, var_bias=0.1)]
        elif kind == "conv7+relu":
            mods += [G.Conv2d(7, var_bias=0.1), G.ReLU()]
        elif kind == "relu":           # standalone: the ReLU output feeds two consumers
            mods += [G.Sum([G.Sequential(), G.ReLU()])]
        elif kind == "block":          # identity resnet block
            mods += [G.resnet_block(1)]
    mods += [G.Conv2d(side, padding=0)]
    return G.Sequential(G.Conv2d(3, var_bias=0.5), *mods)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tile", type=int, default=512)
    ap.add_argument("--repeat", type=int, default=16)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    B = args.tile
    s = torch.cuda.current_stream()
    sh = s.cuda_stream
    lib = N.load()
    base = {}
    for side in (28, 14, 7):
        for kind in ("none", "relu", "conv3", "conv3+relu", "conv7+relu", "block"):
            if kind == "conv7+relu" and side != 28:
                continue
            n = 0 if kind == "none" else args.repeat
            m = chain(kind if n else "relu", side, n).double().cuda()
            g = torch.Generator().manual_seed(0)
            X = torch.rand((B, 1, side, side), generator=g, dtype=torch.float64).cuda()
            Z = torch.rand((B, 1, side, side), generator=g, dtype=torch.float64).cuda()
            plan = m._plan(side, side)
            net = m._net_plan(plan, 8)
            if net is None:
                print(side, kind, "unsupported")
                continue
            var0 = torch.empty((2 * B, side, side), dtype=torch.float64, device="cuda")
            N.check(lib.cgp_moments_var_f64(N.ptr(X), N.ptr(Z), B, B, 1, side * side,
                                            N.ptr(var0[:B]), N.ptr(var0[B:]), sh), "mv")
            var = plan.run_variances(var0[:B], var0[B:], B, B, False, sh, need=net.need_var)
            out = torch.empty((B, B), dtype=torch.float64, device="cuda")
            net.run(X, Z, var, B, B, False, sh, 0, out=out)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(args.reps):
                net.run(X, Z, var, B, B, False, sh, 0, out=out)
            e1.record(s)
            e1.synchronize()
            ms = e0.elapsed_time(e1) / args.reps
            occ = lib.cgp_net_occupancy(net.lds_elems * 8, 1, 4 if net.dual else 0, 1)
            if kind == "none":
                base[side] = ms
                print(f"{side:3d} {'base':12s} ops={net.n_ops:3d} occ={occ:2d} {ms:8.3f} ms/tile")
            else:
                per = (ms - base[side]) / args.repeat / (B * B) * 1e9 * 256 * occ / 1e3
                print(f"{side:3d} {kind:12s} ops={net.n_ops:3d} occ={occ:2d} {ms:8.3f} ms/tile "
                      f" {(ms - base[side]) / args.repeat * 1e3 / (B * B) * 1e3:8.3f} ps/pair/op"
                      f"  ~{per:7.1f} k block-cycles@2.4GHz/op")


if __name__ == "__main__":
    main()
