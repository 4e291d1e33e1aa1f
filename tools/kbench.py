"""Kernel microbenchmark: time single libcnngp launches on one full Gram tile with HIP
events (interleaved rounds in one process), report GB/s of algorithmic traffic.

    python tools/kbench.py [--tile 1024] [--reps 10]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cnn-gp_amd"), ROOT]

import torch  # noqa: E402

from cnn_gp import _native as N  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tile", type=int, default=1024)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--dtype", default="f64")
    ap.add_argument("--only", default="", help="comma-separated case-name substrings")
    ap.add_argument("--rounds", type=int, default=3)
    args = ap.parse_args()
    dt = torch.float64 if args.dtype == "f64" else torch.float32
    sfx = args.dtype
    lib = N.load()
    B = args.tile
    P = B * B
    dev = "cuda"
    s = torch.cuda.current_stream().cuda_stream
    g = torch.Generator(device="cpu").manual_seed(0)
    item = torch.tensor([], dtype=dt).element_size()

    # realistic covariance maps: xy = 0.5 * sqrt(xx yy) so the ReLU sees |cos| < 1
    def maps(h):
        var = (torch.rand((2 * B, h, h), generator=g, dtype=dt) + 0.5).to(dev)
        xy = (0.5 * (var[:B, None] * var[None, B:]).sqrt()).reshape(P, h, h).contiguous()
        return xy, var[:B].contiguous(), var[B:].contiguous()

    cases = []
    for h, k, st, off, post in [(28, 7, 1, -3, 0), (28, 7, 1, -3, 1), (28, 7, 1, -3, 2),
                                (28, 3, 1, -1, 0), (28, 3, 1, -1, 1), (14, 3, 1, -1, 1),
                                (7, 3, 1, -1, 1), (28, 28, 1, 0, 0), (28, 1, 2, 0, 0),
                                (28, 3, 2, -1, 1), (28, 7, 1, -3, 3), (28, 3, 1, -1, 3)]:
        cases.append(("conv", h, k, st, off, post))
    cases += [("relu", 28, 0), ("relu", 28, 1), ("copy", 28)]
    results = {}
    bufs = {}
    for c in cases:
        h = c[1]
        if h not in bufs:
            bufs[h] = maps(h)
    for c in cases:
        h = c[1]
        xy, vx, vy = bufs[h]
        if c[0] == "conv":
            _, h, k, st, off, post = c
            ho = (h + 2 * (-off) - (k - 1) - 1) // st + 1
            out = torch.empty((P, ho, ho), dtype=dt, device=dev)
            a = N.ConvArgs()
            a.in_, a.out = N.ptr(xy), N.ptr(out)
            a.nmaps, a.n1, a.n2 = P, B, B
            a.h, a.w, a.ho, a.wo = h, h, ho, ho
            a.taps, a.offset, a.stride, a.dilation = k, off, st, 1
            a.weight, a.bias, a.post = 1.0 / (k * k), 0.1, 1 if post else 0
            a.flags = {2: N.CGP_FLAG_EXACT_RELU, 3: N.CGP_FLAG_GENERIC_CONV}.get(post, 0)
            if post:
                pv = bufs.get(ho, maps(ho))
                a.post_xx, a.post_yy = N.ptr(pv[1]), N.ptr(pv[2])
            fn = getattr(lib, f"cgp_conv_{sfx}")
            launch = (lambda fn=fn, a=a: N.check(fn(a, s), "conv"))
            nbytes = (P * h * h + P * ho * ho + (2 * B * ho * ho if post else 0)) * item
            name = f"conv{k}s{st}{['', '+relu', '+relu(exact)', '+relu(generic)'][post]}@{h}->{ho}"
            keep = out
        elif c[0] == "relu":
            out = torch.empty_like(xy)
            r = N.ReluArgs()
            r.xy, r.out, r.xx, r.yy = N.ptr(xy), N.ptr(out), N.ptr(vx), N.ptr(vy)
            r.nmaps, r.n1, r.n2, r.hw = P, B, B, h * h
            r.flags = N.CGP_FLAG_EXACT_RELU if c[2] else 0
            fn = getattr(lib, f"cgp_relu_{sfx}")
            launch = (lambda fn=fn, r=r: N.check(fn(r, s), "relu"))
            nbytes = (2 * P * h * h + 2 * B * h * h) * item
            name = f"relu{'(exact)' if c[2] else ''}@{h}"
            keep = out
        else:
            out = torch.empty_like(xy)
            launch = (lambda out=out, xy=xy: out.copy_(xy))
            nbytes = 2 * P * h * h * item
            name = f"torch_copy@{h}"
            keep = out
        if args.only and not any(o == name for o in args.only.split(",")):
            continue
        results[name] = (launch, nbytes, keep)
    times = {k: [] for k in results}
    for _ in range(args.rounds):            # interleaved rounds
        for name, (launch, nbytes, _) in results.items():
            launch()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.reps):
                launch()
            e1.record()
            e1.synchronize()
            times[name].append(e0.elapsed_time(e1) / args.reps)
    for name, (launch, nbytes, _) in results.items():
        ms = min(times[name])
        print(f"{name:28s} {ms:8.3f} ms  {nbytes / ms / 1e6:8.1f} GB/s  "
              f"({P * (int(name.split('->')[-1]) if '->' in name else 28) ** 2 / ms / 1e6:.1f} Gpx/s)")


if __name__ == "__main__":
    main()
