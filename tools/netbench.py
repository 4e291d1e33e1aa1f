"""Time the whole-network kernel (cgp_net_*) on one Kxz / Kxx tile per config, with HIP
events on the launch stream, next to the full forward (variance pipeline included).

    python tools/netbench.py [--tile 1024] [--configs a,b] [--reps 3] [--dtype f64]
"""
import argparse
import importlib
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cnn-gp_amd"), ROOT]

import torch  # noqa: E402

from cnn_gp import _native as N  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tile", type=int, default=1024)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--dtype", default="f64")
    ap.add_argument("--configs", default="mnist_paper_convnet_gp,mnist_paper_residual_cnn_gp,"
                                         "mnist_as_tf,cifar10")
    ap.add_argument("--same", action="store_true", help="Kxx diagonal tile (i<j pairs)")
    ap.add_argument("--data", default="rand", choices=["rand", "zeros", "half", "mnist"],
                    help="image data: uniform, all zero, every pixel 0.5 (switching-"
                         "activity probe: the arithmetic is the same, the toggling is not), "
                         "or MNIST-like (k/255, ~60%% zero pixels, 4-pixel zero border)")
    ap.add_argument("--per-stage", action="store_true",
                    help="also time each stage's launches (multi-pair stages)")
    args = ap.parse_args()
    dt = torch.float64 if args.dtype == "f64" else torch.float32
    B = args.tile
    for name in args.configs.split(","):
        cfg = importlib.import_module(f"configs.{name}")
        m = cfg.initial_model.to("cuda", dt)
        C = getattr(cfg, "in_channels", 1)
        side = 32 if C == 3 else 28
        g = torch.Generator().manual_seed(0)
        X = torch.rand((B, C, side, side), generator=g, dtype=dt).cuda()
        Z = X if args.same else torch.rand((B, C, side, side), generator=g, dtype=dt).cuda()
        if args.data == "mnist":
            def mnist_like(t):
                t = torch.floor(t * 256) / 255
                t[torch.rand(t.shape, generator=g, dtype=dt).to(t.device) < 0.6] = 0.0
                t[..., :4, :] = 0.0
                t[..., -4:, :] = 0.0
                t[..., :, :4] = 0.0
                t[..., :, -4:] = 0.0
                return t
            X = mnist_like(X)
            Z = X if args.same else mnist_like(Z)
        elif args.data != "rand":
            v = 0.0 if args.data == "zeros" else 0.5
            X = torch.full_like(X, v)
            Z = X if args.same else torch.full_like(Z, v)
        plan = m._plan(side, side)
        net = m._net_plan(plan, X.element_size())
        assert net is not None, name
        s = torch.cuda.current_stream()
        sh = s.cuda_stream
        lib = N.load()
        sfx = args.dtype
        var0 = torch.empty((2 * B, side, side), dtype=dt, device="cuda")
        N.check(getattr(lib, f"cgp_moments_var_{sfx}")(N.ptr(X), N.ptr(Z), B, B, C,
                                                        side * side, N.ptr(var0[:B]),
                                                        N.ptr(var0[B:]), sh), "mv")
        var = plan.run_variances(var0[:B], var0[B:], B, B, args.same, sh, need=net.need_var)
        out = torch.empty((B, B), dtype=dt, device="cuda")
        net.run(X, Z, var, B, B, args.same, sh, plan.flags, out=out)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(args.reps):
            net.run(X, Z, var, B, B, args.same, sh, plan.flags, out=out)
        e1.record(s)
        e1.synchronize()
        ms_net = e0.elapsed_time(e1) / args.reps
        t0 = time.perf_counter()
        with torch.no_grad():
            for _ in range(args.reps):
                m(X) if args.same else m(X, Z, False, False)
        torch.cuda.synchronize()
        ms_fwd = (time.perf_counter() - t0) / args.reps * 1e3
        pairs = B * (B - 1) // 2 if args.same else B * B
        if args.per_stage and len(net.stages) > 1:
            from cnn_gp import netplan as NP_
            lib_fn = getattr(lib, f"cgp_net_{sfx}")
            ev = []

            class Timed:
                def __call__(self, a, st):
                    e0 = torch.cuda.Event(enable_timing=True)
                    e1 = torch.cuda.Event(enable_timing=True)
                    e0.record(s)
                    rc = lib_fn(a, st)
                    e1.record(s)
                    ev.append((a._obj.pairs, e0, e1))
                    return rc
            real = N.load

            class Wrap:                 # the library with cgp_net_<sfx> timed
                def __init__(self, lib_):
                    self._lib = lib_
                    setattr(self, f"cgp_net_{sfx}", Timed())

                def __getattr__(self, k):
                    return getattr(self._lib, k)
            wrapped = Wrap(real())
            N.load = lambda: wrapped
            try:
                net.run(X, Z, var, B, B, args.same, sh, plan.flags, out=out)
            finally:
                N.load = real
            torch.cuda.synchronize()
            per = {}
            for pairs_, e0, e1 in ev:
                per[pairs_] = per.get(pairs_, 0.0) + e0.elapsed_time(e1)
            print("   per stage (ms): " + "  ".join(f"{k}p {v:.2f}" for k, v in per.items()))
        it = X.element_size()
        stages = " ".join(
            f"[{st.pairs}p {st.n_ops}ops {st.lds_elems * it * st.pairs}B "
            f"occ(interp)={lib.cgp_net_occupancy(st.lds_elems * it, int(dt == torch.float64), 4 if st.dual else 0, st.pairs)}]"
            for st in net.stages)
        print(f"{name:28s} net {ms_net:8.2f} ms ({pairs / ms_net / 1e3:7.2f} M pairs/s)  "
              f"forward {ms_fwd:8.2f} ms  {stages}")


if __name__ == "__main__":
    main()
