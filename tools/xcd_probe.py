"""Per-XCD balance of the whole-network kernel: every workgroup's exit time (a build with
-DCGP_NET_XCD_PROBE=1, selected with CNNGP_LIB) on one B = 1024 Kxz tile per config.
Workgroup b runs on XCD b % 8; prints, per XCD, when its last workgroup left, relative to
the first exit of the launch, and the whole launch's spread.

    CNNGP_LIB=.../lib_probe.so python tools/xcd_probe.py [--configs a,b] [--tile 1024]
"""
import argparse
import ctypes
import importlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cnn-gp_amd"), ROOT]

import torch  # noqa: E402

from cnn_gp import _native as N  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tile", type=int, default=1024)
    ap.add_argument("--configs", default="mnist_paper_convnet_gp,mnist_as_tf")
    args = ap.parse_args()
    lib = N.load()
    lib.cgp_net_probe_read.restype = ctypes.c_int32
    lib.cgp_net_probe_read.argtypes = [ctypes.c_void_p, ctypes.c_int32]
    B = args.tile
    for name in args.configs.split(","):
        cfg = importlib.import_module(f"configs.{name}")
        m = cfg.initial_model.to("cuda", torch.float64)
        C = getattr(cfg, "in_channels", 1)
        side = 32 if C == 3 else 28
        g = torch.Generator().manual_seed(0)
        X = torch.rand((B, C, side, side), generator=g, dtype=torch.float64).cuda()
        Z = torch.rand((B, C, side, side), generator=g, dtype=torch.float64).cuda()
        for rep in range(3):
            with torch.no_grad():
                m(X, Z, False, False)
            torch.cuda.synchronize()
        n = 1 << 16
        buf = (ctypes.c_uint64 * n)()
        assert lib.cgp_net_probe_read(buf, n) == 0
        t = [v for v in buf]
        # the last launch of the forward is the final stage; its workgroups hold the
        # newest stamps: keep the stamps within 50 ms of the newest
        newest = max(t)
        live = [(b, v) for b, v in enumerate(t) if v and newest - v < 5_000_000]
        t0 = min(v for _, v in live)
        per = {}
        for b, v in live:
            per.setdefault(b % 8, []).append(v - t0)
        span = (newest - t0) / 100.0   # us at 100 MHz
        print(f"{name}: {len(live)} workgroups, exits spread over {span:.1f} us")
        for x in sorted(per):
            last = max(per[x]) / 100.0
            first = min(per[x]) / 100.0
            print(f"  XCD {x}: first exit {first:8.1f} us, last exit {last:8.1f} us")


if __name__ == "__main__":
    main()
