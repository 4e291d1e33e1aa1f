"""Calibrate the CPU baseline (oracle/torch_cpu.py) against the REFERENCE itself, in the
build container only (the reference is not on the GPU box):

    python tools/calibrate_cpu.py [--threads 8] [--reps 3]

SURVEY.md §8(d): C1 = mnist_paper_convnet_gp, X = Z = 128 random 1×28×28 images, Kxx on
the CPU.  Both are timed on the same cores with the same torch thread count, fp64
(``.double()``, the build's dtype) and fp32 (the reference's production dtype); the
ratio restatement/reference is what bench.py's cpu_baseline quotes next to its own
measurement on the GPU box's host.  Also mnist_as_tf (C3's architecture) on 64 images.
Also cifar10 (configs[4]'s network, 3×32×32) on 48 images.  The reference is imported
with the two shims SURVEY.md §8(c) records (stub torchvision, np.int = int); nothing of
it is copied.  Output: profiles/r4/cpu_calibration.json.
"""
import argparse
import importlib
import json
import os
import sys
import time
import types

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def load_reference():
    np.int = int
    tv = types.ModuleType("torchvision")
    tv.datasets = types.SimpleNamespace(MNIST=None, CIFAR10=None)
    tv.transforms = types.SimpleNamespace(ToTensor=None, Compose=None)
    sys.modules["torchvision"] = tv
    sys.path.insert(0, "/root/reference")
    import cnn_gp  # noqa: F401  (the reference's package)
    return importlib


def best_of(fn, reps):
    best = float("inf")
    out = None
    for _ in range(reps):
        t0 = time.perf_counter()
        out = fn()
        best = min(best, time.perf_counter() - t0)
    return best, out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    import torch
    torch.set_num_threads(args.threads)
    imp = load_reference()
    sys.path.insert(0, ROOT)
    from oracle import specs, torch_cpu
    res = {"threads": args.threads, "nproc": os.cpu_count(),
           "cpu_model": next((ln.split(":", 1)[1].strip() for ln in open("/proc/cpuinfo")
                              if ln.startswith("model name")), "?"),
           "torch": torch.__version__, "cases": []}
    for cfg_name, n in (("mnist_paper_convnet_gp", 128), ("mnist_as_tf", 64), ("cifar10", 48)):
        cfg = imp.import_module(f"configs.{cfg_name}")
        spec = specs.CONFIGS[cfg_name]()
        g = torch.Generator().manual_seed(0)
        for dtn, dt in (("f64", torch.float64), ("f32", torch.float32)):
            C, side = specs.GEOMETRY[cfg_name]
            X = torch.rand((n, C, side, side), generator=g, dtype=dt)
            model = cfg.initial_model.to(dt)
            with torch.no_grad():
                t_ref, k_ref = best_of(lambda: model(X), args.reps)
            t_port, k_port = best_of(lambda: torch_cpu.kernel(spec, X), args.reps)
            rel = float(((k_port - k_ref).abs() / k_ref.abs()).max())
            pairs = n * n             # the reference evaluates the whole same tile
            res["cases"].append({
                "config": cfg_name, "dtype": dtn, "images": n, "pairs": pairs,
                "reference_s": round(t_ref, 3), "restatement_s": round(t_port, 3),
                "reference_pairs_per_s": round(pairs / t_ref, 1),
                "restatement_pairs_per_s": round(pairs / t_port, 1),
                "restatement_over_reference": round(t_ref / t_port, 3),
                "max_rel_diff": rel})
            print(json.dumps(res["cases"][-1]), flush=True)
            cfg.initial_model.to(torch.float32)
    out = os.path.join(ROOT, "profiles", "r4", "cpu_calibration.json")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    json.dump(res, open(out, "w"), indent=1)
    print("wrote", out)


if __name__ == "__main__":
    main()
