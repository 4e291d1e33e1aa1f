"""Repeatability of the full-scale Kxx strips with several ranks sharing one GPU (the
gloo rehearsal's geometry): every rank builds its strip of tools/fullscale.py's Kxx the
way cnn_gp.pipeline.classify_distributed does (X[r0:] bound, strip_tiles in local rows),
REPS times, and checks each repetition bit-equal to its first (the kernels are
deterministic); rank 0 also starts the solver warm-up thread beside each build, as the
pipeline does, and checks its leading block against model(X[:L]).

    torchrun --nproc-per-node 4 tools/strip_stress.py [--config cifar10] [--n 16384]
"""
import argparse
import datetime
import importlib
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cnn-gp_amd"), ROOT, os.path.join(ROOT, "tools")]

import cnn_gp  # noqa: E402
from cnn_gp.gram import gram_strip, model_kern, row_slice, strip_plan  # noqa: E402
from fullscale import mnist_like  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cifar10")
    ap.add_argument("--n", type=int, default=16384)
    ap.add_argument("--reps", type=int, default=6)
    ap.add_argument("--lead", type=int, default=256)
    ap.add_argument("--no-warm", action="store_true")
    args = ap.parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    if world > 1:
        dist.init_process_group("gloo", timeout=datetime.timedelta(seconds=300))
    cfg = importlib.import_module(f"configs.{args.config}")
    model = cfg.initial_model.to(dev, torch.float64)
    C = getattr(cfg, "in_channels", 1)
    side = 32 if C == 3 else 28
    n = args.n
    X = mnist_like(n, C, side, 0).to(dev, torch.float64)
    r0, r1 = strip_plan(n, None, world)[rank]
    kern = model_kern(model)
    first = None
    bad_reps = 0
    for rep in range(args.reps):
        if world > 1:
            dist.barrier()
        t = time.perf_counter()
        warming = cnn_gp.warm_up_solver(dev) if (rank == 0 and not args.no_warm) else None
        out = torch.full((r1 - r0, n), float("nan"), dtype=torch.float64, device=dev)
        with torch.no_grad():
            gram_strip(kern, row_slice(X, r0, n), None, 4096, (0, r1 - r0), out=out[:, r0:],
                       dtype=torch.float64)
        torch.cuda.synchronize()
        if warming is not None:
            warming.join()
        el = time.perf_counter() - t
        up = torch.triu(torch.ones((r1 - r0, n - r0), dtype=torch.bool, device=dev))
        nan_up = int(torch.isnan(out[:, r0:][up]).sum())
        msg = f"rank {rank} rep {rep}: {el:.2f} s, NaN in the upper strip {nan_up}"
        h = out.cpu()
        if first is None:
            first = h
        else:
            same = (h == first) | (torch.isnan(h) & torch.isnan(first))
            nd = int((~same).sum())
            msg += f", entries differing from rep 0: {nd}"
            if nd:
                idx = torch.nonzero(~same)[:4].tolist()
                msg += " first " + str([(r0 + i, j, float(h[i, j]), float(first[i, j]))
                                        for i, j in idx])
                bad_reps += 1
        if rank == 0 and args.lead:
            L = min(args.lead, r1 - r0)
            with torch.no_grad():
                ref = model(X[:L]).cpu().numpy()
            got = h[:L, :L].numpy()
            iu = np.triu_indices(L)
            nl = int((got[iu] != ref[iu]).sum())
            msg += f", leading {L}x{L} upper entries != model(X[:{L}]): {nl}"
            if nl:
                bad_reps += 1
        print(msg, flush=True)
    if world > 1:
        t = torch.tensor([bad_reps])
        dist.all_reduce(t)
        bad_reps = int(t)
        dist.destroy_process_group()
    if rank == 0:
        print(f"strip_stress: {'FAIL' if bad_reps else 'ok'} ({bad_reps} bad repetitions)",
              flush=True)
    return 1 if bad_reps else 0


if __name__ == "__main__":
    sys.exit(main())
