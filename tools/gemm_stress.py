"""Repeatability of a plain device GEMM (torch.matmul, float64) with several processes
sharing one GPU: every rank multiplies the same two seeded matrices REPS times at the
same moment (a barrier before each) and compares each product with its first and with a
host (CPU) product on sampled rows.  A companion of tools/solve_stress.py: it tells a
problem of concurrent library GEMMs apart from one of the factorisation.

    torchrun --nproc-per-node 4 tools/gemm_stress.py [--n 8192] [--reps 6]
"""
import argparse
import datetime
import os
import sys

import torch
import torch.distributed as dist


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=8192)
    ap.add_argument("--reps", type=int, default=6)
    args = ap.parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    if world > 1:
        dist.init_process_group("gloo", timeout=datetime.timedelta(seconds=300))
    g = torch.Generator(device=dev).manual_seed(11)
    A = torch.rand((args.n, args.n), generator=g, device=dev, dtype=torch.float64)
    B = torch.rand((args.n, args.n), generator=g, device=dev, dtype=torch.float64)
    rows = torch.arange(0, args.n, args.n // 8)
    ref = (A[rows.to(dev)].cpu() @ B.cpu())          # host product of 8 rows
    first, bad = None, 0
    for rep in range(args.reps):
        if world > 1:
            dist.barrier()
        C = A @ B
        torch.cuda.synchronize()
        Ch = C.cpu()
        host = float(((Ch[rows] - ref).norm() / ref.norm()))
        msg = f"rank {rank} rep {rep}: vs host {host:.1e}"
        if first is None:
            first = Ch
        else:
            nd = int((Ch != first).sum())
            msg += f", entries differing from rep 0: {nd} (normwise {float((Ch - first).norm() / first.norm()):.1e})"
        bad += bool(not host < 1e-13)
        print(msg, flush=True)
    if world > 1:
        t = torch.tensor([bad])
        dist.all_reduce(t)
        bad = int(t)
        dist.destroy_process_group()
    if rank == 0:
        print(f"gemm_stress: {'FAIL' if bad else 'ok'} ({bad} products off the host's)", flush=True)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
