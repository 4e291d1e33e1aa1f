"""Repeatability of the blocked Cholesky (cnn_gp.solve_system, rocSOLVER/rocBLAS) with
several processes sharing one GPU, the way the gloo rehearsal shares it: every rank, REPS
times, starts the solver warm-up thread, builds a Kxz block with the fused kernels
beside it (cifar10, B = 4096), then factors a copy of one fixed well-conditioned SPD matrix
in place and solves.  Each factorisation must succeed and agree with the rank's first one
within TOL (bit equality is reported, not required: the reduction order inside rocBLAS may
change between calls).

    torchrun --nproc-per-node 4 tools/solve_stress.py [--n 16384] [--reps 6]
"""
import argparse
import datetime
import importlib
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cnn-gp_amd"), ROOT, os.path.join(ROOT, "tools")]

import cnn_gp  # noqa: E402
from cnn_gp.gram import gram_strip, model_kern  # noqa: E402
from fullscale import mnist_like  # noqa: E402


# rounding-level differences (a reduction order that changes between runs) stay far below
# this; a wrong factorisation does not
TOL = 1e-10


def spd(n, dev, seed):
    """A fixed SPD matrix with eigenvalues in [0.02, ~45] (the cifar10 Kxx's range):
    G Gᵀ / k + 0.02 I from a seeded device generator; only its upper triangle is read."""
    g = torch.Generator(device=dev).manual_seed(seed)
    G = torch.rand((n, 64), generator=g, device=dev, dtype=torch.float64)
    return G @ G.T / 64.0 + 0.02 * torch.eye(n, device=dev, dtype=torch.float64)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=16384)
    ap.add_argument("--reps", type=int, default=6)
    ap.add_argument("--no-warm", action="store_true", help="no solver warm-up thread")
    ap.add_argument("--no-kernels", action="store_true", help="no Kxz block before the solve")
    ap.add_argument("--serial", action="store_true",
                    help="the ranks factor one at a time (barriers between turns)")
    ap.add_argument("--solvers", type=int, default=0,
                    help="only ranks below this factor (0: every rank); the others build "
                         "Kxz blocks while they do")
    args = ap.parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    if world > 1:
        dist.init_process_group("gloo", timeout=datetime.timedelta(seconds=300))
    cfg = importlib.import_module("configs.cifar10")
    kern = model_kern(cfg.initial_model.to(dev, torch.float64))
    Z = mnist_like(1024, 3, 32, 1).to(dev, torch.float64)
    X = mnist_like(4096, 3, 32, 0).to(dev, torch.float64)
    A = spd(args.n, dev, 7)
    Y = torch.ones((args.n, 10), dtype=torch.float64, device=dev)
    Ah = A.cpu()                             # the residual on the host: ‖A·α − Y‖ / ‖Y‖
    first, bad, exact = None, 0, 0
    for rep in range(args.reps):
        if world > 1:
            dist.barrier()
        t = time.perf_counter()
        warming = None if args.no_warm else cnn_gp.warm_up_solver(dev)
        if not args.no_kernels:
            with torch.no_grad():
                gram_strip(kern, Z, X, 4096, (0, len(Z)), device=dev, dtype=torch.float64)
        torch.cuda.synchronize()
        if warming is not None:
            warming.join()
        K = A.clone()
        msg = f"rank {rank} rep {rep}:"
        if args.solvers and rank >= args.solvers:
            # a kernel-only rank: Kxz blocks for about as long as the solvers factor
            with torch.no_grad():
                for _ in range(3):
                    gram_strip(kern, Z, X, 4096, (0, len(Z)), device=dev, dtype=torch.float64)
            torch.cuda.synchronize()
            print(f"{msg} kernels only ({time.perf_counter() - t:.2f} s)", flush=True)
            continue
        for turn in range(world if args.serial else 1):
            if args.serial:
                dist.barrier()
            if args.serial and turn != rank:
                continue
            try:
                alpha = cnn_gp.solve_system(K, Y, overwrite_a=True)
                torch.cuda.synchronize()
                U = torch.triu(K).cpu()
                res = float((Ah @ alpha.cpu() - 1.0).norm() / (args.n * 10) ** 0.5)
                msg += f" residual {res:.1e};"
                bad += bool(not res < 1e-8)
                if first is None:
                    first = (U, alpha.cpu())
                    msg += " factored"
                else:
                    nd = int((U != first[0]).sum())
                    ac = alpha.cpu()
                    na = int((ac != first[1]).sum())
                    # normwise: entries near zero make elementwise ratios meaningless
                    du = float((U - first[0]).norm() / first[0].norm())
                    da = float((ac - first[1]).norm() / first[1].norm())
                    msg += (f" factor entries differing from rep 0: {nd} (normwise {du:.1e}), "
                            f"alpha: {na} (normwise {da:.1e})")
                    bad += bool(du > TOL or da > TOL)
                    exact += bool(nd or na)
            except Exception as e:  # noqa: BLE001
                msg += f" FAILED: {type(e).__name__}: {e}"
                bad += 1
        print(f"{msg} ({time.perf_counter() - t:.2f} s)", flush=True)
    if world > 1:
        t = torch.tensor([bad])
        dist.all_reduce(t)
        bad = int(t)
        dist.destroy_process_group()
    if rank == 0:
        print(f"solve_stress: {'FAIL' if bad else 'ok'} ({bad} repetitions beyond {TOL:g}; "
              f"rank 0: {exact} not bit-equal to its first)", flush=True)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
