"""Full-scale ResNet-GP run (BASELINE.json configs[3]): Kxx of N training images, Kxz of
M test images against them, then the GP solve and prediction — the whole of
exp_mnist_resnet/run.bash (save_kernel.py → merge_h5_files.py → classify_gp.py) on the
device, in memory.

    python tools/fullscale.py [--n 60000 --m 10000 --tile 4096 --config mnist_as_tf]
    torchrun --nproc-per-node 8 tools/fullscale.py ...   # tiles split, one gather to rank 0

bench.py runs the same function as its full-scale leg (on every rank at --gpus N).

Data: synthetic MNIST-like images (values k/255, ~60% zero pixels, 4-pixel zero border;
no dataset files here) with synthetic labels, so the accuracy line only proves the path
runs.  Kxx keeps the reference's layout (upper tiles, NaN strictly-lower tiles) and is
factored in place by rocSOLVER dpotrf_64 (upper triangle, like scipy's posv).

Checks printed at the end: potrf info (positive definite), a spot check of random Kxx
and Kxz entries recomputed one pair at a time through model(x_i, x_j, False, False), and
the solve residual ‖Kxx·α − Y‖ / ‖Y‖ on a random subset of rows.
"""
import argparse
import importlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cnn-gp_amd"), ROOT]

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import cnn_gp  # noqa: E402
from cnn_gp.gram import gather_gram, tile_cost, tile_plan  # noqa: E402


def mnist_like(n, C, side, seed):
    g = torch.Generator().manual_seed(seed)
    x = torch.floor(torch.rand((n, C, side, side), generator=g, dtype=torch.float64) * 256) / 255
    x[torch.rand(x.shape, generator=g) < 0.6] = 0.0
    x[..., :4, :] = 0.0
    x[..., -4:, :] = 0.0
    x[..., :, :4] = 0.0
    x[..., :, -4:] = 0.0
    return x


def log(rank, msg):
    if rank == 0:
        print(msg, flush=True)


def build(model, X, X2, B, rank, world, name, t_start, dev, out=None, dtype=torch.float64):
    """This rank's tiles of Kxx (X2 None) or Kxz.  One rank: written straight into the
    NaN-filled device matrix ``out``.  Several ranks: packed into one flat device buffer
    (gram.gram_local's layout, split by evaluated pairs) for gather_gram.  Returns
    (out or buffer, pairs evaluated)."""
    n = len(X)
    n2 = None if X2 is None else len(X2)
    split = "reference" if world == 1 else "balanced"
    tiles = tile_plan(n, n2, B, rank, world, split)
    if world > 1:
        cap = max(sum(a * b for *_, a, b in tile_plan(n, n2, B, r, world, split))
                  for r in range(world))
        out = torch.empty(max(cap, 1), dtype=dtype, device=dev)
    pairs = 0
    off = 0
    last = time.perf_counter()
    with torch.no_grad():
        for k, (same, i0, j0, a, b) in enumerate(tiles):
            x = X[i0:i0 + a]
            if same:
                t = model(x)
            else:
                src = X if X2 is None else X2
                t = model(x, src[j0:j0 + b], False, False)
            if world > 1:
                out[off:off + a * b].view(a, b).copy_(t)
                off += a * b
            else:
                out[i0:i0 + a, j0:j0 + b].copy_(t)
            pairs += tile_cost((same, i0, j0, a, b))
            now = time.perf_counter()
            if now - last > 20:
                torch.cuda.synchronize()
                log(rank, f"  {name}: tile {k + 1}/{len(tiles)} "
                          f"({time.perf_counter() - t_start:.0f} s)")
                last = now
    return out, pairs


def widen(t):
    """float32 device matrix -> float64 (classify_gp.py:45-48's load_kern widening, on the
    device through cgp_cast_f32_f64); the float32 source is released."""
    out = torch.empty(t.shape, dtype=torch.float64, device=t.device)
    from cnn_gp import _native as N
    N.call("cgp_cast_f32_f64", N.ptr(t), N.ptr(out), t.numel(),
           torch.cuda.current_stream(t.device).cuda_stream)
    return out


def fullscale(config="mnist_as_tf", n=60000, m=10000, tile=4096, jitter=0.0, spot=16,
              pred_var=False, rank=0, world=1, dev=None, group=None,
              kernel_dtype=torch.float64):
    """Kxx (n) + Kxz (m × n) + rocSOLVER solve + predict on the device; with world > 1
    the tiles are split over the ranks and gathered once to rank 0 (one RCCL gather per
    matrix), which solves.  Returns the result dict on rank 0, None elsewhere.

    kernel_dtype float32 runs the kernels the way the reference's own pipeline does
    (save_kernel.py:19-24: the float32 model on float32 images, K stored float32 by
    kernel_save_tools.py:21) and widens K to float64 for the solve (classify_gp.py:45-48);
    the spot check then also reports the float32 entries against the float64 model."""
    dev = dev or torch.device("cuda", torch.cuda.current_device())
    cfg = importlib.import_module(f"configs.{config}")
    model = cfg.initial_model.to(dev, kernel_dtype)
    C = getattr(cfg, "in_channels", 1)
    side = 32 if C == 3 else 28
    X = mnist_like(n, C, side, 0).to(dev, kernel_dtype)
    Z = mnist_like(m, C, side, 1).to(dev, kernel_dtype)
    g = torch.Generator().manual_seed(2)
    ytr = torch.randint(0, 10, (n,), generator=g)
    yte = torch.randint(0, 10, (m,), generator=g)
    B = tile
    res = {"config": config, "n": n, "m": m, "tile": B, "gpus": world,
           "kernel_dtype": str(kernel_dtype).replace("torch.", "")}
    kd = kernel_dtype

    if world > 1:
        dist.barrier(group)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    K = None if world > 1 else torch.full((n, n), float("nan"), dtype=kd, device=dev)
    K, p_xx = build(model, X, None, B, rank, world, "Kxx", t0, dev, K, kd)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    Kxz = None if world > 1 else torch.full((m, n), float("nan"), dtype=kd, device=dev)
    Kxz, p_xz = build(model, Z, X, B, rank, world, "Kxz", t0, dev, Kxz, kd)
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    if world > 1:
        # the slowest rank sets the build time; then ONE gather per matrix
        dist.barrier(group)
        t2 = time.perf_counter()
        K = gather_gram(K, n, None, B, group)
        Kxz = gather_gram(Kxz, m, n, B, group)
        torch.cuda.synchronize()
    t3 = time.perf_counter()
    res.update(kxx_s=round(t1 - t0, 2), kxz_s=round(t2 - t1, 2), gather_s=round(t3 - t2, 3),
               kxx_pairs_per_s_rank0=round(p_xx / (t1 - t0), 1),
               kxz_pairs_per_s_rank0=round(p_xz / max(t2 - t1, 1e-9), 1))
    log(rank, f"kernels built in {t3 - t0:.1f} s")
    if rank != 0:
        if world > 1:
            dist.barrier(group)
        return None
    # spot check: single pairs through the same drop-in call, other tile shapes
    gs = torch.Generator().manual_seed(3)
    ii = torch.randint(0, n, (spot,), generator=gs)
    jj = torch.randint(0, n, (spot,), generator=gs)
    kk = torch.randint(0, m, (spot,), generator=gs)
    worst = 0.0
    with torch.no_grad():
        for a, b, c in zip(ii.tolist(), jj.tolist(), kk.tolist()):
            a, b = min(a, b), max(a, b)
            ref = model(X[a:a + 1], X[b:b + 1], False, False).item() if a != b else \
                model(X[a:a + 1]).item()
            worst = max(worst, abs(K[a, b].item() - ref) / abs(ref))
            ref = model(Z[c:c + 1], X[b:b + 1], False, False).item()
            worst = max(worst, abs(Kxz[c, b].item() - ref) / abs(ref))
    # HIP against HIP: the same drop-in call on single pairs (other tile shapes, no
    # chunking) — a self-consistency check; parity with the CPU oracle at this tile
    # geometry is tests/test_gpu_fullgeom.py
    res["spot_check_hip_vs_hip_max_rel_err"] = worst
    if kd != torch.float64:
        # the float32 entries against the float64 model on the same (exactly widened)
        # images: the north star's 1e-5 relative tolerance
        m64 = cfg.initial_model.to(dev, torch.float64)
        dev64 = 0.0
        with torch.no_grad():
            for a, b, c in zip(ii.tolist(), jj.tolist(), kk.tolist()):
                a, b = min(a, b), max(a, b)
                xa, xb = X[a:a + 1].double(), X[b:b + 1].double()
                ref = m64(xa, xb, False, False).item() if a != b else m64(xa).item()
                dev64 = max(dev64, abs(K[a, b].item() - ref) / abs(ref))
                ref = m64(Z[c:c + 1].double(), xb, False, False).item()
                dev64 = max(dev64, abs(Kxz[c, b].item() - ref) / abs(ref))
        res["spot_vs_f64_max_rel_err"] = dev64
        torch.cuda.synchronize()
        tw = time.perf_counter()
        K = widen(K)                    # the solve runs in float64 (classify_gp.py:19-22)
        Kxz = widen(Kxz)
        torch.cuda.synchronize()
        res["widen_s"] = round(time.perf_counter() - tw, 3)
    # residual rows: K is symmetric, its upper triangle is filled
    rows = torch.randint(0, n, (8,), generator=gs).to(dev)
    Krows = torch.where(torch.arange(n, device=dev)[None, :] >= rows[:, None],
                        K[rows], K[:, rows].T)
    Y = cnn_gp.one_hot_pm1(ytr, 10).to(dev)
    torch.cuda.synchronize()
    t4 = time.perf_counter()
    A = cnn_gp.solve_system(K, Y, jitter=jitter, overwrite_a=True)   # K -> factor
    torch.cuda.synchronize()
    t5 = time.perf_counter()
    diag_j = torch.arange(len(rows), device=dev)
    Krows[diag_j, rows] += jitter
    r = (Krows @ A - Y[rows]).norm() / Y[rows].norm()
    pred = cnn_gp.predict(A, Kxz)
    torch.cuda.synchronize()
    t6 = time.perf_counter()
    acc = cnn_gp.accuracy(pred, yte)
    res.update(solve_s=round(t5 - t4, 2),
               solve_tflops=round(n ** 3 / 3 / (t5 - t4) / 1e12, 2),
               predict_s=round(t6 - t5, 3), residual=float(r),
               synthetic_accuracy=acc, total_s=round(t6 - t0, 2))
    if pred_var:
        with torch.no_grad():
            t7 = time.perf_counter()
            kz = model(Z, Z, True, True).double()    # Kt_diag, save_kernel.py:33-36
            torch.cuda.synchronize()
            t8 = time.perf_counter()
            var = cnn_gp.predictive_variance(K, Kxz, kz, overwrite_kxz=True)
            torch.cuda.synchronize()
            t9 = time.perf_counter()
        res.update(kz_diag_s=round(t8 - t7, 3), pred_var_s=round(t9 - t8, 3),
                   pred_var_tflops=round(n ** 2 * m / (t9 - t8) / 1e12, 2),
                   pred_var_min=float(var.min()),
                   pred_var_max_over_prior=float((var / kz).max()))
    del K, Kxz
    if world > 1:
        dist.barrier(group)
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="mnist_as_tf")
    ap.add_argument("--n", type=int, default=60000)
    ap.add_argument("--m", type=int, default=10000)
    ap.add_argument("--tile", type=int, default=4096)
    ap.add_argument("--jitter", type=float, default=0.0)
    ap.add_argument("--spot", type=int, default=16)
    ap.add_argument("--dtype", default="f64", choices=["f64", "f32"],
                    help="kernel precision (f32: the reference pipeline's; K widened to "
                         "f64 for the solve)")
    ap.add_argument("--pred-var", action="store_true",
                    help="also the posterior variance of the test points (prior diag "
                         "+ dtrsm on the factor), reported outside total_s")
    args = ap.parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
    res = fullscale(args.config, args.n, args.m, args.tile, args.jitter, args.spot,
                    args.pred_var, rank, world, dev,
                    kernel_dtype=torch.float64 if args.dtype == "f64" else torch.float32)
    if rank == 0:
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
