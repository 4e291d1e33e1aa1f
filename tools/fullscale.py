"""Full-scale ResNet-GP run (BASELINE.json configs[3]): Kxx of N training images, Kxz of
M test images against them, then the GP solve and prediction — the whole of
exp_mnist_resnet/run.bash (save_kernel.py → merge_h5_files.py → classify_gp.py) on the
device, in memory.

    python tools/fullscale.py [--n 60000 --m 10000 --tile 4096 --config mnist_as_tf]
    torchrun --nproc-per-node 8 tools/fullscale.py ...   # row strips, gathered to rank 0

bench.py runs the same function as its full-scale leg (on every rank at --gpus N).

Data: synthetic MNIST-like images (values k/255, ~60% zero pixels, 4-pixel zero border;
no dataset files here) with synthetic labels, so the accuracy line only proves the path
runs.  The pipeline is cnn_gp.pipeline.classify_distributed: Kxx row strips (upper
triangle filled; strictly-lower entries NaN or mirrored — only the upper triangle is
read), received into the full matrix on rank 0, factored in place by rocSOLVER dpotrf_64
(upper triangle, like scipy's posv) while the other ranks build their Kxz rows; α is
broadcast and the [m, 10] scores gathered (Kxz itself only with --pred-var).

Checks printed at the end: potrf info (positive definite), a HIP-vs-HIP spot check of
random Kxx and Kxz entries recomputed one pair at a time through model(x_i, x_j, False,
False) (oracle parity at this geometry: tests/test_gpu_fullgeom.py), and the solve
residual ‖Kxx·α − Y‖ / ‖Y‖ on a random subset of rows.
"""
import argparse
import datetime
import importlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cnn-gp_amd"), ROOT]

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import cnn_gp  # noqa: E402


def mnist_like(n, C, side, seed):
    g = torch.Generator().manual_seed(seed)
    x = torch.floor(torch.rand((n, C, side, side), generator=g, dtype=torch.float64) * 256) / 255
    x[torch.rand(x.shape, generator=g) < 0.6] = 0.0
    x[..., :4, :] = 0.0
    x[..., -4:, :] = 0.0
    x[..., :, :4] = 0.0
    x[..., :, -4:] = 0.0
    return x


# the leading LEAD x LEAD block of Kxx is kept before the in-place factorisation; a failed
# solve reports it against a fresh build of the same images (tools/fullscale.py's only
# source of a "not positive definite" that is not the matrix's own conditioning)
LEAD = int(os.environ.get("CGP_FS_LEAD", "256"))


def lead_report(model, X, lead):
    """What a failed factorisation saw in the leading block: its own Cholesky on the host
    (numpy), and the entries that differ from model(X[:L]) built again now."""
    L = lead.shape[0]
    got = lead.double().cpu().numpy()
    upper = np.triu(got) + np.triu(got, 1).T
    try:
        np.linalg.cholesky(upper)
        host = "host Cholesky of the saved block ok"
    except np.linalg.LinAlgError:
        host = "host Cholesky of the saved block fails"
    with torch.no_grad():
        ref = model(X[:L]).double().cpu().numpy()
    iu = np.triu_indices(L)
    rel = np.abs(got[iu] - ref[iu]) / np.abs(ref[iu])
    bad = np.flatnonzero(~(rel <= 1e-12))
    first = [(int(iu[0][k]), int(iu[1][k]), float(got[iu][k]), float(ref[iu][k]))
             for k in bad[:4]]
    return (f"{host}; leading {L}x{L} upper block vs a fresh build: {len(bad)} entries "
            f"differ (max rel {np.nanmax(rel) if len(rel) else 0:.3e}), first {first}")


def log(rank, msg):
    if rank == 0:
        print(msg, flush=True)


def widen(t):
    """float32 device matrix -> float64 (classify_gp.py:45-48's load_kern widening, on the
    device through cgp_cast_f32_f64); Kxx itself is widened in place by the pipeline."""
    return cnn_gp.cast_into(t.contiguous(), torch.empty(t.shape, dtype=torch.float64,
                                                         device=t.device))


def fullscale(config="mnist_as_tf", n=60000, m=10000, tile=4096, jitter=0.0, spot=16,
              pred_var=False, rank=0, world=1, dev=None, group=None,
              kernel_dtype=torch.float64, stats_group=None):
    """Kxx (n) + rocSOLVER solve + Kxz (m × n) + predict on the device, through
    cnn_gp.pipeline.classify_distributed: with world > 1 every rank builds a row strip of
    Kxx (balanced by evaluated pairs), rank 0 receives the strips into the full matrix and
    solves while the other ranks build their Kxz rows, then α is broadcast and only the
    [m, 10] scores come back.  Returns the result dict on rank 0, None elsewhere.

    kernel_dtype float32 runs the kernels the way the reference's own pipeline does
    (save_kernel.py:19-24: the float32 model on float32 images, K stored float32 by
    kernel_save_tools.py:21) and widens K to float64 for the solve (classify_gp.py:45-48);
    the spot check then also reports the float32 entries against the float64 model.
    With world > 1 the result carries every rank's own phase times (``ranks``), gathered
    over ``stats_group`` (e.g. a gloo side group; default the pipeline's group)."""
    from cnn_gp.gram import model_kern
    from cnn_gp.pipeline import classify_distributed
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
    Y = cnn_gp.one_hot_pm1(ytr, 10)
    kd = kernel_dtype
    res = {"config": config, "n": n, "m": m, "tile": tile, "gpus": world,
           "kernel_dtype": str(kd).replace("torch.", "")}
    gs = torch.Generator().manual_seed(3)
    rows = torch.randint(0, n, (8,), generator=gs)
    saved = {}

    def residual_rows(K):
        # the residual rows of K before it is factored in place (K is symmetric, its
        # upper triangle is filled); harness work, outside solve_s (pipeline pre_solve)
        t = time.perf_counter()
        r = rows.to(K.device)
        saved["Krows"] = torch.where(torch.arange(n, device=K.device)[None, :] >= r[:, None],
                                     K[r], K[:, r].T).to(torch.float64)
        if LEAD > 0:                 # for the diagnosis of a failed factorisation
            saved["lead"] = K[:LEAD, :LEAD].clone()
        torch.cuda.synchronize(K.device)
        saved["rows_s"] = time.perf_counter() - t

    def solve(K, Yd):
        try:
            # jitter and the solution check: the pipeline's (classify_distributed)
            A = cnn_gp.solve_system(K, Yd, overwrite_a=True, check=False)
        except np.linalg.LinAlgError as e:
            if "lead" not in saved:
                raise
            raise np.linalg.LinAlgError(f"{e}; {lead_report(model, X, saved['lead'])}") from e
        saved["phases"] = cnn_gp.solve_phases(K.device)
        return A

    torch.cuda.reset_peak_memory_stats(dev)
    times = {}
    t0 = time.perf_counter()
    with torch.no_grad():
        out = classify_distributed(model_kern(model), X, Z, Y, solve, cnn_gp.scores,
                                   batch_size=tile, group=group, device=dev, dtype=kd,
                                   gather_kxz=pred_var,
                                   widen=widen if kd != torch.float64 else None,
                                   log=lambda msg: log(rank, msg),
                                   warm=lambda: cnn_gp.warm_up_solver(dev),
                                   cast=cnn_gp.cast_into, rank_times=times,
                                   pre_solve=residual_rows, jitter=jitter)
    wall = time.perf_counter() - t0
    ranks = [times]
    if world > 1:
        ranks = [None] * world
        dist.all_gather_object(ranks, times, group=stats_group or group)
    if rank != 0:
        return None
    kxx_bytes = n * n * 8
    res.update({k: out[k] for k in ("kxx_s", "gather_kxx_s", "kxx_to_kxz_s", "predict_s",
                                    "total_s")})
    ph = saved.get("phases")
    res.update(solve_s=out["solve_s"], kxz_s_rank0=out["kxz_s_rank"],
               alpha_backward_error=out.get("alpha_backward_error"),
               co_resident_ranks=out.get("co_resident_ranks"),
               solve_tflops=round(n ** 3 / 3 / out["solve_s"] / 1e12, 2),
               harness_s=round(saved["rows_s"], 4))
    if ph is not None:              # the solve's own HIP-event phases (solve.solve_phases)
        res["solve_split"] = {"widen_s": out.get("widen_s", 0.0),
                              "jitter_s": round(ph["jitter_s"], 4),
                              "factor_s": round(ph["factor_s"], 4),
                              "potrs_s": round(ph["potrs_s"], 4),
                              "rest_s": round(out["solve_s"] - out.get("widen_s", 0.0) -
                                              sum(ph.values()), 4),
                              "factor_tflops": round(n ** 3 / 3 / ph["factor_s"] / 1e12, 2),
                              "note": "solve_s = widen (float32 K only) + jitter + Cholesky "
                                      "+ dpotrs (HIP events inside the solve) + rest (Y/alpha "
                                      "transposes, host); harness_s = the 8 residual rows "
                                      "copied before K is factored in place (outside "
                                      "solve_s, inside total_s)"}
    res.update(kxx_pairs_per_s=round(n * (n - 1) / 2 / out["kxx_s"], 1),
               plan_kxx=out["plan_kxx"], plan_kxz=out["plan_kxz"],
               kxz_share=out["kxz_share"],
               rank0_peak_gb_kxx_build=round(out["peak_bytes_kxx_build"] / 1e9, 2),
               rank0_peak_gb_gather_solve=round(out["peak_bytes_gather_solve"] / 1e9, 2),
               rank0_peak_gb_kxz=round(out["peak_bytes_kxz"] / 1e9, 2),
               rank0_peak_gather_solve_over_kxx=round(out["peak_bytes_gather_solve"] /
                                                      kxx_bytes, 3))
    if world == 1:
        res["kxz_s"] = out["kxz_s_rank"]
    else:
        res["ranks"] = ranks
    K, A = out["K"], out["alpha"]
    # residual on 8 rows of the (jittered) system: ‖K·α − Y‖ / ‖Y‖
    Kr = saved["Krows"].double()
    Yd = Y.to(dev)
    Kr[torch.arange(len(rows), device=dev), rows.to(dev)] += jitter
    res["residual"] = float((Kr @ A - Yd[rows.to(dev)]).norm() / Yd[rows.to(dev)].norm())
    res["synthetic_accuracy"] = cnn_gp.accuracy(out["pred"], yte)
    # spot check (HIP against HIP): single pairs through the same drop-in call — other tile
    # shapes, no chunking; a self-consistency check.  Parity with the CPU oracle at this
    # tile geometry is tests/test_gpu_fullgeom.py.  K is factored now: Kxx entries are
    # checked through the saved rows, Kxz entries through rank 0's own Kxz rows.
    z0, z1 = out["kxz_rows"]
    worst = 0.0
    with torch.no_grad():
        for k, a in enumerate(rows.tolist()):
            for b in torch.randint(0, n, (max(1, spot // 8),), generator=gs).tolist():
                # the upper triangle holds pair (min, max): the kernel's own orientation
                lo, hi = min(a, b), max(a, b)
                ref = model(X[a:a + 1]).item() if a == b else \
                    model(X[lo:lo + 1], X[hi:hi + 1], False, False).item()
                worst = max(worst, abs(saved["Krows"][k, b].item() - ref) / abs(ref))
        if z1 > z0:
            Kz = out["Kxz_rows"]
            for c, b in zip(torch.randint(z0, z1, (spot,), generator=gs).tolist(),
                            torch.randint(0, n, (spot,), generator=gs).tolist()):
                ref = model(Z[c:c + 1], X[b:b + 1], False, False).item()
                worst = max(worst, abs(Kz[c - z0, b].item() - ref) / abs(ref))
    res["spot_check_hip_vs_hip_max_rel_err"] = worst
    if kd != torch.float64:
        # the float32 entries against the float64 model on the same (exactly widened)
        # images: the north star's 1e-5 relative tolerance
        m64 = cfg.initial_model.to(dev, torch.float64)
        dev64 = 0.0
        with torch.no_grad():
            for k, a in enumerate(rows.tolist()):
                for b in (0, n // 2, n - 1):
                    xa, xb = X[a:a + 1].double(), X[b:b + 1].double()
                    ref = m64(xa).item() if a == b else m64(xa, xb, False, False).item()
                    dev64 = max(dev64, abs(saved["Krows"][k, b].item() - ref) / abs(ref))
        res["spot_vs_f64_max_rel_err"] = dev64
    if pred_var:
        with torch.no_grad():
            t7 = time.perf_counter()
            kz = model(Z, Z, True, True).double()    # Kt_diag, save_kernel.py:33-36
            torch.cuda.synchronize()
            t8 = time.perf_counter()
            Kxz = out["Kxz"] if out["Kxz"].dtype == torch.float64 else widen(out["Kxz"])
            var = cnn_gp.predictive_variance(K, Kxz, kz, overwrite_kxz=True)
            torch.cuda.synchronize()
            t9 = time.perf_counter()
        res.update(kz_diag_s=round(t8 - t7, 3), pred_var_s=round(t9 - t8, 3),
                   pred_var_tflops=round(n ** 2 * m / (t9 - t8) / 1e12, 2),
                   pred_var_min=float(var.min()),
                   pred_var_max_over_prior=float((var / kz).max()))
    res["wall_s"] = round(wall, 2)
    del K, out
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
        tmo = datetime.timedelta(seconds=float(os.environ.get("CGP_DIST_TIMEOUT_S", "300")))
        os.environ.setdefault("TORCH_NCCL_BLOCKING_WAIT", "1")
        dist.init_process_group("nccl", device_id=dev, timeout=tmo)
    res = fullscale(args.config, args.n, args.m, args.tile, args.jitter, args.spot,
                    args.pred_var, rank, world, dev,
                    kernel_dtype=torch.float64 if args.dtype == "f64" else torch.float32)
    if rank == 0:
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
