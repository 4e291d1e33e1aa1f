"""Benchmark: NNGP Gram-matrix build (kernel entries/s) + GP solve on MI355X.

Workload (BASELINE.json configs[1]): mnist_paper_convnet_gp, Kxx of N = 4096 synthetic
28×28×1 images, float64, Gram tiles of B = 1024 in the reference's schedule (upper
triangular tiles).  One STEP = one Gram build: every image's variance maps computed
once (cnn_gp.gram.ModelKern.bind; the reference recomputes them per tile and side), then
every Gram tile of this rank evaluated in place into a device-resident Kxx.

    python bench.py [--gpus N --steps K --warmup W] [--config C --n N --tile B]

value = kernel entries the device EVALUATES per second, whole job: B1·B2 for an
off-diagonal tile, B(B−1)/2 for a diagonal tile (the kernel computes i < j there and
mirrors; K[i, i] comes from the per-image variance chain).  The reference's schedule
would count B² for a diagonal tile; that figure is reported as
``reference_schedule_pairs_per_s`` beside it.

Also on the same JSON line:
  roofline           the whole-network kernel (net_kernel, fp64 VALU-bound): credited
                     direct-stencil flops vs the fp64 peak, plus the VALU issue
                     utilisation and HBM traffic per launch from the committed PMC
                     passes (profiles/r3/net_pmc.json, rocprofv3)
  mnist_as_tf        the same harness on BASELINE configs[2] (ResNet-GP, 32 layers)
  solve              rocSOLVER dpotrf_64 + dpotrs_64 on the assembled 4096² Kxx
  fullscale          BASELINE configs[3]: mnist_as_tf Kxx 60 000² + Kxz 10 000 × 60 000
                     + solve + predict, row strips per rank, Kxx received into rank 0's
                     matrix point-to-point, solve overlapped with the Kxz strips, only
                     the scores gathered (tools/fullscale.py, cnn_gp/pipeline.py)
  fullscale_cifar10  BASELINE configs[4]: cifar10 Kxx 50 000² + Kxz + solve + predict
  conv_stencil_roofline  Conv2d.propagate alone (the north star's "Conv2d covariance
                     kernel") against the 8 TB/s HBM roof, PMC traffic committed
  cpu_baseline       the torch-CPU restatement of the reference (oracle/torch_cpu.py,
                     bit-identical to the reference at C1) on the host threads torch
                     is given, with the committed calibration against the reference

Multi-GPU (one process per GPU, torchrun): the Kxx grows with the world
(n_blocks² half-tile units >= world × the 1-GPU units, divisible by world) and its tiles
are split over the ranks by evaluated pairs — no data-path collective; per-rank work is
~constant ("scaling": "weak").  The full-scale legs shard their fixed problems
("strong"): Kxx strips to rank 0 point-to-point, α broadcast, scores gathered.
"""
from __future__ import annotations

import argparse
import importlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(ROOT, "cnn-gp_amd"), ROOT, os.path.join(ROOT, "tools")]

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import cnn_gp  # noqa: E402
from cnn_gp import _native as N  # noqa: E402
from cnn_gp.data import tile_schedule  # noqa: E402
from cnn_gp.gram import model_kern  # noqa: E402

HBM_PEAK_GBS = 8000.0          # MI355X spec (MI355X_MICROARCH.md): 8 TB/s
FP64_PEAK_TFLOPS = 78.6        # MI355X spec FP64 (vector = matrix); half the FP32 157.3
SIMDS = 256 * 4                # 256 CUs × 4 SIMDs
CLOCK_HZ = 2.4e9               # peak engine clock
PMC_FILE = os.path.join(ROOT, "profiles", "r3", "net_pmc.json")
CALIB_FILE = os.path.join(ROOT, "profiles", "r2", "cpu_calibration.json")
PIPELINE_NOTE = (
    "cnn_gp.pipeline.classify_distributed: Kxx row strips (B=4096 tiles) balanced by "
    "evaluated pairs, received point-to-point into the full matrix on rank 0 (RCCL with "
    "nccl); rank 0 factors it (blocked dpotrf/dtrsm/dsyrk, nb 2048) while the other ranks "
    "build their Kxz row strips (rank 0's share sized to end with them); alpha broadcast, "
    "scores = Kxz rows @ alpha per rank, only the scores gathered; solver code objects "
    "loaded on a side thread during the Kxx build; spot check = HIP vs HIP single pairs "
    "(oracle parity at this geometry: tests/test_gpu_fullgeom.py)")


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=3)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--config", default="mnist_paper_convnet_gp")
    p.add_argument("--n", type=int, default=4096, help="Kxx size at world size 1")
    p.add_argument("--tile", type=int, default=1024)
    p.add_argument("--dtype", default="f64", choices=["f64", "f32"])
    p.add_argument("--no-solve", action="store_true")
    p.add_argument("--no-cpu", action="store_true")
    p.add_argument("--no-probe", action="store_true")
    p.add_argument("--no-second", action="store_true", help="skip the mnist_as_tf leg")
    p.add_argument("--no-f32", action="store_true",
                   help="skip the float32 repeat of the Kxx legs")
    p.add_argument("--no-fullscale", action="store_true")
    p.add_argument("--no-fullscale-f32", action="store_true",
                   help="skip the float32-kernel repeat of the full-scale leg")
    p.add_argument("--no-fullscale-cifar10", action="store_true",
                   help="skip BASELINE configs[4]: cifar10 Kxx 50 000² + Kxz + solve")
    p.add_argument("--fullscale-n", type=int, default=60000)
    p.add_argument("--cifar10-n", type=int, default=50000)
    p.add_argument("--fullscale-m", type=int, default=10000)
    p.add_argument("--cpu-seconds", type=float, default=15.0,
                   help="target duration of the CPU-baseline sample")
    return p.parse_args()


def blocks_for_world(n1: int, tile: int, world: int) -> int:
    """Smallest n_blocks whose evaluated work covers world × the 1-GPU work and splits
    evenly.  Work is counted in half-tile units (a diagonal tile evaluates half the pairs
    of an off-diagonal one): nb blocks hold nb(nb−1) + nb = nb² units, so nb² must reach
    world · b1² and divide by the world size.  At B = 1024 that is 4 / 6 / 8 / 12 blocks
    at N = 1 / 2 / 4 / 8, i.e. 16 / 18 / 16 / 18 units per rank (an earlier rule counted tiles
    instead of units, which gave 16 / 18 / 25 / 32: per-rank work grew with N)."""
    b1 = -(-n1 // tile)
    target = b1 * b1 * world
    nb = b1
    while nb * nb < target or (world > 1 and (nb * nb) % world):
        nb += 1
    return nb


def tile_eval_pairs(t, B, n):
    """pairs the device evaluates for tile (same, bi, bj): i < j on a diagonal tile"""
    same, i, j = t
    a, b = min(B, n - i * B), min(B, n - j * B)
    return a * (a - 1) // 2 if same else a * b


def balanced_split(all_tiles, B, n, world):
    """Per-rank tile lists with equal evaluated pairs: longest-processing-time greedy on
    the pairs each tile evaluates (a diagonal tile costs half), in the reference's tile
    order within a rank."""
    load = [0] * world
    parts = [[] for _ in range(world)]
    for k in sorted(range(len(all_tiles)), key=lambda k: -tile_eval_pairs(all_tiles[k], B, n)):
        r = min(range(world), key=lambda r: load[r])
        load[r] += tile_eval_pairs(all_tiles[k], B, n)
        parts[r].append(k)
    return [[all_tiles[k] for k in sorted(p)] for p in parts]


def timed_events(stream, launch, reps):
    launch()
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(reps):
        launch()
    e1.record(stream)
    e1.synchronize()
    return e0.elapsed_time(e1) / reps


def load_json(path):
    try:
        with open(path) as f:
            return json.load(f)
    except (OSError, ValueError):
        return None


def conv_stencil_roofline(model, x, B, reps=5):
    """Conv2d.propagate alone (kernels.py:92-98; no fused ReLU / moments / Sum) — the
    north star's "Conv2d covariance kernel" — at the config's most frequent conv shape, on
    the B·B pair maps of one tile, timed with HIP events on the launch stream; against the
    8 TB/s HBM roof with algorithmic bytes 8·P·(H·W + Ho·Wo).  A torch copy of the same
    input is timed beside it as the achievable-bandwidth reference.  ``traffic``: the
    committed PMC pass over the same launch (profiles/r3/net_pmc.json "conv_stencil")."""
    from collections import Counter
    _, C, h, w = x.shape
    plan = model._plan(h, w)
    convs = Counter((op.geom.taps, op.geom.offset, op.geom.stride, op.shape_in, op.shape_out)
                    for op in plan.prog.ops
                    if op.kind == "conv" and op.geom.dilation == 1 and op.shape_out[0] > 1)
    if not convs:
        return None
    (k, off, st, (hi, wi), (ho, wo)), _ = convs.most_common(1)[0]
    P = B * B
    g = torch.Generator(device="cpu").manual_seed(0)
    var = torch.rand((2 * B, hi, wi), generator=g, dtype=x.dtype).add_(0.5).to(x.device)
    xy = (0.5 * (var[:B, None] * var[None, B:]).sqrt()).reshape(P, hi, wi).contiguous()
    del var
    out = torch.empty((P, ho, wo), dtype=x.dtype, device=x.device)
    stream = torch.cuda.current_stream()
    s = stream.cuda_stream
    a = N.ConvArgs()
    a.in_, a.out = N.ptr(xy), N.ptr(out)
    a.nmaps, a.n1, a.n2 = P, B, B
    a.h, a.w, a.ho, a.wo = hi, wi, ho, wo
    a.taps, a.offset, a.stride, a.dilation = k, off, st, 1
    a.weight, a.bias = 1.0 / (k * k), 0.1
    fn = getattr(N.load(), "cgp_conv_" + ("f64" if x.dtype == torch.float64 else "f32"))
    ms = timed_events(stream, lambda: N.check(fn(a, s), "cgp_conv"), reps)
    cp = torch.empty_like(xy)
    ms_copy = timed_events(stream, lambda: cp.copy_(xy), reps)
    item = x.element_size()
    nbytes = P * (hi * wi + ho * wo) * item
    ach = nbytes / (ms * 1e-3) / 1e9
    copy_gbs = 2 * P * hi * wi * item / (ms_copy * 1e-3) / 1e9
    del xy, out, cp
    torch.cuda.empty_cache()
    kname = f"conv{k}s{st}@{hi}->{ho}"
    traffic, pmc_ms = None, None
    pmc = (load_json(PMC_FILE) or {}).get("conv_stencil")
    if pmc and pmc.get("kernel") == kname and pmc.get("maps") == P:
        traffic, pmc_ms = int(pmc["hbm_bytes_per_launch"]), pmc.get("avg_ms")
    return {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": traffic,
            "kernel": kname, "avg_ms": round(ms, 4), "pmc_avg_ms": pmc_ms,
            "alg_bytes_per_launch": int(nbytes), "maps_per_launch": P,
            "torch_copy_GBs": round(copy_gbs, 1),
            "note": "Conv2d.propagate alone on one tile's pair maps (cgp_conv, no fused "
                    "epilogue); traffic = 2·FETCH_SIZE + WRITE_SIZE (gfx950 correction) "
                    "from the committed rocprofv3 pass"}


def alg_flops_per_pair(plan):
    """The reference's direct-stencil conv flops per pair: F.conv2d does
    2·extent² flops per output pixel (extent = k, or k + 1 for an even "same" kernel).
    The ReLU arc-cosine arithmetic — the fused kernel's main VALU cost — is not counted."""
    f = 0
    for op in plan.prog.ops:
        if op.kind == "conv":
            e = op.geom.extent or op.geom.taps
            f += 2 * e * e * op.shape_out[0] * op.shape_out[1]
    return f


def alg_flops_pointwise_per_pair(plan):
    """The reference's elementwise work per pair on top of the conv stencils: the bias
    add after every F.conv2d (kernels.py:98), the ReLU map's 14 pointwise ops per pixel
    (kernels.py:146-152: mul, add, rsqrt, mul, clamp, mul, sub, clamp, sqrt, acos, sub,
    mul, add, div; a transcendental counted as one) and one add per Sum/Mixture term."""
    f = 0
    for op in plan.prog.ops:
        hw = op.shape_out[0] * op.shape_out[1]
        if op.kind == "conv":
            f += hw
        elif op.kind == "relu":
            f += 14 * hw
        elif op.kind == "add":
            f += (len(op.terms) - 1) * hw
    return f


def net_roofline(model, x, cfg_name, timing):
    """Roofline of the whole-network kernel from the HIP events recorded around each of its
    launches in the timed region (cnn_gp.netplan.TIMING, on the launch stream).

    The kernel is fp64-VALU bound ("valu_f64"): per pair it reads two images and L2-resident
    variance maps and writes one entry, everything else stays in LDS.  ``achieved`` credits
    the reference's direct-stencil conv flops (the kernel executes fewer: separable window
    sums), so ``frac`` is a credited figure; ``valu_issue_frac`` is the hardware meter —
    the fraction of SIMD cycles issuing a VALU instruction (SQ_ACTIVE_INST_VALU, in
    quad-cycles, × 4 / (1024 SIMDs × clock × kernel time)), from the committed PMC pass
    scaled per pair to this run's launches."""
    n, C, h, w = x.shape
    plan = model._plan(h, w)
    net = model._net_plan(plan, x.element_size())
    if net is None or not timing:
        return None
    ms = sum(e0.elapsed_time(e1) for e0, e1, _ in timing)
    pairs = sum(p for _, _, p in timing)
    fl = alg_flops_per_pair(plan)
    achieved = fl * pairs / (ms * 1e-3) / 1e12
    fl_pw = fl + alg_flops_pointwise_per_pair(plan)
    achieved_pw = fl_pw * pairs / (ms * 1e-3) / 1e12
    per_launch = pairs / len(timing)
    avg_s = ms * 1e-3 / len(timing)
    traffic = valu = valu_insts = None
    pmc_note = "no committed PMC pass for this config/dtype"
    pmc = (load_json(PMC_FILE) or {}).get(cfg_name)
    if pmc and pmc.get("dtype") == str(x.dtype):
        traffic = int(pmc["hbm_bytes_per_pair"] * per_launch)
        quad = pmc["valu_active_quadcycles_per_pair"] * per_launch
        valu = round(4 * quad / (SIMDS * CLOCK_HZ * avg_s), 4)
        valu_insts = round(pmc["valu_insts_per_pair"], 1)
        pmc_note = (f"PMC: {pmc['source']}; per pair: {pmc['hbm_bytes_per_pair']:.0f} HBM "
                    f"bytes, {pmc['valu_insts_per_pair']:.0f} VALU wave-instructions")
    kname = f"net_kernel<{'double' if x.dtype == torch.float64 else 'float'}>"
    return {"bound": "valu_f64", "achieved": round(achieved, 2), "peak": FP64_PEAK_TFLOPS,
            "unit": "TFLOP/s", "frac": round(achieved / FP64_PEAK_TFLOPS, 4),
            "traffic": traffic, "valu_issue_frac": valu,
            "kernel": kname, "launches": len(timing), "avg_ms": round(ms / len(timing), 4),
            "pairs_per_launch": int(per_launch), "alg_flops_per_pair": fl,
            "alg_flops_per_launch": int(fl * per_launch),
            "alg_flops_incl_pointwise_per_pair": fl_pw,
            "achieved_incl_pointwise": round(achieved_pw, 2),
            "frac_incl_pointwise": round(achieved_pw / FP64_PEAK_TFLOPS, 4),
            "valu_insts_per_pair": valu_insts,
            "ops_per_pair": net.n_ops, "lds_bytes": net.lds_elems * x.element_size(),
            "stages": [{"pairs_per_workgroup": st.pairs, "ops": st.n_ops} for st in net.stages],
            "note": "bound valu_f64: the kernel keeps every map in LDS (HBM carries images, "
                    "L2-resident variance maps and one entry per pair); peak = fp64 VALU "
                    "(= fp64 MFMA) 78.6 TF; achieved = credited direct-stencil conv flops of "
                    "the pairs evaluated (i < j on diagonal tiles); one launch = one tile "
                    "(all its stage kernels). " + pmc_note}


def cpu_info():
    model = "?"
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                model = ln.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return model


def host_cpu_budget():
    """CPU threads this process may use on the host: its affinity set, capped by a cgroup
    CPU quota (cgroup v2 cpu.max, v1 cfs_quota) and by the pool's per-GPU CPU share when
    the environment states one (OMP_NUM_THREADS: the GPU pool sets it to the box's share,
    16 per GPU, while nproc / os.cpu_count() report the whole machine).  Returns (threads,
    facts) — every number the choice was made from, for the bench line."""
    facts = {"affinity": len(os.sched_getaffinity(0)), "cpu_count": os.cpu_count()}
    quota = None
    for path, parse in (("/sys/fs/cgroup/cpu.max", lambda t: t.split()),
                        ("/sys/fs/cgroup/cpu/cpu.cfs_quota_us", None)):
        try:
            txt = open(path).read().strip()
        except OSError:
            continue
        if parse:
            q, per = parse(txt)
            if q != "max":
                quota = -(-int(q) // int(per))
        else:
            q = int(txt)
            if q > 0:
                per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
                quota = -(-q // per)
        break
    facts["cgroup_cpu_quota"] = quota
    omp = os.environ.get("OMP_NUM_THREADS")
    facts["OMP_NUM_THREADS"] = int(omp) if omp and omp.isdigit() else None
    threads = facts["affinity"]
    for cap in (quota, facts["OMP_NUM_THREADS"]):
        if cap:
            threads = min(threads, cap)
    return max(1, threads), facts


def cpu_baseline(cfg_name, dtype, seconds):
    """The torch-CPU restatement of the reference (oracle/torch_cpu.py — the reference's
    op sequence, bit-identical to it at C1) on the host's CPU budget (host_cpu_budget:
    affinity, cgroup quota, the pool's per-GPU share), on a Kxz tile sized for about
    ``seconds`` of work after a small warm-up that measures the rate.  The calibration
    restatement/reference measured in the build container (tools/calibrate_cpu.py) is
    quoted beside it."""
    from oracle import specs, torch_cpu
    threads, facts = host_cpu_budget()
    torch.set_num_threads(threads)
    spec = specs.CONFIGS[cfg_name]()
    C, hw = specs.GEOMETRY[cfg_name]
    g = torch.Generator().manual_seed(0)
    dt = dtype
    w = torch.rand((32, C, hw, hw), generator=g, dtype=dt)
    for _ in range(2):                  # the second run measures the warm rate
        t0 = time.perf_counter()
        torch_cpu.kernel(spec, w, w.flip(0), False, False)
        rate = 32 * 32 / (time.perf_counter() - t0)
    side = int(min(256, max(64, (rate * seconds) ** 0.5)))
    X = torch.rand((side, C, hw, hw), generator=g, dtype=dt)
    Z = torch.rand((side, C, hw, hw), generator=g, dtype=dt)
    t0 = time.perf_counter()
    torch_cpu.kernel(spec, X, Z, False, False)
    el = time.perf_counter() - t0
    dtn = "f64" if dt == torch.float64 else "f32"
    res = dict(value=round(side * side / el, 1), unit="pairs/s", cores=torch.get_num_threads(),
               kind="port", nproc=os.cpu_count(), cpu_model=cpu_info(), host_cpus=facts,
               threads_rule="min(affinity, cgroup quota, OMP_NUM_THREADS = the pool's "
                            "per-GPU CPU share)",
               sample=f"one {side}x{side} Kxz tile of {cfg_name} ({side * side} pairs, {dtn}) "
                      f"through oracle/torch_cpu.py (the reference's torch op sequence) "
                      f"in {el:.1f} s on {torch.get_num_threads()} threads")
    cal = load_json(CALIB_FILE)
    if cal:
        case = next((c for c in cal["cases"] if c["config"] == cfg_name and c["dtype"] == dtn),
                    None)
        if case:
            res["calibration"] = {
                "restatement_over_reference": case["restatement_over_reference"],
                "reference_pairs_per_s_build_container": case["reference_pairs_per_s"],
                "threads": cal["threads"], "cpu_model": cal["cpu_model"],
                "max_rel_diff_vs_reference": case["max_rel_diff"],
                "source": "profiles/r2/cpu_calibration.json (tools/calibrate_cpu.py)"}
            res["reference_equivalent_pairs_per_s"] = round(
                res["value"] / case["restatement_over_reference"], 1)
    return res


def time_config(cfg_name, n1, B, steps, warmup, world, rank, dev, dtype, backend, probe):
    """The step loop for one config: Kxx tiles of this rank into a device matrix."""
    cfg = importlib.import_module(f"configs.{cfg_name}")
    model = cfg.initial_model.to(dev, dtype)
    C = getattr(cfg, "in_channels", 1)
    side = 32 if C == 3 else 28
    nb = blocks_for_world(n1, B, world)
    n_total = nb * B if world > 1 else n1
    g = torch.Generator(device="cpu").manual_seed(0)
    X = torch.rand((n_total, C, side, side), generator=g, dtype=dtype).to(dev)
    all_tiles = tile_schedule(n_total, None, B, 0, 1)
    tiles = balanced_split(all_tiles, B, n_total, world)[rank]
    evaluated = sum(tile_eval_pairs(t, B, n_total) for t in all_tiles)
    ref_sched = sum(min(B, n_total - i * B) * min(B, n_total - j * B) for _, i, j in all_tiles)
    K = torch.full((n_total, n_total), float("nan"), dtype=torch.float64, device=dev)

    mk = model_kern(model)

    def step():
        # one Gram build: every image's variance maps once (ModelKern.bind), then each
        # tile from slices of them, written in place into K (cnn_gp.gram's builders)
        bound = mk.bind(X)
        with torch.no_grad():
            for same, i, j in tiles:
                a, b = min(B, n_total - i * B), min(B, n_total - j * B)
                view = K[i * B:i * B + a, j * B:j * B + b]
                if bound is not None:
                    bound.tile((same, i * B, j * B, a, b), view)
                    continue
                xi = X[i * B:(i + 1) * B]
                view.copy_(model(xi) if same else model(xi, X[j * B:(j + 1) * B], False, False))

    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    from cnn_gp import netplan
    netplan.TIMING = [] if rank == 0 and probe else None
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64,
                      device=dev if backend == "nccl" else "cpu")
    if world > 1:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    elapsed = float(el.item())
    timing, netplan.TIMING = netplan.TIMING, None
    return dict(model=model, X=X, K=K, n_total=n_total, tiles=tiles, all_tiles=all_tiles,
                elapsed=elapsed, value=evaluated * steps / elapsed,
                ref_sched_value=ref_sched * steps / elapsed, evaluated=evaluated,
                ms_step=elapsed / steps * 1e3,
                unique=n_total * (n_total + 1) / 2 * steps / elapsed, timing=timing)


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # CGP_BENCH_BACKEND=gloo: rehearse the multi-rank path with several ranks sharing the
    # GPUs there are (RCCL needs one rank per GPU); the default is nccl (RCCL over xGMI)
    backend = os.environ.get("CGP_BENCH_BACKEND", "nccl")
    if backend != "nccl":
        local %= max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
    dtype = torch.float64 if args.dtype == "f64" else torch.float32
    B = args.tile
    probe = not args.no_probe

    r = time_config(args.config, args.n, B, args.steps, args.warmup, world, rank, dev, dtype,
                    backend, probe)
    n_total = r["n_total"]
    extra = {}

    # --- solve of the assembled Kxx (single GPU) ---
    if rank == 0 and world == 1 and not args.no_solve:
        g = torch.Generator().manual_seed(1)
        labels = torch.randint(0, 10, (n_total,), generator=g)
        Y = cnn_gp.one_hot_pm1(labels, 10).to(dev)
        # untimed warm-up solve at the full size (rocBLAS/rocSOLVER load the code objects
        # of each blocked path on first use)
        cnn_gp.solve_system(r["K"], Y, jitter=1e-6)
        times = []
        for _ in range(3):
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            cnn_gp.solve_system(r["K"], Y, jitter=1e-6)      # Kxx kept: copy + factor
            torch.cuda.synchronize()
            times.append(time.perf_counter() - t1)
        t_solve = min(times)
        extra["solve"] = {"n": n_total, "s": round(t_solve, 4),
                          "tflops": round(n_total ** 3 / 3 / t_solve / 1e12, 3),
                          "peak_tflops": FP64_PEAK_TFLOPS,
                          "note": "dpotrf_64 + dpotrs_64 (10 rhs) on a device copy of Kxx "
                                  "(NaN lower triangle), best of 3 after a warm-up"}
        extra["build_solve_wall_s"] = round(r["ms_step"] / 1e3 + t_solve, 4)

    # --- dominant kernel, timed live ---
    roof = None
    if rank == 0 and probe:
        roof = net_roofline(r["model"], r["X"][:B], args.config, r["timing"])
        with torch.no_grad():
            stencil = conv_stencil_roofline(r["model"], r["X"][:B], B)
        if stencil is not None:
            extra["conv_stencil_roofline"] = stencil
    del r["K"]
    torch.cuda.empty_cache()

    # --- BASELINE configs[2]: the ResNet-GP on the same harness ---
    if not args.no_second and args.config != "mnist_as_tf":
        r2 = time_config("mnist_as_tf", args.n, B, max(2, args.steps // 4), 1, world, rank,
                         dev, dtype, backend, probe)
        del r2["K"]
        if rank == 0:
            extra["mnist_as_tf"] = {
                "value": round(r2["value"], 1), "unit": "pairs/s",
                "ms_per_step": round(r2["ms_step"], 3),
                "unique_entries_per_s": round(r2["unique"], 1),
                "reference_schedule_pairs_per_s": round(r2["ref_sched_value"], 1),
                "config": {"workload": f"mnist_as_tf Kxx {r2['n_total']}x{r2['n_total']}, "
                                       f"tiles {B}", "pairs_per_step": r2["evaluated"]},
                "roofline": net_roofline(r2["model"], r2["X"][:B], "mnist_as_tf",
                                         r2["timing"]) if probe else None}
            if world == 1 and not args.no_cpu:
                extra["mnist_as_tf"]["cpu_baseline"] = cpu_baseline(
                    "mnist_as_tf", dtype, args.cpu_seconds)
        torch.cuda.empty_cache()

    # --- the same two workloads at the reference pipeline's own kernel precision ---
    # (exp_mnist_resnet/save_kernel.py runs the float32 model; kernel_save_tools.py:21
    # stores K as float32).  Reported beside the fp64 headline, never as `value`.
    if not args.no_f32 and dtype == torch.float64:
        f32 = {}
        for name in ((args.config,) if args.no_second or args.config == "mnist_as_tf"
                     else (args.config, "mnist_as_tf")):
            r3 = time_config(name, args.n, B, max(2, args.steps // 2), 1, world, rank, dev,
                             torch.float32, backend, False)
            del r3["K"]
            f32[name] = {"value": round(r3["value"], 1), "unit": "pairs/s",
                         "ms_per_step": round(r3["ms_step"], 3),
                         "pairs_per_step": r3["evaluated"]}
            torch.cuda.empty_cache()
        if rank == 0:
            f32["note"] = ("float32 model and images, as the reference's save_kernel.py runs "
                           "them; same Kxx harness as the fp64 legs.  Entries stay within "
                           "3e-7 relative of the fp64 kernel (tests/test_gpu_parity.py "
                           "test_f32_kernel_within_north_star_tolerance; north star 1e-5)")
            extra["f32"] = f32

    # --- BASELINE configs[3]: the full-scale ResNet-GP pipeline ---
    if not args.no_fullscale and dtype == torch.float64:
        from fullscale import fullscale
        t0 = time.perf_counter()
        fs = fullscale("mnist_as_tf", args.fullscale_n, args.fullscale_m, 4096, rank=rank,
                       world=world, dev=dev)
        if rank == 0:
            fs["fullscale_wall_s"] = round(time.perf_counter() - t0, 2)
            fs["data"] = "synthetic MNIST-like (k/255, 60% zeros, 4-px zero border)"
            fs["note"] = PIPELINE_NOTE
            extra["fullscale"] = fs
        torch.cuda.empty_cache()
        if not args.no_fullscale_f32:
            # the same pipeline at the reference pipeline's own kernel precision
            # (save_kernel.py runs the float32 model; K stored float32, widened to float64
            # for the solve by classify_gp.py's load_kern)
            t0 = time.perf_counter()
            fs = fullscale("mnist_as_tf", args.fullscale_n, args.fullscale_m, 4096,
                           rank=rank, world=world, dev=dev, kernel_dtype=torch.float32)
            if rank == 0:
                fs["fullscale_wall_s"] = round(time.perf_counter() - t0, 2)
                fs["note"] = ("kernels in float32 as exp_mnist_resnet/save_kernel.py runs "
                              "them; K widened to float64 on the device for the rocSOLVER "
                              "solve; spot_vs_f64_max_rel_err = float32 entries against "
                              "the float64 model (north-star tolerance 1e-5)")
                extra["fullscale_f32"] = fs
            torch.cuda.empty_cache()

    # --- BASELINE configs[4]: cifar10 ResNet-GP, Kxx 50 000² on 3×32×32 ---
    if not args.no_fullscale_cifar10 and dtype == torch.float64:
        from fullscale import fullscale
        t0 = time.perf_counter()
        fs = fullscale("cifar10", args.cifar10_n, args.fullscale_m, 4096, rank=rank,
                       world=world, dev=dev)
        if rank == 0:
            fs["fullscale_wall_s"] = round(time.perf_counter() - t0, 2)
            fs["data"] = "synthetic CIFAR-like 3x32x32 (k/255, 60% zeros, 4-px zero border)"
            fs["note"] = ("BASELINE configs[4] (configs/cifar10.py:4-47 architecture). " +
                          PIPELINE_NOTE)
            extra["fullscale_cifar10"] = fs
        torch.cuda.empty_cache()

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        cpu = cpu_baseline(args.config, dtype, args.cpu_seconds)

    if rank == 0:
        line = {
            "metric": "kernel entries/s (N×M pairs) + full-Kxx build+solve wall-clock, "
                      "MNIST 28×28",
            "value": round(r["value"], 1),
            "unit": "pairs/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(r["ms_step"], 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": args.dtype,
            "data": "synthetic (torch.rand seed 0, 28x28x1)",
            "config": {"workload": f"{args.config} Kxx {n_total}x{n_total}, tiles {B}",
                       "n": n_total, "tile": B, "tiles_total": len(r["all_tiles"]),
                       "tiles_rank0": len(r["tiles"]), "pairs_per_step": r["evaluated"],
                       "parallelism": f"tiles-dp{world}"},
            "value_counts": "pairs the device evaluates: i < j on diagonal tiles",
            "reference_schedule_pairs_per_s": round(r["ref_sched_value"], 1),
            "unique_entries_per_s": round(r["unique"], 1),
            "roofline": roof,
            "cpu_baseline": cpu,
        }
        line.update(extra)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
