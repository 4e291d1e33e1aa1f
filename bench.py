"""Benchmark: NNGP Gram-matrix build (kernel entries/s) + GP solve on MI355X.

Workload (BASELINE.json configs[1]): mnist_paper_convnet_gp, Kxx of N = 4096 synthetic
28×28×1 images, float64, Gram tiles of B = 1024 in the reference's schedule (upper
triangular tiles).  One STEP = one Gram build: every image's variance maps computed
once (cnn_gp.gram.ModelKern.bind; the reference recomputes them per tile and side), then
every Gram tile of this rank evaluated in place into a device-resident Kxx.

    python bench.py [--gpus N --steps K --warmup W] [--config C --n N --tile B]

--gpus N > 1 without a torchrun environment: this process does no GPU work, starts
``python -m torch.distributed.run --nproc-per-node N ... bench.py <same args>`` as a
child (one rank per GPU, RCCL over xGMI — the reference's run.bash:14-36 starts one
save_kernel.py per visible GPU the same way) and exits with its status.  Under torchrun
--gpus must equal WORLD_SIZE.  CGP_BENCH_BACKEND=gloo rehearses the multi-rank path with
ranks sharing the GPUs there are.

value = kernel entries the device EVALUATES per second, whole job: B1·B2 for an
off-diagonal tile, B(B−1)/2 for a diagonal tile (the kernel computes i < j there and
mirrors; K[i, i] comes from the per-image variance chain).  The reference's schedule
would count B² for a diagonal tile; that figure is reported as
``reference_schedule_pairs_per_s`` beside it.

Also on the same JSON line (each in its own slot; a leg that fails records
{"error": ...} there and the line still prints):
  roofline           the whole-network kernel (net_kernel, fp64 VALU-bound): credited
                     direct-stencil flops vs the fp64 peak, plus the VALU issue
                     utilisation and HBM traffic per launch from the committed PMC
                     passes (profiles/r4/net_pmc.json, rocprofv3)
  mnist_as_tf        the same harness on BASELINE configs[2] (ResNet-GP, 32 layers)
  cifar10            the same harness on configs[4]'s network (3×32×32, Kxx 4096²)
  solve              rocSOLVER/rocBLAS blocked Cholesky + dpotrs_64 on the assembled Kxx
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

Multi-GPU (one process per GPU): the Kxx grows with the world (n_blocks² half-tile units
>= world × the 1-GPU units, divisible by world) and its tiles are split over the ranks by
evaluated pairs — no data-path collective; per-rank work is ~constant ("scaling":
"weak").  The full-scale legs shard their fixed problems ("strong"): Kxx strips to rank 0
point-to-point, α broadcast, scores gathered.  Every collective has a timeout
(CGP_DIST_TIMEOUT_S, default 300 s) and raises instead of hanging; the legs' outcomes are
exchanged over a gloo side group after each leg, so a failure on any rank is recorded
and the remaining multi-rank legs are skipped.
"""
from __future__ import annotations

import argparse
import datetime
import importlib
import json
import os
import socket
import subprocess
import sys
import time
import traceback

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
# committed PMC passes, newest first (a config missing from a newer file is looked up in
# the older one)
PMC_FILES = [os.path.join(ROOT, "profiles", r, "net_pmc.json") for r in ("r4", "r3")]
CALIB_FILES = [os.path.join(ROOT, "profiles", r, "cpu_calibration.json") for r in ("r4", "r2")]
DIST_TIMEOUT_S = float(os.environ.get("CGP_DIST_TIMEOUT_S", "300"))
PIPELINE_NOTE = (
    "cnn_gp.pipeline.classify_distributed: Kxx row strips (B=4096 tiles) balanced by "
    "evaluated pairs, received point-to-point into the full matrix on rank 0 (RCCL with "
    "nccl; that path first runs on the driver's multi-GPU node: every multi-rank run so "
    "far used gloo ranks sharing one GPU); rank 0 factors it (blocked dpotrf/dtrsm/dsyrk, "
    "nb 2048) while the other ranks build their Kxz row strips (rank 0's share sized to "
    "end with them); alpha broadcast, scores = Kxz rows @ alpha per rank, only the scores "
    "gathered; solver code objects loaded on a side thread during the Kxx build; spot "
    "check = HIP vs HIP single pairs in the computed orientation (oracle parity at this "
    "geometry: tests/test_gpu_fullgeom.py, tests/test_gpu_fullscale_bound.py)")


def parse(argv=None):
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
    p.add_argument("--no-cifar10", action="store_true", help="skip the cifar10 Kxx leg")
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
    p.add_argument("--cpu-seconds", type=float, default=12.0,
                   help="target duration of each CPU-baseline sample")
    return p.parse_args(argv)


# ------------------------------------------------------------------------------------------
# launcher: --gpus N starts its own N ranks
# ------------------------------------------------------------------------------------------

def world_error(gpus: int, world: int, n_devices: int, backend: str):
    """Why this rank set cannot run (a message), or None."""
    if gpus < 1:
        return f"--gpus {gpus}: at least one GPU"
    if world != gpus:
        return (f"--gpus {gpus} but WORLD_SIZE is {world}: run `python bench.py --gpus "
                f"{gpus}` (it starts its own ranks) or torchrun with --nproc-per-node {gpus}")
    if backend == "nccl" and world > 1 and world > n_devices:
        return (f"--gpus {gpus} needs {gpus} visible GPUs (one rank per GPU over RCCL); "
                f"{n_devices} visible")
    return None


def launch_cmd(argv, gpus: int, port: int):
    """The child command of the launcher: one rank per GPU on this node, rendezvous on
    127.0.0.1 (the container's hostname may not resolve)."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1",
            "--nproc-per-node", str(gpus), "--master-addr", "127.0.0.1",
            "--master-port", str(port), os.path.abspath(__file__), *argv]


def free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_or_check(args, argv):
    """None: this process runs the bench (one rank).  An int: the exit status to leave
    with — the launched ranks' status, or 2 for a refused rank set.  Makes no GPU call
    (torch.cuda.device_count() does not initialise the runtime on this image), so the
    launcher's child is a fresh process, never an exec of one that touched the GPU."""
    backend = os.environ.get("CGP_BENCH_BACKEND", "nccl")
    env_world = os.environ.get("WORLD_SIZE")
    world = args.gpus if env_world is None else int(env_world)
    err = world_error(args.gpus, world, torch.cuda.device_count(), backend)
    if err:
        print(f"bench.py: {err}", file=sys.stderr, flush=True)
        return 2
    if env_world is not None or args.gpus == 1:
        return None
    cmd = launch_cmd(argv, args.gpus, free_port())
    print(f"bench.py: launching {args.gpus} ranks: {' '.join(cmd)}", file=sys.stderr,
          flush=True)
    return subprocess.call(cmd)


# ------------------------------------------------------------------------------------------
# legs: one failure costs its own slot, not the line
# ------------------------------------------------------------------------------------------

class Legs:
    """Runs each measurement leg and agrees on its outcome across the ranks.

    A leg's exception is caught and recorded as {"error": ...} in its slot; with several
    ranks every rank's outcome is exchanged over a gloo side group (``group``: host
    memory, its own timeout, independent of the RCCL communicator's state), and once any
    rank has failed a leg the remaining multi-rank legs are skipped — a collective could
    otherwise pair with a different leg's on another rank.  CGP_BENCH_FAIL_LEG=<name>[,…]
    forces a failure (tests of this mechanism)."""

    def __init__(self, world: int = 1, rank: int = 0, group=None):
        self.world, self.rank, self.group = world, rank, group
        self.stopped = None

    def run(self, name, fn, multi_rank=True):
        if self.stopped and multi_rank and self.world > 1:
            return {"error": f"skipped: leg {self.stopped!r} failed on a rank"}
        err, out = None, None
        try:
            if name in os.environ.get("CGP_BENCH_FAIL_LEG", "").split(","):
                raise RuntimeError(f"forced failure of leg {name!r} (CGP_BENCH_FAIL_LEG)")
            out = fn()
        except Exception as e:                 # noqa: BLE001 — recorded, never swallowed
            err = f"{type(e).__name__}: {e}"[:1000]
            print(f"bench.py: rank {self.rank}: leg {name!r} failed", file=sys.stderr)
            traceback.print_exc(file=sys.stderr)
            out = None
        if torch.cuda.is_available():
            torch.cuda.empty_cache()
        if self.world > 1 and multi_rank:
            errs = [None] * self.world
            try:
                dist.all_gather_object(errs, err, group=self.group)
            except Exception as e:             # noqa: BLE001
                errs = [f"leg status exchange failed: {type(e).__name__}: {e}"]
            bad = {str(r): m for r, m in enumerate(errs) if m}
            if bad:
                self.stopped = name
                return {"error": bad}
        elif err:
            return {"error": err}
        return out


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


def committed(files, key):
    """(entry, file) of ``key`` in the newest committed JSON that has it, else (None, None)"""
    for f in files:
        v = (load_json(f) or {}).get(key)
        if v is not None:
            return v, os.path.relpath(f, ROOT)
    return None, None


def conv_stencil_roofline(model, x, B, reps=5):
    """Conv2d.propagate alone (kernels.py:92-98; no fused ReLU / moments / Sum) — the
    north star's "Conv2d covariance kernel" — at the config's most frequent conv shape, on
    the B·B pair maps of one tile, timed with HIP events on the launch stream; against the
    8 TB/s HBM roof with algorithmic bytes 8·P·(H·W + Ho·Wo).  A torch copy of the same
    input is timed beside it as the achievable-bandwidth reference.  ``traffic``: the
    committed PMC pass over the same launch (profiles/r*/net_pmc.json "conv_stencil")."""
    from collections import Counter
    _, C, h, w = x.shape
    plan = model._plan(h, w)
    convs = Counter((op.geom.taps, op.geom.offset, op.geom.stride, op.shape_in, op.shape_out)
                    for op in plan.prog.ops
                    if op.kind == "conv" and op.geom.dilation == 1 and op.shape_out[0] > 1)
    if not convs:
        return None
    (k, off, st, (hi, wi), (ho, wo)), _ = convs.most_common(1)[0]
    # the maps of one B = 1024 tile (13 GB of fp64 input at 28²): larger tiles would ask
    # for B²-sized copies (98 GiB at B = 4096) and the committed PMC pass is of this size
    Bs = min(B, 1024)
    P = Bs * Bs
    g = torch.Generator(device="cpu").manual_seed(0)
    var = torch.rand((2 * Bs, hi, wi), generator=g, dtype=x.dtype).add_(0.5).to(x.device)
    xy = (0.5 * (var[:Bs, None] * var[None, Bs:]).sqrt()).reshape(P, hi, wi).contiguous()
    del var
    out = torch.empty((P, ho, wo), dtype=x.dtype, device=x.device)
    stream = torch.cuda.current_stream()
    s = stream.cuda_stream
    a = N.ConvArgs()
    a.in_, a.out = N.ptr(xy), N.ptr(out)
    a.nmaps, a.n1, a.n2 = P, Bs, Bs
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
    pmc, _ = committed(PMC_FILES, "conv_stencil")
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
    pmc, pmc_file = committed(PMC_FILES, cfg_name)
    if pmc and pmc.get("dtype") == str(x.dtype):
        traffic = int(pmc["hbm_bytes_per_pair"] * per_launch)
        quad = pmc["valu_active_quadcycles_per_pair"] * per_launch
        valu = round(4 * quad / (SIMDS * CLOCK_HZ * avg_s), 4)
        valu_insts = round(pmc["valu_insts_per_pair"], 1)
        pmc_note = (f"PMC ({pmc_file}): {pmc['source']}; per pair: {pmc['hbm_bytes_per_pair']:.0f} HBM "
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
    cal, cal_file = None, None
    for f in CALIB_FILES:
        c = load_json(f)
        if c and any(k["config"] == cfg_name for k in c["cases"]):
            cal, cal_file = c, os.path.relpath(f, ROOT)
            break
    if cal:
        case = next((c for c in cal["cases"] if c["config"] == cfg_name and c["dtype"] == dtn),
                    None)
        if case:
            res["calibration"] = {
                "restatement_over_reference": case["restatement_over_reference"],
                "reference_pairs_per_s_build_container": case["reference_pairs_per_s"],
                "threads": cal["threads"], "cpu_model": cal["cpu_model"],
                "max_rel_diff_vs_reference": case["max_rel_diff"],
                "source": f"{cal_file} (tools/calibrate_cpu.py)"}
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
    mine = sum(tile_eval_pairs(t, B, n_total) for t in tiles)
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
    mine_s = time.perf_counter() - t0
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
                unique=n_total * (n_total + 1) / 2 * steps / elapsed, timing=timing,
                rank_stats={"rank": rank, "tiles": len(tiles), "pairs_per_step": mine,
                            "ms_per_step": round(mine_s / steps * 1e3, 3)})


def gather_rank_stats(stats, world, group):
    """every rank's stats dict, on every rank (gloo side group), rank order"""
    if world <= 1:
        return [stats]
    out = [None] * world
    dist.all_gather_object(out, stats, group=group)
    return out


def kxx_leg(cfg_name, args, B, world, rank, dev, dtype, backend, probe, group, steps,
            with_cpu):
    """configs[2] / configs[4]'s network on the headline's harness (Kxx 4096², B = 1024),
    with its own roofline object and CPU baseline"""
    r2 = time_config(cfg_name, args.n, B, steps, 1, world, rank, dev, dtype, backend, probe)
    del r2["K"]
    ranks = gather_rank_stats(r2["rank_stats"], world, group)
    if rank != 0:
        return None
    out = {
        "value": round(r2["value"], 1), "unit": "pairs/s",
        "ms_per_step": round(r2["ms_step"], 3), "steps": steps,
        "unique_entries_per_s": round(r2["unique"], 1),
        "reference_schedule_pairs_per_s": round(r2["ref_sched_value"], 1),
        "config": {"workload": f"{cfg_name} Kxx {r2['n_total']}x{r2['n_total']}, "
                               f"tiles {B}", "pairs_per_step": r2["evaluated"]},
        "ranks": ranks,
        "roofline": net_roofline(r2["model"], r2["X"][:B], cfg_name, r2["timing"])
        if probe else None}
    if with_cpu:
        out["cpu_baseline"] = cpu_baseline(cfg_name, dtype, args.cpu_seconds)
    return out


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse(argv)
    rc = launch_or_check(args, argv)
    if rc is not None:
        return rc
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
    status = None
    if world > 1:
        # a collective that does not complete raises after the timeout instead of hanging
        # until the driver kills the run (blocking wait: the RCCL watchdog would abort)
        os.environ.setdefault("TORCH_NCCL_BLOCKING_WAIT", "1")
        tmo = datetime.timedelta(seconds=DIST_TIMEOUT_S)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev, timeout=tmo)
        else:
            dist.init_process_group(backend, timeout=tmo)
        status = dist.new_group(backend="gloo",
                                timeout=datetime.timedelta(seconds=2 * DIST_TIMEOUT_S + 60))
    legs = Legs(world, rank, status)
    dtype = torch.float64 if args.dtype == "f64" else torch.float32
    B = args.tile
    probe = not args.no_probe
    extra = {}

    def put(name, value):
        if rank == 0 and value is not None:
            extra[name] = value

    # --- the headline: BASELINE configs[1] ---
    r = legs.run("headline", lambda: time_config(args.config, args.n, B, args.steps,
                                                 args.warmup, world, rank, dev, dtype,
                                                 backend, probe))
    failed = "error" in r
    ranks = None
    if not failed:
        ranks = legs.run("rank_stats", lambda: gather_rank_stats(r["rank_stats"], world,
                                                                   status))
    n_total = None if failed else r["n_total"]

    # --- solve of the assembled Kxx (single GPU) ---
    def solve_leg():
        g = torch.Generator().manual_seed(1)
        labels = torch.randint(0, 10, (n_total,), generator=g)
        Y = cnn_gp.one_hot_pm1(labels, 10).to(dev)
        # untimed warm-up solve at the full size (rocBLAS/rocSOLVER load the code objects
        # of each blocked path on first use)
        cnn_gp.solve_system(r["K"], Y, jitter=1e-6)
        times, phases = [], []
        for _ in range(3):
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            cnn_gp.solve_system(r["K"], Y, jitter=1e-6)      # Kxx kept: copy + factor
            torch.cuda.synchronize()
            times.append(time.perf_counter() - t1)
            phases.append(cnn_gp.solve_phases(dev))
        k = min(range(3), key=lambda q: times[q])
        t_solve = times[k]
        ph = {p: round(v, 5) for p, v in phases[k].items()}
        return {"n": n_total, "s": round(t_solve, 4),
                "tflops": round(n_total ** 3 / 3 / t_solve / 1e12, 3),
                "factor_tflops": round(n_total ** 3 / 3 / max(ph["factor_s"], 1e-9) / 1e12, 3),
                "peak_tflops": FP64_PEAK_TFLOPS, **ph,
                "copy_and_transposes_s": round(t_solve - sum(ph.values()), 5),
                "build_solve_wall_s": round(r["ms_step"] / 1e3 + t_solve, 4),
                "note": "blocked dpotrf/dtrsm/dsyrk + dpotrs_64 (10 rhs) on a device copy "
                        "of Kxx (NaN lower triangle), best of 3 after a warm-up; phases "
                        "from HIP events inside cgp_chol_solve_f64"}

    if not failed and rank == 0 and world == 1 and not args.no_solve:
        put("solve", legs.run("solve", solve_leg, multi_rank=False))

    # --- dominant kernel, timed live ---
    roof = None
    if not failed and rank == 0 and probe:
        roof = legs.run("roofline", lambda: net_roofline(r["model"], r["X"][:B], args.config,
                                                         r["timing"]), multi_rank=False)

        def stencil():
            with torch.no_grad():
                return conv_stencil_roofline(r["model"], r["X"][:B], B)
        put("conv_stencil_roofline", legs.run("conv_stencil_roofline", stencil,
                                              multi_rank=False))
    if not failed:
        del r["K"]
    torch.cuda.empty_cache()

    # --- BASELINE configs[2] (ResNet-GP) and configs[4]'s network on the same harness ---
    cpu_ok = world == 1 and not args.no_cpu
    if not args.no_second and args.config != "mnist_as_tf":
        put("mnist_as_tf", legs.run("mnist_as_tf", lambda: kxx_leg(
            "mnist_as_tf", args, B, world, rank, dev, dtype, backend, probe, status,
            max(2, args.steps // 4), cpu_ok)))
    if not args.no_cifar10 and args.config != "cifar10":
        put("cifar10", legs.run("cifar10", lambda: kxx_leg(
            "cifar10", args, B, world, rank, dev, dtype, backend, probe, status,
            max(2, args.steps // 4), cpu_ok)))

    # --- the same workloads at the reference pipeline's own kernel precision ---
    # (exp_mnist_resnet/save_kernel.py runs the float32 model; kernel_save_tools.py:21
    # stores K as float32).  Reported beside the fp64 headline, never as `value`.
    if not args.no_f32 and dtype == torch.float64:
        def f32_leg():
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
            f32["note"] = ("float32 model and images, as the reference's save_kernel.py runs "
                           "them; same Kxx harness as the fp64 legs.  Entries stay within "
                           "3e-7 relative of the fp64 kernel (tests/test_gpu_parity.py "
                           "test_f32_kernel_within_north_star_tolerance; north star 1e-5)")
            return f32 if rank == 0 else None
        put("f32", legs.run("f32", f32_leg))

    # --- BASELINE configs[3] / [4]: the full-scale ResNet-GP pipelines ---
    def fullscale_leg(config, n, kernel_dtype, data, note):
        from fullscale import fullscale
        t0 = time.perf_counter()
        fs = fullscale(config, n, args.fullscale_m, 4096, rank=rank, world=world, dev=dev,
                       kernel_dtype=kernel_dtype, stats_group=status)
        if rank != 0:
            return None
        fs["fullscale_wall_s"] = round(time.perf_counter() - t0, 2)
        fs["data"] = data
        fs["note"] = note
        return fs

    mnist_data = "synthetic MNIST-like (k/255, 60% zeros, 4-px zero border)"
    if not args.no_fullscale and dtype == torch.float64:
        put("fullscale", legs.run("fullscale", lambda: fullscale_leg(
            "mnist_as_tf", args.fullscale_n, torch.float64, mnist_data, PIPELINE_NOTE)))
        if not args.no_fullscale_f32:
            # the same pipeline at the reference pipeline's own kernel precision
            # (save_kernel.py runs the float32 model; K stored float32, widened to float64
            # for the solve by classify_gp.py's load_kern)
            put("fullscale_f32", legs.run("fullscale_f32", lambda: fullscale_leg(
                "mnist_as_tf", args.fullscale_n, torch.float32, mnist_data,
                "kernels in float32 as exp_mnist_resnet/save_kernel.py runs them; K widened "
                "to float64 on the device for the rocSOLVER solve; spot_vs_f64_max_rel_err "
                "= float32 entries against the float64 model (north-star tolerance 1e-5)")))
    if not args.no_fullscale_cifar10 and dtype == torch.float64:
        put("fullscale_cifar10", legs.run("fullscale_cifar10", lambda: fullscale_leg(
            "cifar10", args.cifar10_n, torch.float64,
            "synthetic CIFAR-like 3x32x32 (k/255, 60% zeros, 4-px zero border)",
            "BASELINE configs[4] (configs/cifar10.py:4-47 architecture). " + PIPELINE_NOTE)))

    cpu = None
    if rank == 0 and cpu_ok:
        cpu = legs.run("cpu_baseline", lambda: cpu_baseline(args.config, dtype,
                                                            args.cpu_seconds),
                       multi_rank=False)

    if rank == 0:
        line = {
            "metric": "kernel entries/s (N×M pairs) + full-Kxx build+solve wall-clock, "
                      "MNIST 28×28",
            "value": None if failed else round(r["value"], 1),
            "unit": "pairs/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": None if failed else round(r["ms_step"], 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": args.dtype,
            "data": "synthetic (torch.rand seed 0, 28x28x1)",
            "config": {"workload": f"{args.config} Kxx {n_total}x{n_total}, tiles {B}",
                       "n": n_total, "tile": B,
                       "tiles_total": None if failed else len(r["all_tiles"]),
                       "tiles_rank0": None if failed else len(r["tiles"]),
                       "pairs_per_step": None if failed else r["evaluated"],
                       "parallelism": f"tiles-dp{world}"},
            "world": world,
            "backend": backend if world > 1 else None,
            "value_counts": "pairs the device evaluates: i < j on diagonal tiles",
            "reference_schedule_pairs_per_s": None if failed else round(r["ref_sched_value"], 1),
            "unique_entries_per_s": None if failed else round(r["unique"], 1),
            "ranks": ranks,
            "roofline": roof,
            "cpu_baseline": cpu,
        }
        if failed:
            line["error"] = r["error"]
        line.update(extra)
        print(json.dumps(line), flush=True)
    if world > 1:
        try:
            dist.destroy_process_group()
        except Exception:                      # noqa: BLE001 — after a failed leg
            pass
    return 1 if failed else 0


if __name__ == "__main__":
    sys.exit(main())
