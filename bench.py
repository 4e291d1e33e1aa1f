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

Also on the same JSON line, in this order (each in its own slot; a leg that fails records
{"error": ...} there and the line still prints; the line is compact_line() of the full
result, which is written to gpurun_out/bench_full.json — DESIGN.md §6 defines each leg):
  roofline           the whole-network kernel (net_kernel, fp64 VALU-bound): credited
                     direct-stencil flops vs the fp64 peak, the issued fp64 flops and the
                     VALU issue fraction and HBM traffic from the committed PMC passes
  cpu_baseline       the torch-CPU restatement of the reference (oracle/torch_cpu.py,
                     bit-identical to the reference at C1) on the host threads torch is
                     given, with the committed calibration against the reference
  conv_stencil_roofline  Conv2d.propagate alone (the north star's "Conv2d covariance
                     kernel") against the 8 TB/s HBM roof, PMC traffic committed
  mnist_as_tf        the same harness on BASELINE configs[2] (ResNet-GP, 32 layers)
  solve              the blocked Cholesky + dpotrs_64 on the assembled Kxx
  cifar10            the same harness on configs[4]'s network (3×32×32, Kxx 4096²)
  dropin             save_kernel.py's own loop (save_K + a per-tile kern, float32) at
                     batch 200 and 1024 beside the bound build (one rank only)
  f32                the Kxx legs with float32 kernels (the reference pipeline's precision)
  fullscale          BASELINE configs[3]: mnist_as_tf Kxx 60 000² + Kxz 10 000 × 60 000
                     + solve + predict (tools/fullscale.py, cnn_gp/pipeline.py)
  fullscale_cifar10  BASELINE configs[4]: cifar10 Kxx 50 000² + Kxz + solve + predict
  fullscale_f32      configs[3] with float32 kernels

Multi-GPU (one process per GPU): the Kxx grows with the world (n_blocks² half-tile units
>= world × the 1-GPU units, divisible by world) and its tiles are split over the ranks by
evaluated pairs — no data-path collective; per-rank work is ~constant ("scaling":
"weak").  The full-scale legs shard their fixed problems ("strong"): Kxx strips to rank 0
point-to-point, α broadcast, scores gathered.  Every collective has a timeout
(CGP_DIST_TIMEOUT_S, default 120 s) and raises instead of hanging; the legs' outcomes are
exchanged over a gloo side group after each leg, so a failure on any rank is recorded
and the remaining multi-rank legs are skipped.  A leg that would start past
CGP_BENCH_BUDGET_S (420 s) is skipped, and a watchdog prints the line at CGP_BENCH_HARD_S
(540 s) whatever a rank is stuck in.
"""
from __future__ import annotations

import argparse
import datetime
import importlib
import json
import os
import socket
import statistics
import subprocess
import sys
import threading
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
PMC_FILES = [os.path.join(ROOT, "profiles", r, "net_pmc.json") for r in ("r6", "r5", "r4", "r3")]
# the fp64 flop counters of the same kernel code (tools/pmc_flops.sh)
FLOPS_FILES = [os.path.join(ROOT, "profiles", r, "flops_pmc.json") for r in ("r6", "r5")]
CALIB_FILES = [os.path.join(ROOT, "profiles", r, "cpu_calibration.json") for r in ("r4", "r2")]
DIST_TIMEOUT_S = float(os.environ.get("CGP_DIST_TIMEOUT_S", "120"))


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
    p.add_argument("--no-dropin", action="store_true",
                   help="skip the literal save_kernel.py loop (save_K + per-tile kern)")
    p.add_argument("--dropin-n", type=int, default=4096)
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

class Deadline:
    """The run's wall-clock budget (the driver allows the bench 600 s).  A leg that would
    start after ``budget_s`` (its estimate included) is recorded as skipped; at ``hard_s``
    a watchdog on rank 0 prints the line from what has been recorded and ends the process
    (a hung collective cannot hold the line back).  CGP_BENCH_BUDGET_S / CGP_BENCH_HARD_S
    override the defaults (420 s / 540 s)."""

    def __init__(self, budget_s=None, hard_s=None, t0=None):
        env = os.environ.get
        self.budget_s = float(budget_s if budget_s is not None
                              else env("CGP_BENCH_BUDGET_S", "420"))
        self.hard_s = float(hard_s if hard_s is not None else env("CGP_BENCH_HARD_S", "540"))
        self.t0 = time.monotonic() if t0 is None else t0

    def elapsed(self):
        return time.monotonic() - self.t0

    def over(self, est_s=0.0):
        return self.elapsed() + est_s > self.budget_s


class Emitter:
    """Prints the one JSON line exactly once: from the main thread at the end of the run,
    or from the watchdog at the hard deadline, whichever comes first."""

    def __init__(self, write=None):
        self.lock = threading.Lock()
        self.done = False
        self.write = write or (lambda s: (sys.stdout.write(s + "\n"), sys.stdout.flush()))

    def emit(self, make_line) -> bool:
        with self.lock:
            if self.done:
                return False
            self.done = True
            self.write(json.dumps(make_line()))
            return True


class Watchdog(threading.Thread):
    """Rank 0's guard against a leg that never returns (e.g. a collective whose peer hung):
    at the deadline's hard limit it emits the line (the running leg marked) and calls
    ``exit_fn`` (default os._exit(3): torchrun then tears the other ranks down)."""

    def __init__(self, deadline, emitter, make_line, exit_fn=None):
        super().__init__(daemon=True, name="bench-watchdog")
        self.deadline, self.emitter, self.make_line = deadline, emitter, make_line
        self.exit_fn = exit_fn or (lambda: os._exit(3))
        self.stop = threading.Event()

    def run(self):
        if self.stop.wait(max(0.0, self.deadline.hard_s - self.deadline.elapsed())):
            return
        print(f"bench.py: watchdog: {self.deadline.hard_s:.0f} s reached, printing the line",
              file=sys.stderr, flush=True)

        def line():
            # the main thread may be updating the result while it is read: retry once,
            # then fall back to the headline keys alone
            for _ in range(2):
                try:
                    return json.loads(json.dumps(self.make_line(watchdog=True)))
                except Exception:              # noqa: BLE001
                    time.sleep(0.5)
            return {"metric": None, "value": None, "watchdog": "line unavailable"}
        if self.emitter.emit(line):
            self.exit_fn()


class Legs:
    """Runs each measurement leg and agrees on its outcome across the ranks.

    A leg's exception is caught and recorded as {"error": ...} in its slot; with several
    ranks every rank's outcome is exchanged over a gloo side group (``group``: host
    memory, its own timeout, independent of the RCCL communicator's state), and once any
    rank has failed a leg the remaining multi-rank legs are skipped — a collective could
    otherwise pair with a different leg's on another rank.  A leg that would start past
    the deadline's budget (``est_s`` its expected duration) is skipped on every rank (the
    ranks agree on it first).  CGP_BENCH_FAIL_LEG=<name>[,…] forces a failure and
    CGP_BENCH_HANG_LEG=<name>:<rank> makes that rank block inside the leg (tests of these
    mechanisms)."""

    def __init__(self, world: int = 1, rank: int = 0, group=None, deadline=None):
        self.world, self.rank, self.group = world, rank, group
        self.deadline = deadline
        self.stopped = None
        self.current = None

    def _agree(self, flag):
        flags = [None] * self.world
        dist.all_gather_object(flags, flag, group=self.group)
        return any(flags)

    def run(self, name, fn, multi_rank=True, est_s=0.0):
        if self.stopped and multi_rank and self.world > 1:
            return {"error": f"skipped: leg {self.stopped!r} failed on a rank"}
        over = self.deadline is not None and self.deadline.over(est_s)
        if self.world > 1 and multi_rank:
            over = self._agree(over)
        if over:
            return {"error": f"skipped: budget ({self.deadline.elapsed():.0f} s used, "
                             f"~{est_s:.0f} s needed, {self.deadline.budget_s:.0f} s allowed)"}
        err, out = None, None
        self.current = name
        try:
            if name in os.environ.get("CGP_BENCH_FAIL_LEG", "").split(","):
                raise RuntimeError(f"forced failure of leg {name!r} (CGP_BENCH_FAIL_LEG)")
            if f"{name}:{self.rank}" in os.environ.get("CGP_BENCH_HANG_LEG", "").split(","):
                threading.Event().wait()          # blocks for good (watchdog test)
            out = fn()
        except Exception as e:                 # noqa: BLE001 — recorded, never swallowed
            err = f"{type(e).__name__}: {e}"[:300]
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
                errs = [f"leg status exchange failed: {type(e).__name__}: {e}"[:300]]
            bad = {str(r): m for r, m in enumerate(errs) if m}
            self.current = None
            if bad:
                self.stopped = name
                return {"error": bad}
        elif err:
            self.current = None
            return {"error": err}
        self.current = None
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
    # issued fp64 flops: every lane of every issued fp64 instruction (PMC flop counters of
    # the same code, per pair) over this run's live launch time — what the kernel executes,
    # where `achieved` credits the reference's direct-stencil flops
    issued = issued_frac = None
    fpmc, _ = committed(FLOPS_FILES, cfg_name)
    if fpmc and x.dtype == torch.float64:
        issued = fpmc["issued_lane_flops_per_pair"] * pairs / (ms * 1e-3) / 1e12
        issued_frac = round(issued / FP64_PEAK_TFLOPS, 4)
        issued = round(issued, 2)
    kname = f"net_kernel<{'double' if x.dtype == torch.float64 else 'float'}>"
    return {"bound": "valu_f64", "achieved": round(achieved, 2), "peak": FP64_PEAK_TFLOPS,
            "unit": "TFLOP/s", "frac": round(achieved / FP64_PEAK_TFLOPS, 4),
            "traffic": traffic, "valu_issue_frac": valu,
            "issued_fp64_tflops": issued, "issued_fp64_frac": issued_frac,
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


def time_config(cfg_name, n1, B, steps, warmup, world, rank, dev, dtype, backend, probe,
                ctl=None):
    """The step loop for one config: Kxx tiles of this rank into a device matrix.  The
    barriers around the timed steps and the max over ranks run on ``ctl`` (the gloo side
    group, host memory): the build has no data-path collective, so the measurement does
    not depend on RCCL."""
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
    K = torch.full((n_total, n_total), float("nan"), dtype=dtype, device=dev)

    mk = model_kern(model)

    def step():
        build_kxx(mk, model, X, K, tiles, B, n_total)

    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier(group=ctl)
    from cnn_gp import netplan
    netplan.TIMING = [] if rank == 0 and probe else None
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    mine_s = time.perf_counter() - t0
    if world > 1:
        dist.barrier(group=ctl)
    el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
    if world > 1:
        dist.all_reduce(el, op=dist.ReduceOp.MAX, group=ctl)
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
    r2 = time_config(cfg_name, args.n, B, steps, 1, world, rank, dev, dtype, backend, probe,
                     group)
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


# ------------------------------------------------------------------------------------------
# the drop-in path itself: save_kernel.py's loop, timed
# ------------------------------------------------------------------------------------------

class MemH5:
    """In-memory stand-in for the h5py.File save_K writes (h5py is not installed here):
    create_dataset(...) -> a NaN-filled float32 numpy array with slice assignment."""

    def __init__(self):
        self.d = {}

    def keys(self):
        return self.d.keys()

    def create_dataset(self, name, shape, dtype, fillvalue, chunks, maxshape):
        import numpy as np
        self.d[name] = np.full(shape, fillvalue, dtype=dtype)
        return self.d[name]


def build_kxx(mk, model, X, K, tiles, B, n):
    """One Gram build of the bench's step: every image's variance maps once
    (ModelKern.bind), then each tile written in place into K (cnn_gp.gram's builders)."""
    bound = mk.bind(X)
    with torch.no_grad():
        for same, i, j in tiles:
            a, b = min(B, n - i * B), min(B, n - j * B)
            view = K[i * B:i * B + a, j * B:j * B + b]
            if bound is not None:
                bound.tile((same, i * B, j * B, a, b), view)
                continue
            xi = X[i * B:(i + 1) * B]
            view.copy_(model(xi) if same else model(xi, X[j * B:(j + 1) * B], False, False))


def dropin_leg(cfg_names, n, tiles, dev, reps=5):
    """exp_mnist_resnet/save_kernel.py:19-29 verbatim in effect: the float32 model
    (config.initial_model.cuda()), host float32 images in a Dataset, and
    ``kern(x, x2, same, diag) = model(x.cuda(), x2.cuda(), same, diag).cpu().numpy()`` driven
    tile by tile by save_K (kernel_save_tools.py:26-58: ProductIterator batches, the
    isfinite check, the write into a float32 (1, N, N) dataset; an in-memory stand-in for
    the h5py file), timed ``reps`` times after two warm passes (the median is reported: one
    pass is 20-140 ms, and single passes spread by ±15%).  Beside it, the bound build (the
    bench's step: maps once, tiles in place, no host copies) on the same images, model and
    tile size.  The two matrices are compared on the upper tiles after every case has been
    timed: the comparison's 64 MB pageable copy back made the helper threads' next-case
    H2D copies wait on the other threads' kernels (ConvNet B = 1024: 0.38 → 4-7 ms per
    call, profiles/r6/r6x_dropin_copy_stall.log).  pairs = N(N−1)/2 for both (the
    headline's count).  CGP_DROPIN_TRACE=1 adds each call's mean H2D / forward / copy-back
    times (a diagnostic: the timed kern is the plain one otherwise)."""
    import contextlib
    import numpy as np
    from torch.utils.data import TensorDataset
    from cnn_gp.kernel_save_tools import save_K
    pairs = n * (n - 1) // 2
    out, checks = {}, []
    pin = os.environ.get("CGP_DROPIN_PIN", "1") != "0"       # save_K's default: pinned
    for name in cfg_names:
        cfg = importlib.import_module(f"configs.{name}")
        # float32 buffers, as save_kernel.py:19 gets them from a fresh import (the fp64 legs
        # before this one converted the shared config module in place)
        model = cfg.initial_model.to(dev, torch.float32)
        C = getattr(cfg, "in_channels", 1)
        side = 32 if C == 3 else 28
        g = torch.Generator().manual_seed(0)
        X = torch.rand((n, C, side, side), generator=g, dtype=torch.float32)
        ds = TensorDataset(X, torch.zeros(n, dtype=torch.int64))
        trace = []

        def kern(x, x2, same, diag):                # save_kernel.py:21-24
            with torch.no_grad():
                return model(x.cuda(dev), x2.cuda(dev), same, diag).detach().cpu().numpy()

        if os.environ.get("CGP_DROPIN_TRACE"):
            def kern(x, x2, same, diag):            # noqa: F811
                with torch.no_grad():
                    t0 = time.perf_counter()
                    a, b = x.cuda(dev), x2.cuda(dev)
                    t1 = time.perf_counter()
                    k = model(a, b, same, diag)
                    t2 = time.perf_counter()
                    o = k.detach().cpu().numpy()
                    trace.append((t1 - t0, t2 - t1, time.perf_counter() - t2))
                    return o

        Xd = X.to(dev)
        mk = model_kern(model)
        for B in tiles:
            with contextlib.redirect_stdout(sys.stderr):   # save_K's progress lines
                # warm: two whole passes (every tile shape, the ragged edge's included, on
                # every helper thread of save_K: each keeps its stream's tile recipes — the
                # steady state of save_kernel.py's five save_K calls)
                for _ in range(2):
                    save_K(MemH5(), kern, "Kxx", ds, None, False, B, print_interval=1e9,
                           pin=pin)
                torch.cuda.synchronize()
                els = []
                trace.clear()
                for _ in range(reps):
                    f = MemH5()
                    t0 = time.perf_counter()
                    save_K(f, kern, "Kxx", ds, None, False, B, print_interval=1e9, pin=pin)
                    els.append(time.perf_counter() - t0)
            el = statistics.median(els)
            K = torch.full((n, n), float("nan"), dtype=torch.float32, device=dev)
            sched = tile_schedule(n, None, B, 0, 1)
            build_kxx(mk, model, Xd, K, sched, B, n)        # warm
            torch.cuda.synchronize()
            els_b = []
            for _ in range(reps):
                t0 = time.perf_counter()
                build_kxx(mk, model, Xd, K, sched, B, n)
                torch.cuda.synchronize()
                els_b.append(time.perf_counter() - t0)
            el_b = statistics.median(els_b)
            key = f"{name}/B{B}"
            checks.append((key, f.d["Kxx"][0], K))
            out[key] = {
                "pairs_per_s": round(pairs / el), "s": round(el, 4), "tiles": len(sched),
                "ms_per_tile": round(el / len(sched) * 1e3, 3),
                "bound_pairs_per_s": round(pairs / el_b), "over_bound": round(el_b / el, 3),
                "reps": reps, "s_range": [round(min(els), 4), round(max(els), 4)]}
            if trace:
                out[key]["trace_ms_h2d_fwd_d2h"] = [
                    round(sum(t[c] for t in trace) / len(trace) * 1e3, 3) for c in range(3)]
        del Xd
    for key, Kf, K in checks:                       # after every case's timing (docstring)
        Kb = K.cpu().numpy()
        mask = ~np.isnan(Kf)
        out[key]["max_rel_diff_vs_bound"] = float(
            np.max(np.abs(Kf[mask] - Kb[mask]) / np.abs(Kb[mask])))
    checks.clear()                                  # the matrices go before the next leg
    K = None
    torch.cuda.empty_cache()
    return {"n": n, "dtype": "f32", "cases": out}


# ------------------------------------------------------------------------------------------
# the line: every leg's numbers, compact (the driver keeps ~8 KB of stdout)
# ------------------------------------------------------------------------------------------

LINE_MAX_CHARS = 7000


def _sig(x, digits=4):
    """x rounded to ``digits`` significant digits (ints and None pass through)"""
    if not isinstance(x, float) or x != x or x in (float("inf"), float("-inf")):
        return x
    if x == 0.0:
        return 0.0
    import math
    d = digits - int(math.floor(math.log10(abs(x)))) - 1
    return round(x, d) if d > 0 else float(round(x, d))


def _pick(d, keys, digits=4):
    if not isinstance(d, dict):
        return d
    if "error" in d:
        e = d["error"]
        return {"error": e if isinstance(e, str) else {k: str(v)[:200] for k, v in e.items()}}
    return {k: _sig(d[k], digits) for k in keys if d.get(k) is not None}


_ROOF_KEYS = ("bound", "achieved", "peak", "unit", "frac", "traffic", "avg_ms",
              "valu_issue_frac", "issued_fp64_frac", "valu_insts_per_pair", "launches")
_CPU_KEYS = ("value", "unit", "cores", "kind", "sample", "reference_equivalent_pairs_per_s")
_FS_KEYS = ("n", "m", "total_s", "kxx_s", "kxx_pairs_per_s", "kxz_s", "kxz_s_rank0",
            "gather_kxx_s", "solve_s", "solve_tflops", "predict_s", "residual",
            "spot_check_hip_vs_hip_max_rel_err", "spot_vs_f64_max_rel_err",
            "rank0_peak_gather_solve_over_kxx", "fullscale_wall_s")


def _cpu(c):
    if not isinstance(c, dict) or "error" in c:
        return _pick(c, ())
    out = _pick(c, _CPU_KEYS)
    out["sample"] = str(c.get("sample", ""))[:90]
    return out


def _kxx_leg(d):
    if not isinstance(d, dict) or "error" in d:
        return _pick(d, ())
    out = {"value": round(d["value"]), "ms_per_step": _sig(d["ms_per_step"]),
           "workload": d["config"]["workload"], "roofline": _pick(d.get("roofline"), _ROOF_KEYS)}
    if d.get("cpu_baseline") is not None:
        out["cpu_baseline"] = _cpu(d["cpu_baseline"])
    if len(d.get("ranks") or []) > 1:
        out["ranks_ms"] = [_sig(r["ms_per_step"]) for r in d["ranks"]]
    return out


def _fullscale(d):
    if not isinstance(d, dict) or "error" in d:
        return _pick(d, ())
    out = _pick(d, _FS_KEYS, 5)
    sp = d.get("solve_split") or {}
    out.update({k: _sig(sp[k]) for k in ("factor_s", "factor_tflops", "potrs_s", "widen_s")
                if sp.get(k) is not None})
    if d.get("harness_s") is not None:
        out["residual_rows_s_outside_solve"] = _sig(d["harness_s"])
    if d.get("ranks"):
        out["ranks"] = {k: [_sig(r.get(k)) for r in d["ranks"]]
                        for k in ("kxx_s", "gather_kxx_s", "kxz_s")}
    return out


def compact_line(full: dict) -> dict:
    """The printed line: the headline keys of the bench contract, then every leg with its
    value, roofline and CPU baseline, headline-first and full-scale last; per-leg prose,
    plans and per-rank dicts stay in the full result file (``full_result``) and in
    DESIGN.md §6.  Kept under LINE_MAX_CHARS (tests/test_bench_launcher.py)."""
    keep = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
            "higher_is_better", "scaling", "vs_baseline", "dtype", "data")
    line = {k: full.get(k) for k in keep}
    line["value"] = None if full.get("value") is None else round(full["value"])
    cfg = full.get("config") or {}
    line["config"] = {k: cfg[k] for k in ("workload", "n", "tile", "pairs_per_step",
                                          "parallelism") if k in cfg}
    if full.get("world", 1) > 1:
        line["backend"] = full.get("backend")
        line["ranks_ms"] = [_sig(r["ms_per_step"]) for r in (full.get("ranks") or [])
                            if isinstance(r, dict) and "ms_per_step" in r]
    for k in ("error", "watchdog"):
        if full.get(k) is not None:
            line[k] = str(full[k])[:300]
    if full.get("elapsed_s") is not None:
        line["elapsed_s"] = full["elapsed_s"]          # the whole run, rank 0's clock
    line["roofline"] = _pick(full.get("roofline"), _ROOF_KEYS)
    line["cpu_baseline"] = _cpu(full.get("cpu_baseline"))
    line["reference_schedule_pairs_per_s"] = _sig(full.get("reference_schedule_pairs_per_s"))
    line["unique_entries_per_s"] = _sig(full.get("unique_entries_per_s"))
    if "conv_stencil_roofline" in full:
        line["conv_stencil_roofline"] = _pick(
            full["conv_stencil_roofline"], ("bound", "achieved", "peak", "unit", "frac",
                                            "traffic", "kernel", "avg_ms", "pmc_avg_ms",
                                            "alg_bytes_per_launch", "torch_copy_GBs"))
    for k in ("mnist_as_tf", "cifar10"):
        if k in full:
            line[k] = _kxx_leg(full[k])
    if "solve" in full:
        line["solve"] = _pick(full["solve"], ("n", "s", "factor_s", "factor_tflops", "potrs_s",
                                              "build_solve_wall_s"))
    if "dropin" in full:
        d = full["dropin"]
        if isinstance(d, dict) and "cases" in d:
            line["dropin"] = {"n": d["n"], "dtype": d["dtype"], **{
                k: _pick(v, ("pairs_per_s", "ms_per_tile", "bound_pairs_per_s", "over_bound",
                             "max_rel_diff_vs_bound"), 3) for k, v in d["cases"].items()}}
        else:
            line["dropin"] = _pick(d, ())
    if "f32" in full:
        f = full["f32"]
        line["f32"] = {k: round(v["value"]) for k, v in f.items() if isinstance(v, dict)
                       and "value" in v} if "error" not in f else _pick(f, ())
    for k in ("fullscale", "fullscale_f32", "fullscale_cifar10"):
        if k in full:
            line[k] = _fullscale(full[k])
    if full.get("full_result"):
        line["full_result"] = full["full_result"]
    line["notes"] = "per-leg definitions: DESIGN.md §6; full result: full_result"
    return line


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse(argv)
    rc = launch_or_check(args, argv)
    if rc is not None:
        return rc
    deadline = Deadline()
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
            # host tensors on gloo, device tensors on RCCL (its communicator is created at
            # the first device collective, i.e. in the full-scale legs): the Kxx legs'
            # control plane never waits on RCCL, so a broken RCCL costs those legs only
            dist.init_process_group("cpu:gloo,cuda:nccl", timeout=tmo)
        else:
            dist.init_process_group(backend, timeout=tmo)
        # the status exchange waits for a rank still inside a timed-out collective; the
        # watchdog bounds the whole run
        status = dist.new_group(backend="gloo",
                                timeout=datetime.timedelta(seconds=DIST_TIMEOUT_S + 60))
    legs = Legs(world, rank, status, deadline)
    dtype = torch.float64 if args.dtype == "f64" else torch.float32
    B = args.tile
    probe = not args.no_probe
    full = {
        "metric": "kernel entries/s (N×M pairs) + full-Kxx build+solve wall-clock, "
                  "MNIST 28×28",
        "value": None, "unit": "pairs/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": None, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": args.dtype,
        "data": "synthetic (torch.rand seed 0, 28x28x1)",
        "config": {"workload": f"{args.config} Kxx {args.n}x{args.n}, tiles {B}",
                   "n": args.n, "tile": B, "parallelism": f"tiles-dp{world}"},
        "world": world, "backend": backend if world > 1 else None,
        "value_counts": "pairs the device evaluates: i < j on diagonal tiles",
        "roofline": None, "cpu_baseline": None}
    full_path = os.environ.get("CGP_BENCH_FULL_OUT",
                               os.path.join(ROOT, "gpurun_out", "bench_full.json"))
    full["full_result"] = os.path.relpath(full_path, ROOT)

    def make_line(watchdog=False):
        snap = dict(full)
        snap["elapsed_s"] = round(deadline.elapsed(), 1)
        if watchdog:
            snap["watchdog"] = (f"hard limit {deadline.hard_s:.0f} s reached during leg "
                                f"{legs.current!r}; later legs not run")
        return compact_line(snap)

    emitter = Emitter()
    dog = None
    if rank == 0:
        dog = Watchdog(deadline, emitter, make_line)
        dog.start()

    def put(name, value):
        if rank == 0 and value is not None:
            full[name] = value

    # --- the headline: BASELINE configs[1] ---
    r = legs.run("headline", lambda: time_config(args.config, args.n, B, args.steps,
                                                 args.warmup, world, rank, dev, dtype,
                                                 backend, probe, status))
    failed = "error" in r
    if failed:
        full["error"] = r["error"]
    else:
        n_total = r["n_total"]
        full.update(value=r["value"], ms_per_step=round(r["ms_step"], 3),
                    reference_schedule_pairs_per_s=round(r["ref_sched_value"], 1),
                    unique_entries_per_s=round(r["unique"], 1))
        full["config"].update(workload=f"{args.config} Kxx {n_total}x{n_total}, tiles {B}",
                              n=n_total, tiles_total=len(r["all_tiles"]),
                              tiles_rank0=len(r["tiles"]), pairs_per_step=r["evaluated"])
        full["ranks"] = legs.run("rank_stats", lambda: gather_rank_stats(r["rank_stats"],
                                                                         world, status))

    # --- dominant kernel (timed live in the headline) and the Conv2d stencil alone ---
    if not failed and rank == 0 and probe:
        full["roofline"] = legs.run("roofline", lambda: net_roofline(
            r["model"], r["X"][:B], args.config, r["timing"]), multi_rank=False)

        def stencil():
            with torch.no_grad():
                return conv_stencil_roofline(r["model"], r["X"][:B], B)
        put("conv_stencil_roofline", legs.run("conv_stencil_roofline", stencil,
                                              multi_rank=False))

    # --- BASELINE configs[2] (ResNet-GP) on the same harness, with its CPU baseline ---
    cpu_ok = world == 1 and not args.no_cpu
    if not args.no_second and args.config != "mnist_as_tf":
        put("mnist_as_tf", legs.run("mnist_as_tf", lambda: kxx_leg(
            "mnist_as_tf", args, B, world, rank, dev, dtype, backend, probe, status,
            max(2, args.steps // 4), cpu_ok), est_s=40))
    if rank == 0 and cpu_ok:
        full["cpu_baseline"] = legs.run("cpu_baseline", lambda: cpu_baseline(
            args.config, dtype, args.cpu_seconds), multi_rank=False, est_s=20)

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
                "build_solve_wall_s": round(r["ms_step"] / 1e3 + t_solve, 4)}

    if not failed and rank == 0 and world == 1 and not args.no_solve:
        put("solve", legs.run("solve", solve_leg, multi_rank=False, est_s=5))
    if not failed:
        del r["K"]
    torch.cuda.empty_cache()

    # --- configs[4]'s network on the same harness ---
    if not args.no_cifar10 and args.config != "cifar10":
        put("cifar10", legs.run("cifar10", lambda: kxx_leg(
            "cifar10", args, B, world, rank, dev, dtype, backend, probe, status,
            max(2, args.steps // 4), cpu_ok), est_s=40))

    # --- the literal drop-in path (save_kernel.py's loop), beside the bound build ---
    if world == 1 and not args.no_dropin:       # a per-process path: measured at N = 1
        put("dropin", legs.run("dropin", lambda: dropin_leg(
            (args.config, "mnist_as_tf"), args.dropin_n, (200, 1024), dev),
            multi_rank=False, est_s=20))

    # --- the same workloads at the reference pipeline's own kernel precision ---
    # (exp_mnist_resnet/save_kernel.py runs the float32 model; kernel_save_tools.py:21
    # stores K as float32).  Reported beside the fp64 headline, never as `value`.
    if not args.no_f32 and dtype == torch.float64:
        def f32_leg():
            f32 = {}
            for name in ((args.config,) if args.no_second or args.config == "mnist_as_tf"
                         else (args.config, "mnist_as_tf")):
                r3 = time_config(name, args.n, B, max(2, args.steps // 2), 1, world, rank, dev,
                                 torch.float32, backend, False, status)
                del r3["K"]
                f32[name] = {"value": round(r3["value"], 1), "unit": "pairs/s",
                             "ms_per_step": round(r3["ms_step"], 3),
                             "pairs_per_step": r3["evaluated"]}
                torch.cuda.empty_cache()
            return f32 if rank == 0 else None
        put("f32", legs.run("f32", f32_leg, est_s=20))

    # --- BASELINE configs[3] / [4]: the full-scale ResNet-GP pipelines ---
    def fullscale_leg(config, n, kernel_dtype, data):
        from fullscale import fullscale
        t0 = time.perf_counter()
        fs = fullscale(config, n, args.fullscale_m, 4096, rank=rank, world=world, dev=dev,
                       kernel_dtype=kernel_dtype, stats_group=status)
        if rank != 0:
            return None
        fs["fullscale_wall_s"] = round(time.perf_counter() - t0, 2)
        fs["data"] = data
        return fs

    # expected durations at one GPU, shrinking with the ranks (strong scaling)
    def est(s1):
        return s1 / world + 15
    mnist_data = "synthetic MNIST-like (k/255, 60% zeros, 4-px zero border)"
    if not args.no_fullscale and dtype == torch.float64:
        put("fullscale", legs.run("fullscale", lambda: fullscale_leg(
            "mnist_as_tf", args.fullscale_n, torch.float64, mnist_data), est_s=est(60)))
    if not args.no_fullscale_cifar10 and dtype == torch.float64:
        put("fullscale_cifar10", legs.run("fullscale_cifar10", lambda: fullscale_leg(
            "cifar10", args.cifar10_n, torch.float64,
            "synthetic CIFAR-like 3x32x32 (k/255, 60% zeros, 4-px zero border)"),
            est_s=est(55)))
    if not args.no_fullscale and not args.no_fullscale_f32 and dtype == torch.float64:
        # the same pipeline at the reference pipeline's own kernel precision
        # (save_kernel.py runs the float32 model; K stored float32, widened to float64
        # for the solve by classify_gp.py's load_kern)
        put("fullscale_f32", legs.run("fullscale_f32", lambda: fullscale_leg(
            "mnist_as_tf", args.fullscale_n, torch.float32, mnist_data), est_s=est(35)))

    if rank == 0:
        full["elapsed_s"] = round(deadline.elapsed(), 1)
        try:
            os.makedirs(os.path.dirname(full_path), exist_ok=True)
            with open(full_path, "w") as fh:
                json.dump(full, fh, default=str)
        except OSError as e:
            print(f"bench.py: could not write {full_path}: {e}", file=sys.stderr)
        dog.stop.set()
        emitter.emit(make_line)
    if world > 1:
        try:
            dist.destroy_process_group()
        except Exception:                      # noqa: BLE001 — after a failed leg
            pass
    return 1 if failed else 0


if __name__ == "__main__":
    sys.exit(main())
