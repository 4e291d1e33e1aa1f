"""bench.py's multi-GPU launcher and leg isolation, on CPU (no GPU call anywhere here).

* ``--gpus N`` without a torchrun environment starts ``torch.distributed.run`` with N
  ranks as a child (the reference's run.bash:14-36 starts one save_kernel.py process per
  visible GPU); under torchrun ``--gpus`` must equal WORLD_SIZE, and RCCL needs one GPU per
  rank — mismatches exit with status 2 before any GPU work;
* a failing leg records {"error": ...} in its own slot; with several ranks the outcome
  is agreed over a gloo side group, so a failure on one rank reaches rank 0's line and the
  remaining multi-rank legs are skipped on every rank (no collective pairs with another
  leg's)."""
import importlib.util
import os
import socket
import subprocess
import sys

import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_launch_command_runs_one_rank_per_gpu_on_loopback():
    b = _bench()
    argv = ["--gpus", "8", "--steps", "20", "--warmup", "5"]
    cmd = b.launch_cmd(argv, 8, 29512)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    i = cmd.index("--nproc-per-node")
    assert cmd[i + 1] == "8"
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[cmd.index("--master-port") + 1] == "29512"
    assert cmd[cmd.index("--nnodes") + 1] == "1"
    assert cmd[-len(argv) - 1] == os.path.join(ROOT, "bench.py")
    assert cmd[-len(argv):] == argv               # the same arguments reach every rank


def test_world_checks():
    b = _bench()
    assert b.world_error(1, 1, 0, "nccl") is None
    assert b.world_error(8, 8, 8, "nccl") is None
    assert b.world_error(4, 4, 1, "gloo") is None          # gloo rehearsal shares the GPU
    assert "WORLD_SIZE is 3" in b.world_error(2, 3, 8, "nccl")
    assert "needs 8 visible GPUs" in b.world_error(8, 8, 1, "nccl")
    assert "at least one" in b.world_error(0, 0, 1, "nccl")


def _run_bench(args, env_extra):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "CGP_BENCH_BACKEND"):
        env.pop(k, None)
    env.update(env_extra)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args],
                          capture_output=True, text=True, env=env, timeout=300)


def test_refuses_gpus_unequal_world_size():
    p = _run_bench(["--gpus", "2"], {"WORLD_SIZE": "3", "RANK": "0", "LOCAL_RANK": "0"})
    assert p.returncode == 2, p.stderr
    assert "WORLD_SIZE is 3" in p.stderr
    assert p.stdout == ""


def test_refuses_more_rccl_ranks_than_gpus():
    # this container has no GPU: 2 RCCL ranks cannot run, and nothing is launched
    p = _run_bench(["--gpus", "2"], {})
    assert p.returncode == 2, p.stderr
    assert "needs 2 visible GPUs" in p.stderr
    assert "launching" not in p.stderr


def test_single_rank_leg_failure_is_recorded(monkeypatch):
    b = _bench()
    legs = b.Legs()
    monkeypatch.setenv("CGP_BENCH_FAIL_LEG", "second")
    assert legs.run("first", lambda: {"v": 1}) == {"v": 1}
    out = legs.run("second", lambda: {"v": 2})
    assert "forced failure" in out["error"]

    def boom():
        raise MemoryError("out of device memory")
    assert "MemoryError: out of device memory" in legs.run("third", boom)["error"]
    assert legs.run("fourth", lambda: 4) == 4          # one rank: later legs still run


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _leg_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        b = _bench()
        legs = b.Legs(world, rank, dist.new_group(backend="gloo"))
        out = {"a": legs.run("a", lambda: rank)}
        # rank 1 fails before the leg's collective, which rank 0 then waits in until its
        # timeout (3 s here: the bench's collectives time out after CGP_DIST_TIMEOUT_S)
        import datetime
        short = dist.new_group(backend="gloo", timeout=datetime.timedelta(seconds=3))

        def b_leg_short():
            if rank == 1:
                raise RuntimeError("rank 1 fails before the collective")
            dist.barrier(group=short)
            return "b"
        out["b"] = legs.run("b", b_leg_short)
        out["c"] = legs.run("c", lambda: "c")                       # multi-rank: skipped
        out["d"] = legs.run("d", lambda: "d", multi_rank=False)     # rank-local: runs
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


def test_world2_leg_failure_on_one_rank_reaches_every_rank():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_leg_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(world):
        out = got[r]
        assert out["a"] == r
        assert "1" in out["b"]["error"] and "rank 1 fails" in out["b"]["error"]["1"]
        assert "skipped" in out["c"]["error"]
        assert out["d"] == "d"
    assert "0" in got[0]["b"]["error"]          # rank 0's barrier timed out, also recorded


def test_help_lists_every_leg_switch():
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--help"],
                       capture_output=True, text=True, timeout=120)
    assert p.returncode == 0
    for flag in ("--no-cifar10", "--no-fullscale", "--no-fullscale-cifar10", "--gpus"):
        assert flag in p.stdout


def _recorded_full(world=1):
    """A full result in bench.py's format: profiles/r4/bench_r4s_final_box2.json (a
    whole round-4 line, every leg) plus the legs added since, at ``world`` ranks."""
    import copy
    import json
    with open(os.path.join(ROOT, "profiles", "r4", "bench_r4s_final_box2.json")) as f:
        full = json.load(f)
    full = copy.deepcopy(full)
    full["world"] = full["n_gpus"] = world
    case = {"pairs_per_s": 41234567, "s": 0.0508, "tiles": 66, "ms_per_tile": 0.7712,
            "bound_pairs_per_s": 151234567, "over_bound": 0.2727,
            "max_rel_diff_vs_bound": 1.234e-7}
    full["dropin"] = {"n": 2048, "dtype": "f32", "cases": {
        f"{c}/B{b}": dict(case) for c in ("mnist_paper_convnet_gp", "mnist_as_tf")
        for b in (200, 1024)}}
    full["full_result"] = "gpurun_out/bench_full.json"
    if world > 1:
        full["backend"] = "nccl"
        full["ranks"] = [{"rank": r, "tiles": 18, "pairs_per_step": 8386560,
                          "ms_per_step": 80.123 + r} for r in range(world)]
        for leg in ("mnist_as_tf", "cifar10"):
            full[leg]["ranks"] = full["ranks"]
        for leg in ("fullscale", "fullscale_f32", "fullscale_cifar10"):
            full[leg]["ranks"] = [{"rank": r, "kxx_s": 5.123456, "kxx_pairs": 224999999,
                                   "gather_kxx_s": 0.512345, "kxz_s": 1.712345,
                                   "kxz_pairs": 75000000, "kxz_rows": [0, 1250],
                                   "kxx_rows": [0, 2048], "predict_s": 0.001}
                                  for r in range(world)]
            full[leg]["harness_s"] = 0.1701
    return full


def test_line_fits_the_driver_stdout_tail():
    """The driver keeps ~8 KB of the bench's stdout: the printed line (compact_line of the
    full result) stays below 7 000 characters at 1 and 8 ranks and keeps every leg's
    value, roofline and CPU baseline."""
    import json
    b = _bench()
    for world in (1, 8):
        full = _recorded_full(world)
        line = b.compact_line(full)
        s = json.dumps(line)
        assert len(s) < b.LINE_MAX_CHARS == 7000, (world, len(s))
        for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
                  "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config"):
            assert k in line
        for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
            assert k in line["roofline"] and k in line["conv_stencil_roofline"]
            assert k in line["mnist_as_tf"]["roofline"] and k in line["cifar10"]["roofline"]
        for k in ("value", "unit", "cores", "kind", "sample"):
            assert k in line["cpu_baseline"] and k in line["mnist_as_tf"]["cpu_baseline"]
        assert line["conv_stencil_roofline"]["frac"] == full["conv_stencil_roofline"]["frac"]
        assert line["value"] == round(full["value"])
        assert len(line["dropin"]) == 2 + 4
        for leg in ("fullscale", "fullscale_f32", "fullscale_cifar10"):
            assert line[leg]["total_s"] == full[leg]["total_s"]
        if world > 1:
            assert len(line["ranks_ms"]) == world
            assert len(line["fullscale"]["ranks"]["kxx_s"]) == world
        # the stencil and configs[2] come before the full-scale legs (a cut tail keeps them)
        keys = list(line)
        assert keys.index("conv_stencil_roofline") < keys.index("fullscale")
        assert keys.index("mnist_as_tf") < keys.index("fullscale")


def test_line_keeps_leg_errors_short():
    import json
    b = _bench()
    full = _recorded_full(8)
    full["fullscale"] = {"error": {str(r): "RuntimeError: " + "x" * 900 for r in range(8)}}
    full["cifar10"] = {"error": "skipped: budget (430 s used, ~40 s needed, 420 s allowed)"}
    line = b.compact_line(full)
    assert "skipped: budget" in line["cifar10"]["error"]
    assert len(json.dumps(line)) < b.LINE_MAX_CHARS


def test_budget_skips_legs_that_would_start_late():
    b = _bench()
    d = b.Deadline(budget_s=10.0, hard_s=20.0)
    legs = b.Legs(deadline=d)
    assert legs.run("short", lambda: 1, est_s=1) == 1
    out = legs.run("long", lambda: 2, est_s=30)
    assert "skipped: budget" in out["error"]
    d.t0 -= 11                                     # 11 s into the run
    assert "skipped: budget" in legs.run("any", lambda: 3)["error"]


def _hang_worker(rank, world, port, q, hard_s):
    """rank 1 blocks for good inside leg "b"; rank 0 waits for it in the leg's status
    exchange until its watchdog prints the line at the hard limit"""
    import time
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ["CGP_BENCH_HANG_LEG"] = "b:1"
    dist.init_process_group("gloo", rank=rank, world_size=world)
    b = _bench()
    t0 = time.monotonic()
    d = b.Deadline(budget_s=hard_s / 2, hard_s=hard_s)
    legs = b.Legs(world, rank, dist.new_group(backend="gloo"), d)
    full = {"value": 1.0e8, "metric": "m"}
    if rank == 0:
        em = b.Emitter(write=lambda s: q.put(("line", s, time.monotonic() - t0)))
        dog = b.Watchdog(d, em, lambda watchdog=False: b.compact_line(
            dict(full, watchdog=f"leg {legs.current!r}" if watchdog else None)),
            exit_fn=lambda: (q.close(), q.join_thread(), os._exit(3)))
        dog.start()
    full["a"] = legs.run("a", lambda: "a")
    full["b"] = legs.run("b", lambda: "b")        # rank 1 never returns from this leg
    q.put(("end", rank, time.monotonic() - t0))   # not reached by either rank


def test_watchdog_prints_the_line_when_a_rank_hangs():
    import json
    world, hard_s = 2, 8.0
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_hang_worker, args=(r, world, port, q, hard_s))
             for r in range(world)]
    for p in procs:
        p.start()
    try:
        kind, s, t = q.get(timeout=120)
        assert kind == "line"
        line = json.loads(s)
        assert line["value"] == 100000000
        assert "'b'" in line["watchdog"]
        assert t < hard_s + 5, t                  # printed at the hard limit, not later
        procs[0].join(timeout=30)
        assert procs[0].exitcode == 3
    finally:
        for p in procs:
            if p.is_alive():
                p.kill()
            p.join(timeout=30)


def _budget_worker(rank, world, port, q):
    """rank 1 is past the budget, rank 0 is not: both skip the multi-rank leg (they agree
    first, so no collective inside the leg pairs with nothing); rank-local legs follow each
    rank's own clock"""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        b = _bench()
        d = b.Deadline(budget_s=100.0, hard_s=1000.0)
        if rank == 1:
            d.t0 -= 200.0
        legs = b.Legs(world, rank, dist.new_group(backend="gloo"), d)
        out = {"multi": legs.run("multi", lambda: "ran"),
               "local": legs.run("local", lambda: "ran", multi_rank=False)}
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


def test_world2_budget_skip_is_agreed():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_budget_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(world):
        assert "skipped: budget" in got[r]["multi"]["error"]
    assert got[0]["local"] == "ran"
    assert "skipped: budget" in got[1]["local"]["error"]
