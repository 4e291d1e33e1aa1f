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
