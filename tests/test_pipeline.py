"""The row-strip pipeline (cnn_gp.pipeline.classify_distributed, cnn_gp.gram strips) on
CPU: gloo ranks at world size 2 and 3 against the same function in one process, with the
oracle as ``kern`` and scipy's posv (oracle.solve_upper, classify_gp.py:24-26) as the
solve — test infrastructure standing in for the device model and rocSOLVER (the GPU
variant is tests/test_gpu_multi.py).  Reference: exp_mnist_resnet/run.bash:28-43,
classify_gp.py:39-42, 67-77; cnn_gp/data.py:11-19 (the worker split it replaces)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import nngp_oracle as O
from oracle import specs

N, M, B = 37, 13, 8
JITTER = 1e-6


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _data():
    rng = np.random.default_rng(4)
    X = torch.from_numpy(rng.random((N, 1, 28, 28)))
    Z = torch.from_numpy(rng.random((M, 1, 28, 28)))
    labels = torch.from_numpy(rng.integers(0, 10, N))
    Y = -torch.ones((N, 10), dtype=torch.float64)
    Y[torch.arange(N), labels] = 1.0
    return X, Z, Y


def _fns():
    spec = specs.mnist_paper_convnet_gp()

    def kern(x, x2, same):
        return torch.from_numpy(O.kernel(spec, x.numpy(), x2.numpy(), same, False))

    def solve(K, Y):                    # the jitter is the pipeline's (classify_gp.py:66-67)
        return torch.from_numpy(O.solve_upper(K.numpy(), Y.numpy(), 0.0))

    def scores(Kz, A):
        return Kz @ A

    return kern, solve, scores


def _run(world, rank, port, q, gather, dst=0, dtype=torch.float64):
    import sys
    from conftest import PKG, ROOT
    sys.path[:0] = [PKG, ROOT]
    from cnn_gp.pipeline import classify_distributed
    if world > 1:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        X, Z, Y = _data()
        kern, solve, scores = _fns()
        res = classify_distributed(kern, X, Z, Y, solve, scores, batch_size=B, device="cpu",
                                   gather_kxz=gather, dst=dst, dtype=dtype, jitter=JITTER)
        if rank == dst:
            # numpy: pickled by value (a torch tensor on an mp queue travels as a shared
            # memory handle, which dies with this process)
            out = {k: (res[k].numpy() if isinstance(res[k], torch.Tensor) else res[k])
                   for k in ("alpha", "scores", "pred", "K", "plan_kxx", "plan_kxz", "Kxz")}
            if q is None:
                return out
            q.put(out)
        else:
            assert res is None
    finally:
        if world > 1:
            dist.destroy_process_group()


@pytest.mark.parametrize("world,gather,dst", [(2, True, 0), (3, False, 0), (3, True, 0),
                                              (3, True, 2), (8, True, 0)])
def test_gloo_pipeline_matches_single_process(world, gather, dst):
    single = _run(1, 0, None, None, True)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_run, args=(world, r, port, q, gather, dst))
             for r in range(world)]
    for p in procs:
        p.start()
    res = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert len(res["plan_kxx"]) == world
    if world == 8:      # 37 rows on 8-row boundaries: some ranks hold empty strips
        assert any(a == b for a, b in res["plan_kxx"])
    iu = np.triu_indices(N)
    # every upper-triangle entry (what the solve reads) bit-equal; alpha therefore too
    assert np.array_equal(res["K"][iu], single["K"][iu])
    assert np.array_equal(res["alpha"], single["alpha"])
    assert np.array_equal(res["pred"], single["pred"])
    np.testing.assert_allclose(res["scores"], single["scores"], rtol=1e-12, atol=1e-12)
    if gather:
        assert np.array_equal(res["Kxz"], single["Kxz"])
    else:
        assert res["Kxz"] is None
    # against the oracle end to end: Kxx, the posv solve, argmax(Kxz @ A)
    spec = specs.mnist_paper_convnet_gp()
    Kref = O.kernel(spec, _data()[0].numpy())
    # res["K"] is the system the solve saw: Kxx + jitter·I (classify_gp.py:66-67)
    np.testing.assert_allclose(res["K"][iu], (Kref + JITTER * np.eye(N))[iu], rtol=1e-12)
    X, Z, Y = _data()
    A = O.solve_upper(Kref, Y.numpy(), 1e-6)
    Sref = O.kernel(spec, Z.numpy(), X.numpy(), False, False) @ A
    np.testing.assert_allclose(res["scores"], Sref, rtol=1e-6, atol=1e-9)


def test_gloo_pipeline_float32_kernels_widened_in_place():
    """float32 kernels (save_kernel.py's precision) widened to float64 in place on rank 0
    (pipeline.widen_in_place): K and α bit-equal to the one-process run, and K equal to the
    float64 kernel rounded to float32"""
    single = _run(1, 0, None, None, False, 0, torch.float32)
    assert single["K"].dtype == np.float64
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_run, args=(world, r, port, q, True, 1, torch.float32))
             for r in range(world)]
    for p in procs:
        p.start()
    res = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    iu = np.triu_indices(N)
    assert np.array_equal(res["K"][iu], single["K"][iu])
    assert np.array_equal(res["alpha"], single["alpha"])
    Kref = O.kernel(specs.mnist_paper_convnet_gp(), _data()[0].numpy())
    K32 = Kref.astype(np.float32).astype(np.float64)
    K32.flat[::N + 1] += JITTER
    assert np.array_equal(res["K"][iu], K32[iu])
    assert res["Kxz"].dtype == np.float32


@pytest.mark.parametrize("n,n2,tail", [(1, 1, 64), (2, 3, 1), (3, 3, 1), (63, 5, 64),
                                       (64, 64, 1), (65, 7, 64), (1000, 33, 64),
                                       (1000, 1000, 8), (129, 1, 2)])
def test_widen_in_place_equals_a_copy(n, n2, tail):
    """the float32 matrix in the back half of the float64 buffer comes out widened exactly,
    whatever the block sizes, down to one-row blocks"""
    from cnn_gp.pipeline import widen_in_place, widening_matrix
    buf, k32 = widening_matrix(n, n2)
    assert k32.data_ptr() == buf.data_ptr() + 4 * n * n2 and k32.is_contiguous()
    src = torch.randn(n, n2, dtype=torch.float32)
    k32.copy_(src)
    calls = []

    def cast(s, d):
        # every block's source and destination are disjoint byte ranges
        sa, da = s.data_ptr(), d.data_ptr()
        assert sa >= da + 8 * d.numel() or da >= sa + 4 * s.numel()
        calls.append(len(s))
        d.copy_(s)

    out = widen_in_place(buf, k32, cast, tail_rows=tail)
    assert out is buf and torch.equal(buf, src.double())
    assert sum(calls) == n


@pytest.mark.parametrize("n,n2,world", [(60000, None, 8), (10000, 60000, 8), (50000, None, 8),
                                        (60000, None, 2), (4096, None, 3), (37, None, 3),
                                        (13, 37, 3), (5, None, 8), (1, None, 2)])
def test_strip_plan_partitions_and_balances(n, n2, world):
    """contiguous strips cover [0, n); the strips' tiles cover the evaluated entries
    exactly once; at the full-scale sizes the per-rank evaluated pairs stay within 2%"""
    from cnn_gp.gram import strip_cost, strip_plan, strip_tiles, tile_cost, tile_plan
    plan = strip_plan(n, n2, world)
    assert plan[0][0] == 0 and plan[-1][1] == n
    assert all(a[1] == b[0] and a[0] <= a[1] for a, b in zip(plan, plan[1:]))
    costs = [strip_cost(n, n2, r) for r in plan]
    assert sum(costs) == strip_cost(n, n2, (0, n))
    for r in plan:
        assert sum(tile_cost(t) for t in strip_tiles(n, n2, r, 4096)) == strip_cost(n, n2, r)
    if n >= 10000:
        assert max(costs) / min(costs) - 1 <= 0.02, costs
    if n <= 64:                               # exact coverage, entry by entry
        cov = np.zeros((n, n if n2 is None else n2), int)
        for r in plan:
            for same, i0, j0, a, b in strip_tiles(n, n2, r, 4):
                blk = cov[i0:i0 + a, j0:j0 + b]
                if same:
                    blk[np.triu_indices(a, 1)] += 1
                    blk[np.diag_indices(a)] += 1
                else:
                    blk += 1
        want = np.triu(np.ones_like(cov)) if n2 is None else np.ones_like(cov)
        assert np.array_equal(cov, want)
    # one strip over the whole matrix is the reference's tile list
    assert strip_tiles(n, n2, (0, n), 4096) == tile_plan(n, n2, 4096, 0, 1)


def test_kxz_weights_give_the_solving_rank_less():
    from cnn_gp.pipeline import kxz_weights
    assert kxz_weights(1, 60000, 10000, 4e7) is None
    w = kxz_weights(8, 60000, 10000, 4e7, solve_tflops=30)   # solve 2.4 s > 1/7 of 15 s
    assert w[0] == 0.0 and abs(sum(w) - 1) < 1e-12
    w = kxz_weights(2, 60000, 10000, 4e7, solve_tflops=30)
    assert 0 < w[0] < w[1]


def test_strip_plan_weights_zero_share_for_the_solving_rank():
    """rank 0 with weight 0 (its solve outlasts a share of Kxz) gets an empty strip; the
    other ranks split the rows evenly"""
    from cnn_gp.gram import strip_cost, strip_plan, strip_tiles
    w = [0.0] + [1.0] * 7
    plan = strip_plan(10000, 60000, 8, weights=w)
    assert plan[0] == (0, 0) and strip_tiles(10000, 60000, plan[0], 4096) == []
    costs = [strip_cost(10000, 60000, r) for r in plan[1:]]
    assert max(costs) / min(costs) - 1 <= 0.01 and sum(costs) == 10000 * 60000
    # a half share
    plan = strip_plan(10000, 60000, 3, weights=[0.5, 1, 1])
    rows = [b - a for a, b in plan]
    assert abs(rows[0] - 2000) <= 8 and abs(rows[1] - 4000) <= 8


def _run_not_pd(world, rank, port, q):
    import sys
    from conftest import PKG, ROOT
    sys.path[:0] = [PKG, ROOT]
    from cnn_gp.pipeline import classify_distributed
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        X, Z, Y = _data()
        kern, _, scores = _fns()

        def solve(K, Y):                     # an indefinite system, as scipy reports it
            raise np.linalg.LinAlgError("not positive definite")

        try:
            classify_distributed(kern, X, Z, Y, solve, scores, batch_size=B, device="cpu")
            q.put((rank, "no error"))
        except np.linalg.LinAlgError:
            q.put((rank, "LinAlgError"))
        except RuntimeError as e:
            q.put((rank, "RuntimeError" if "solve failed" in str(e) else repr(e)))
    finally:
        dist.destroy_process_group()


def test_gloo_pipeline_failed_solve_raises_on_every_rank():
    """a solve that fails on rank 0 (Kxx not positive definite) must not leave the other
    ranks waiting for α: rank 0 re-raises, the others raise RuntimeError"""
    world = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_run_not_pd, args=(world, r, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert got == {0: "LinAlgError", 1: "RuntimeError", 2: "RuntimeError"}


def _run_guarded(world, rank, port, q, mode, backend="gloo"):
    """one rank of the solve-guard tests: ``mode`` "order" (the solve sleeps, the ranks
    report when their Kxz strips started), "wrong_alpha" (the solve returns a perturbed α),
    "pre_solve_raises" (the hook before the solve raises)"""
    import sys
    import time
    from conftest import PKG, ROOT
    sys.path[:0] = [PKG, ROOT]
    from cnn_gp.pipeline import classify_distributed
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group(backend, rank=rank, world_size=world)
    try:
        X, Z, Y = _data()
        kern0, solve0, scores = _fns()
        first_kxz = []

        def kern(x, x2, same):        # a Kxz tile: its rows are images of Z
            if not first_kxz and len(x) and any(torch.equal(x[0], z) for z in Z):
                first_kxz.append(time.time())
            return kern0(x, x2, same)

        solve_end = []

        def solve(K, Yd):
            a = solve0(K, Yd)
            if mode == "order":
                time.sleep(1.5)
            if mode == "wrong_alpha":      # a wrong factor's α: 1e-6 relative noise
                g = torch.Generator().manual_seed(0)
                a = a * (1 + 1e-6 * torch.randn(a.shape, generator=g, dtype=a.dtype))
            solve_end.append(time.time())
            return a

        def pre_solve(K):
            if mode == "pre_solve_raises":
                raise ValueError("the hook fails")

        try:
            res = classify_distributed(kern, X, Z, Y, solve, scores, batch_size=B,
                                       device="cpu", jitter=JITTER, pre_solve=pre_solve)
            out = ("ok", dist.get_backend(), first_kxz[:1], solve_end,
                   None if res is None else res["co_resident_ranks"],
                   None if res is None else res.get("alpha_backward_error"))
        except np.linalg.LinAlgError as e:
            out = ("LinAlgError", str(e)[:80])
        except RuntimeError as e:
            out = ("RuntimeError" if "solve failed" in str(e) else repr(e),)
        except ValueError as e:
            out = ("ValueError", str(e))
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


def _spawn(world, mode, backend="gloo"):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_run_guarded, args=(world, r, port, q, mode, backend))
             for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return got


def test_gloo_pipeline_co_resident_ranks_wait_for_the_solve():
    """ranks on dst's device (here: three CPU ranks of one host) start their Kxz strips only
    after dst's solve has returned; α is checked (backward error far below the bound)"""
    from cnn_gp.solve import alpha_check_tol
    got = _spawn(3, "order")
    assert all(v[0] == "ok" for v in got.values()), got
    end = got[0][3][0]
    assert got[0][4] == [1, 2]
    started = [got[r][2][0] for r in (1, 2) if got[r][2]]   # 13 rows on 8-row cuts: one
    assert started and min(started) >= end, (started, end)  # rank holds no Kxz rows
    eta = got[0][5]
    assert eta is not None and 0 <= eta < alpha_check_tol(N) / 100


def test_gloo_pipeline_wrong_alpha_raises_on_every_rank():
    """an α that fails the residual check (a factorisation returning info = 0 and a wrong
    factor) is never broadcast: LinAlgError on every rank"""
    got = _spawn(3, "wrong_alpha")
    assert {r: v[0] for r, v in got.items()} == {0: "LinAlgError", 1: "LinAlgError",
                                                 2: "LinAlgError"}, got
    assert "residual check" in got[0][1] and "residual check" in got[1][1]


def test_gloo_pipeline_failing_pre_solve_raises_on_every_rank():
    """an exception in the hook before the solve reaches every rank (no rank is left in
    the status broadcast)"""
    got = _spawn(3, "pre_solve_raises")
    assert got == {0: ("ValueError", "the hook fails"), 1: ("RuntimeError",),
                   2: ("RuntimeError",)}


def test_mixed_backend_group_string():
    """under a mixed group ("cpu:gloo,cuda:gloo" here; "cpu:gloo,cuda:nccl" in bench.py)
    dist.get_backend returns the whole string and the pipeline still runs end to end"""
    got = _spawn(2, "order", backend="cpu:gloo,cuda:gloo")
    assert all(v[0] == "ok" for v in got.values()), got
    assert "gloo" in got[0][1] and "," in got[0][1]


def test_mirror_and_check_alpha():
    """the system mirrored below the diagonal from its upper triangle only (NaN below);
    the check passes scipy's α and rejects the α of a factor wrong in one small block of
    rows (a corrupted trailing-update tile: the residual sits in those rows only)"""
    import scipy.linalg
    from cnn_gp.solve import alpha_backward_error, alpha_check_tol, check_alpha, mirror_upper
    rng = np.random.default_rng(1)
    n = 300
    G = rng.random((n, 16))
    A = G @ G.T / 16 + 0.05 * np.eye(n)
    K = A.copy()
    K[np.tril_indices(n, -1)] = np.nan
    Kt = torch.from_numpy(K)
    d = mirror_upper(Kt)
    assert np.array_equal(Kt.numpy(), A) and np.array_equal(d.numpy(), np.diag(A))
    Y = torch.from_numpy(rng.standard_normal((n, 3)))
    a = scipy.linalg.solve(A, Y.numpy(), assume_a="pos")
    eta = check_alpha(Kt, d, torch.from_numpy(a), Y)
    assert eta < alpha_check_tol(n) / 100
    E = np.zeros_like(A)
    E[200:204, 200:204] = 1e-9 * rng.standard_normal((4, 4))
    bad = scipy.linalg.solve(A + E + E.T, Y.numpy(), assume_a="pos")
    r = A @ bad - Y.numpy()
    assert np.abs(r[:200]).max() < 1e-12 < np.abs(r[200:204]).max()   # a few rows only
    assert alpha_backward_error(Kt, d, torch.from_numpy(bad), Y) > 10 * alpha_check_tol(n)
    with pytest.raises(np.linalg.LinAlgError, match="residual check"):
        check_alpha(Kt, d, torch.from_numpy(bad), Y)
    with pytest.raises(np.linalg.LinAlgError):
        check_alpha(Kt, d, torch.full_like(torch.from_numpy(a), float("nan")), Y)
