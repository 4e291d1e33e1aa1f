"""Rehearse bench.py's process-group layout under torchrun on the box: the default group
"cpu:gloo,cuda:nccl" (host tensors on gloo, device tensors on RCCL, its communicator
created at the first device collective) plus a gloo side group.  Checks the gloo-only
control plane the Kxx legs use (barrier, max all-reduce on host tensors, object gather),
then the device collectives the full-scale pipeline uses (all-reduce, broadcast).

    python -m torch.distributed.run --nproc-per-node 1 --master-addr 127.0.0.1 \\
        tools/dist_probe.py
"""
import datetime
import os
import sys
import time

import torch
import torch.distributed as dist


def main():
    rank = int(os.environ["RANK"])
    world = int(os.environ["WORLD_SIZE"])
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local % max(1, torch.cuda.device_count()))
    tmo = datetime.timedelta(seconds=float(os.environ.get("CGP_DIST_TIMEOUT_S", "60")))
    t0 = time.perf_counter()
    dist.init_process_group("cpu:gloo,cuda:nccl", timeout=tmo)
    side = dist.new_group(backend="gloo", timeout=tmo)
    out = {"backend": dist.get_backend(), "init_s": round(time.perf_counter() - t0, 3)}
    dist.barrier(group=side)
    el = torch.tensor([float(rank + 1)], dtype=torch.float64)
    dist.all_reduce(el, op=dist.ReduceOp.MAX, group=side)
    out["gloo_max"] = float(el)
    el2 = torch.tensor([float(rank + 1)], dtype=torch.float64)
    dist.all_reduce(el2, op=dist.ReduceOp.MAX)          # default group, host tensor: gloo
    out["default_host_max"] = float(el2)
    objs = [None] * world
    dist.all_gather_object(objs, {"rank": rank}, group=side)
    out["gathered"] = len(objs)
    t1 = time.perf_counter()
    d = torch.full((4,), float(rank + 1), device="cuda")
    dist.all_reduce(d, op=dist.ReduceOp.MAX)            # device tensor: RCCL (lazy comm)
    b = torch.arange(3, dtype=torch.float64, device="cuda") * (rank + 1)
    dist.broadcast(b, 0)
    torch.cuda.synchronize()
    out["rccl_max"] = float(d[0])
    out["rccl_bcast"] = b.tolist()
    out["rccl_first_collective_s"] = round(time.perf_counter() - t1, 3)
    print(rank, out, flush=True)
    dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
