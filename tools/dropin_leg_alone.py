"""bench.py's dropin leg alone in a fresh process (diagnostic).

    DL_TILES=200,1024 DL_CFG=mnist_paper_convnet_gp [DL_POISON=1] python tools/dropin_leg_alone.py

DL_POISON=1 copies a 64 MB device buffer back to pageable host memory first (what the
leg's comparison did between cases before round 6: it made the next case's H2D copies
stall behind other threads' kernels).  CGP_DROPIN_TRACE=1 adds per-call phase times."""
import os
import sys

sys.argv = ["bench.py"]
sys.path.insert(0, os.getcwd())
import bench  # noqa: E402
import torch  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
if os.environ.get("DL_POISON"):
    torch.empty(16 << 20, dtype=torch.float32, device=dev).fill_(1.0).cpu().numpy().sum()
r = bench.dropin_leg((os.environ.get("DL_CFG", "mnist_paper_convnet_gp"),), 4096,
                     tuple(int(t) for t in os.environ.get("DL_TILES", "200,1024").split(",")),
                     dev)
for k, v in r["cases"].items():
    print(k, v["s"], v["s_range"], v["ms_per_tile"], v["over_bound"],
          v.get("trace_ms_h2d_fwd_d2h"), v["max_rel_diff_vs_bound"])
