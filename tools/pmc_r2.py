"""Summarise the round-2 PMC passes of tools/gpu_pmc_r2.sh into profiles/r2/net_pmc.json.

Per config (net_kernel, one B = 1024 Kxz tile evaluated 3 times): per pair
  hbm_bytes_per_pair = (2·FETCH_SIZE + WRITE_SIZE)·1024 / pairs  (FETCH_SIZE reads half the
      bytes of wide reads on gfx950 — MI355X_MICROARCH.md §HBM; WRITE_SIZE is exact)
  valu_insts_per_pair, valu_active_quadcycles_per_pair (SQ_ACTIVE_INST_VALU, quad-cycles),
  lds / vmem instructions, wave cycles.
Conv stencil (cgp_conv alone, 3 launches): hbm_bytes_per_launch, avg_ms.

    python tools/pmc_r2.py gpurun_out/pmc_r2 [OUT_JSON]
"""
import csv
import glob
import json
import os
import sys

TILE = 1024


def rows(d, match):
    out = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if match(r["Kernel_Name"]):
                out.append(r)
    return out


def totals(d, match):
    tot, disp = {}, {}
    for r in rows(d, match):
        c = r["Counter_Name"]
        tot[c] = tot.get(c, 0.0) + float(r["Counter_Value"])
        disp.setdefault(c, set()).add(r.get("Dispatch_Id", r.get("Correlation_Id", len(disp))))
    return tot, {k: len(v) for k, v in disp.items()}


def kernel_ms(d, match):
    ts = {}
    for r in rows(d, match):
        key = r.get("Dispatch_Id")
        ts[key] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6
    return sum(ts.values()), len(ts)


def main():
    d = sys.argv[1]
    out = sys.argv[2] if len(sys.argv) > 2 else os.path.join(
        os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles", "r2",
        "net_pmc.json")
    res = {}
    evals = 3
    pairs = evals * TILE * TILE
    is_net = lambda k: "net_kernel" in k  # noqa: E731
    for cfgdir in sorted(glob.glob(os.path.join(d, "*_fetch"))):
        cfg = os.path.basename(cfgdir)[:-len("_fetch")]
        if cfg == "stencil":
            continue
        fetch, nf = totals(cfgdir, is_net)
        write, _ = totals(os.path.join(d, cfg + "_write"), is_net)
        sq, nsq = totals(os.path.join(d, cfg + "_sq"), is_net)
        ms, nd = kernel_ms(os.path.join(d, cfg + "_sq"), is_net)
        hbm = (2 * fetch["FETCH_SIZE"] + write["WRITE_SIZE"]) * 1024
        res[cfg] = {
            "dtype": "torch.float64", "tile": TILE, "tile_evaluations": evals,
            "dispatches": nd,
            "hbm_bytes_per_pair": hbm / pairs,
            "fetch_bytes_per_pair": 2 * fetch["FETCH_SIZE"] * 1024 / pairs,
            "write_bytes_per_pair": write["WRITE_SIZE"] * 1024 / pairs,
            "valu_insts_per_pair": sq["SQ_INSTS_VALU"] / pairs,
            "valu_active_quadcycles_per_pair": sq["SQ_ACTIVE_INST_VALU"] / pairs,
            "lds_insts_per_pair": sq["SQ_INSTS_LDS"] / pairs,
            "vmem_insts_per_pair": sq["SQ_INSTS_VMEM"] / pairs,
            "wave_quadcycles_per_pair": sq["SQ_WAVE_CYCLES"] / pairs,
            "wait_any_frac": sq["SQ_WAIT_ANY"] / sq["SQ_WAVE_CYCLES"],
            "wait_inst_any_frac": sq["SQ_WAIT_INST_ANY"] / sq["SQ_WAVE_CYCLES"],
            "active_inst_any_frac": sq["SQ_ACTIVE_INST_ANY"] / sq["SQ_WAVE_CYCLES"],
            "kernel_ms_per_tile_under_pmc": ms / evals,
            "valu_issue_frac_under_pmc": 4 * sq["SQ_ACTIVE_INST_VALU"] /
                                         (1024 * 2.4e9 * ms * 1e-3),
            # GRBM_GUI_ACTIVE: GPU-busy cycles of the dispatches (summed over the XCDs'
            # records); cycles / duration = the engine clock the kernel actually ran at
            "grbm_gui_active": sq.get("GRBM_GUI_ACTIVE"),
            "grbm_records": nsq.get("GRBM_GUI_ACTIVE"),
            "source": f"rocprofv3 --pmc, tools/gpu_pmc_r2.sh on {cfg} (B={TILE} Kxz tile x "
                      f"{evals}); bytes = 2*FETCH_SIZE + WRITE_SIZE (gfx950 correction)",
        }
    is_conv = lambda k: "conv" in k and "net_kernel" not in k  # noqa: E731
    sf = os.path.join(d, "stencil_fetch")
    if os.path.isdir(sf):
        fetch, _ = totals(sf, is_conv)
        write, _ = totals(os.path.join(d, "stencil_write"), is_conv)
        ms, n = kernel_ms(sf, is_conv)
        res["conv_stencil"] = {
            "kernel": "conv7s1@28->28", "maps": TILE * TILE, "launches": n,
            "hbm_bytes_per_launch": (2 * fetch["FETCH_SIZE"] + write["WRITE_SIZE"]) * 1024 / n,
            "avg_ms": ms / n,
            "source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over "
                      "tools/stencil_once.py (cgp_conv on 1024² conv7 maps)"}
    print(json.dumps(res, indent=1))
    os.makedirs(os.path.dirname(out), exist_ok=True)
    json.dump(res, open(out, "w"), indent=1)


if __name__ == "__main__":
    main()
