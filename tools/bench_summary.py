"""One-screen summary of the bench.py JSON line in a log (the last line starting with
'{"metric"').

    python tools/bench_summary.py gpurun_out/x/bench.log
"""
import json
import sys


def main(path):
    line = None
    for ln in open(path, errors="replace"):
        if ln.startswith('{"metric"'):
            line = json.loads(ln)
    if line is None:
        print("no bench line in", path)
        return 1
    d = line
    r = d.get("roofline") or {}
    print(f"n_gpus {d['n_gpus']} value {d['value']} ms/step {d['ms_per_step']} "
          f"net {r.get('avg_ms')} frac {r.get('frac')} issue {r.get('valu_issue_frac')}"
          + (f" ERROR {d['error']}" if "error" in d else ""))
    if d.get("ranks"):
        print("  ranks", d["ranks"])
    for k in ("mnist_as_tf", "cifar10"):
        m = d.get(k)
        if m:
            mr = m.get("roofline") or {}
            cpu = m.get("cpu_baseline") or {}
            print(f"  {k}: " + (f"ERROR {m['error']}" if "error" in m else
                                f"value {m['value']} ms/step {m['ms_per_step']} frac "
                                f"{mr.get('frac')} issue {mr.get('valu_issue_frac')} "
                                f"cpu {cpu.get('value')}"))
    s = d.get("solve")
    if s:
        print("  solve", {k: v for k, v in s.items() if k != "note"})
    st = d.get("conv_stencil_roofline")
    if st:
        print("  stencil", {k: st.get(k) for k in ("frac", "avg_ms", "traffic", "error")})
    for k in ("fullscale", "fullscale_f32", "fullscale_cifar10"):
        f = d.get(k)
        if f:
            keys = ("kxx_s", "gather_kxx_s", "solve_s", "kxz_s", "kxz_s_rank0", "total_s",
                    "spot_check_hip_vs_hip_max_rel_err", "error")
            print(f"  {k}", {x: f.get(x) for x in keys if x in f})
            if f.get("solve_split"):
                print("    split", {x: v for x, v in f["solve_split"].items() if x != "note"})
            rk = f.get("ranks")
            if rk:
                print("    ranks", rk)
    di = d.get("dropin")
    if di:
        print("  dropin", di)
    if d.get("watchdog"):
        print("  WATCHDOG", d["watchdog"])
    f32 = d.get("f32")
    if f32:
        print("  f32", {k: (v.get("value") if isinstance(v, dict) else v)
                        for k, v in f32.items() if k != "note"})
    cpu = d.get("cpu_baseline")
    if cpu:
        print("  cpu", cpu.get("value"), cpu.get("cores"), cpu.get("sample"))
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1]))
