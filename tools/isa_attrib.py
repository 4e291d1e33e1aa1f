"""Where a compiled net_kernel program's VALU instructions go (verdict r5 item 2): parses
the device assembly of one instantiation (hipcc --cuda-device-only -S of netfuse.hip),
finds its pair loop, and counts the VALU instructions one wave issues per loop iteration
by class — fp64 arithmetic (what the PMC flop counters see), other fp64 (max / min /
ldexp / compares), integer index and address arithmetic, compares and selects, moves,
lane transfers (readfirstlane; readlane / writelane = SGPR spills) — and by op region
(the code between consecutive s_barrier).  The range-adaptive ReLU's polynomial variants
are alternative branches (blocks holding the Horner chains' inline asm): they count once
per vote, at the deepest variant's length over its number of variants (``--poly``).

    python tools/isa_attrib.py [--asm /tmp/netfuse.s] --kernel 'net_kernel<double, false, true, 5, 2, 2>'

Without --asm the source is compiled first (about two minutes).
"""
import argparse
import collections
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CLASSES = [
    ("fp64 arith", re.compile(r"^v_(fma|fmac|mul|add|rsq)_f64")),
    ("fp64 max/min", re.compile(r"^v_(max|min)_f64")),
    ("fp64 ldexp/other", re.compile(r"^v_(ldexp|div_|frexp|trunc|floor|rcp|cvt)\w*f64")),
    ("fp64 compare", re.compile(r"^v_cmp\w*_f64")),
    ("int compare", re.compile(r"^v_cmp")),
    ("select (cndmask)", re.compile(r"^v_cndmask")),
    ("int index/address", re.compile(r"^v_(add|sub|subrev|lshl|lshr|ashr|mul_hi|mul_lo|mad|"
                                      r"and|or|xor|bfe|bfi|alignbit|mul_u32|add3|lshlrev|"
                                      r"lshrrev|ashrrev|not|min_u32|max_u32|min_i32|max_i32|"
                                      r"perm)")),
    ("move", re.compile(r"^v_(mov|accvgpr)")),
    ("readfirstlane", re.compile(r"^v_readfirstlane")),
    ("readlane/writelane (spills)", re.compile(r"^v_(readlane|writelane)")),
    ("other VALU", re.compile(r"^v_")),
]


def classify(op):
    for name, rx in CLASSES:
        if rx.match(op):
            return name
    return None


def function_body(asm_lines, pattern):
    """the assembly lines of the first kernel whose demangled name contains ``pattern``"""
    names = [l.split(":")[0] for l in asm_lines if re.match(r"^_Z\w*:", l)]
    dem = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True,
                         text=True).stdout.split("\n")
    for mangled, d in zip(names, dem):
        if pattern in d.replace("(anonymous namespace)::", ""):
            start = next(i for i, l in enumerate(asm_lines) if l.startswith(mangled + ":"))
            end = next(i for i in range(start, len(asm_lines))
                       if asm_lines[i].startswith(".Lfunc_end"))
            return d, asm_lines[start:end]
    raise SystemExit(f"no kernel matching {pattern!r}")


def blocks(body):
    """[(label, [instruction lines])]: a block starts at a label or a '; %bb.' comment"""
    out, cur, name = [], [], "entry"
    for l in body:
        s = l.strip()
        m = re.match(r"^(\.LBB\w+):", s) or re.match(r"^; %(bb\.\d+):", s)
        if m:
            out.append((name, cur))
            name, cur = m.group(1), []
            continue
        cur.append(l)
    out.append((name, cur))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--asm", default=None)
    ap.add_argument("--kernel", required=True)
    ap.add_argument("--waves-per-pair", type=float, default=1.0,
                    help="loop iterations of one wave per pair (2 for a one-pair half of "
                         "two waves; 2/NP for an NP-pair stage of two waves)")
    args = ap.parse_args()
    path = args.asm
    if path is None:
        path = "/tmp/netfuse_isa.s"
        src = os.path.join(ROOT, "cnn-gp_amd", "csrc")
        subprocess.check_call(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC",
                               "--offload-arch=gfx950", "-ffp-contract=off",
                               "-I" + os.path.join(ROOT, "include"), "-I/opt/rocm/include",
                               "--cuda-device-only", "-S", "netfuse.hip", "-o", path], cwd=src)
    lines = open(path).read().split("\n")
    name, body = function_body(lines, args.kernel)
    bl = blocks(body)
    # the pair loop: the depth-1 loop with the most blocks (labels and "; %bb." comments
    # carry "in Loop: Header=BBx_y" / "Parent Loop BBx_y")
    members = collections.defaultdict(set)
    for l in body:
        s = l.strip()
        m = re.match(r"^(\.LBB\w+):.*=>This (Inner )?Loop Header: Depth=1", s)
        if m:
            members[m.group(1).replace(".L", "")].add(m.group(1))
            continue
        m = re.match(r"^(\.LBB\w+|; %bb\.\d+):?.*(in Loop: Header=|Parent Loop )(BB\w+)", s)
        if m:
            b = m.group(1).replace("; %", "")
            members[m.group(3)].add(b)
    hdr_name, in_loop = max(members.items(), key=lambda kv: len(kv[1]))
    # polynomial variant blocks: Horner chains are inline asm
    totals = collections.Counter()
    regions = [collections.Counter()]
    poly_blocks = 0
    for bname, ins in bl:
        if bname not in in_loop:
            continue
        poly = any("ASMSTART" in l for l in ins)
        if poly:
            poly_blocks += 1
        for l in ins:
            s = l.strip()
            if s.startswith("s_barrier"):
                regions.append(collections.Counter())
                continue
            if not s or s.startswith((";", ".")):
                continue
            op = s.split()[0]
            c = classify(op)
            if c is None:
                continue
            key = ("poly " if poly else "") + c
            totals[key] += 1
            regions[-1][key] += 1
    print(f"{name}: pair loop {len(in_loop)} blocks, {len(regions) - 1} barriers, "
          f"{poly_blocks} polynomial-variant blocks")
    nonpoly = {k: v for k, v in totals.items() if not k.startswith("poly ")}
    poly = {k: v for k, v in totals.items() if k.startswith("poly ")}
    tot_np = sum(nonpoly.values())
    print(f"static VALU per wave-iteration outside the polynomial variants: {tot_np} "
          f"(x {args.waves_per_pair} per pair = {tot_np * args.waves_per_pair:.0f})")
    for k, v in sorted(nonpoly.items(), key=lambda kv: -kv[1]):
        print(f"  {k:30s} {v:6d}  {v * args.waves_per_pair:8.0f} per pair")
    print(f"polynomial variant blocks (static, every variant): {sum(poly.values())}")
    for k, v in sorted(poly.items(), key=lambda kv: -kv[1]):
        print(f"  {k:30s} {v:6d}")
    print("per op region (between barriers), non-fp64 VALU outside the polynomials:")
    for i, r in enumerate(regions):
        n = sum(v for k, v in r.items() if not k.startswith("poly ") and k != "fp64 arith")
        f = r.get("fp64 arith", 0)
        if n or f:
            top = ", ".join(f"{k} {v}" for k, v in r.most_common(4) if not k.startswith("poly"))
            print(f"  region {i:3d}: non-fp64 {n:4d}, fp64 arith {f:4d}   [{top}]")


if __name__ == "__main__":
    main()
