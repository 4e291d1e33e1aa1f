"""CPU emulator of the whole-network kernel's op list (test infrastructure only).

Executes ``NetPlan.records`` exactly as csrc/netfuse.hip does — one flat LDS array per
pair, slots at the planned offsets, zero halos, row-sum scratch with zero rows — so the
host lowering (slot classes, halos, in-place reuse, LINEAR chains) is checked against the
oracle without a GPU.  Variances come from a plain numpy run of the same SSA program on
the per-image maps.
"""
from __future__ import annotations

import math

import numpy as np

from oracle import nngp_oracle as O

TINY = O.F32_TINY
HS_CLEAN = 0x100            # cgp_net_op.code flag (include/cnngp.h CGP_NET_CODE_HS_CLEAN)
SUM, FROM_SUM = 0x200, 0x400  # CGP_NET_CODE_SUM / CGP_NET_CODE_FROM_SUM
GEOMETRY = 0xff


def _conv_maps(m, geom, weight, bias):
    """Direct window sums on [n, H, W] maps: w·Σ_window + b with zero padding."""
    h, w, ho, wo, taps, s, off = geom
    n = m.shape[0]
    out = np.zeros((n, ho, wo), m.dtype)
    for r in range(ho):
        for c in range(wo):
            acc = np.zeros(n, m.dtype)
            for a in range(taps):
                rr = r * s + off + a
                if not 0 <= rr < h:
                    continue
                for b in range(taps):
                    cc = c * s + off + b
                    if 0 <= cc < w:
                        acc = acc + m[:, rr, cc]
            out[:, r, c] = weight * acc + bias
    return out


def variances(plan, x, y):
    """value -> (xx [n1,H,W], yy [n2,H,W]) for every value of the program."""
    C = x.shape[1]
    vals = {plan.v0: ((x * x).sum(1) / C, (y * y).sum(1) / C)}
    for op in plan.prog.ops:
        if op.kind == "conv":
            g = op.geom
            geom = (*op.shape_in, *op.shape_out, g.taps, g.stride, g.offset)
            vals[op.dst] = tuple(_conv_maps(m, geom, g.weight, g.bias) for m in vals[op.src])
        elif op.kind == "relu":
            vals[op.dst] = tuple(m / 2 for m in vals[op.src])
        else:
            acc = None
            for coef, t in op.terms:
                a = vals[t] if coef is None else tuple(m * coef for m in vals[t])
                acc = a if acc is None else (acc[0] + a[0], acc[1] + a[1])
            vals[op.dst] = acc
    return vals


def _relu(c, v1, v2):
    with np.errstate(invalid="ignore", divide="ignore"):
        t = v1 * v2 + TINY
        cos = np.clip(c * (1.0 / np.sqrt(t)), -1.0, 1.0)
        sin = np.sqrt(np.maximum(t - c * c, 0.0))
        return (sin + (math.pi - np.arccos(cos)) * c) / (2 * math.pi)


def validate(stage):
    """The CGP_NET_CODE_SUM / FROM_SUM preconditions of include/cnngp.h (the library's
    cgp_net_validate): ValueError for an op list the kernel would run into zeroed partial
    sums."""
    recs = [f for f, _ in stage.records]
    for k, f in enumerate(recs):
        code = f.get("code", 0)
        if f["kind"] != 0 or code < 0:       # the flags are conv codes (LOAD / STORE use
            continue                         # their code field for the record size)
        h, w, ho, wo, taps, s, off = f["geom"]
        point = taps == 1 and off == 0
        reduce = ho == wo == 1 and off == 0 and taps == h == w
        if code & SUM:
            if taps <= 3 or point or reduce:
                raise ValueError(f"op {k}: SUM needs a separable conv")
            if f["add"] >= 0 or f.get("dst2", -1) >= 0:
                raise ValueError(f"op {k}: SUM with an addend or a second output")
            if stage.pairs > 2:
                raise ValueError(f"op {k}: SUM in a {stage.pairs}-pair stage")
            nxt = recs[k + 1] if k + 1 < len(recs) else None
            if nxt is None or nxt["kind"] != 0 or not nxt.get("code", 0) & FROM_SUM or \
                    nxt["src"] != f["dst"]:
                raise ValueError(f"op {k}: SUM not followed by the FROM_SUM reduction of its map")
            if any(g["src"] == f["dst"] or g["add"] == f["dst"] for g in recs[k + 2:]):
                raise ValueError(f"op {k}: a later op reads the never-stored SUM map")
        if code & FROM_SUM:
            if not reduce or stage.pairs > 2:
                raise ValueError(f"op {k}: FROM_SUM needs a one-pair full-map reduction")
            prev = recs[k - 1] if k else None
            if prev is None or prev["kind"] != 0 or prev.get("code", 0) < 0 or \
                    not prev["code"] & SUM:
                raise ValueError(f"op {k}: FROM_SUM without a SUM conv before it")


def run_stage(stage, x_i, y_j, var, i, j, lds, state):
    """One pair through one stage's op list.  ``lds`` (this pair's arena) persists
    across the pairs a workgroup walks (the kernel zeroes it once per workgroup), so
    stale values of earlier pairs stay in every cell an op does not write — as on the
    device.  ``state``: {"in": record, "out": record} of this pair's unit."""
    validate(stage)
    hs0 = 0
    fused = None               # the map sum a CGP_NET_CODE_SUM conv hands the next reduction

    def plane(off, h, w, ws):
        idx = off + np.arange(h)[:, None] * ws + np.arange(w)[None, :]
        return idx

    for f, v in stage.records:
        kind = f["kind"]
        for key, dst in (("zero", f["dst"]), ("zero2", f.get("dst2", -1))):
            if key in f:                                        # cgp_net_op.zero_halo
                hl, gap = f[key]
                lds[dst - hl:dst] = 0.0
                for r in range(f["h"]):
                    c0 = dst + r * f["ws_out"] + f["w"]
                    lds[c0:c0 + gap] = 0.0
        if kind == 4:                                           # LOAD
            h, w = f["h"], f["w"]
            lds[plane(f["dst"], h, w, f["ws_out"])] = \
                state["in"][f["add"]:f["add"] + h * w].reshape(h, w)
        elif kind == 5:                                         # STORE
            h, w = f["h"], f["w"]
            state["out"][f["add"]:f["add"] + h * w] = \
                lds[plane(f["src"], h, w, f["ws_in"])].reshape(-1)
        elif kind == 2:                                         # MOMENTS
            h, w = f["h"], f["w"]
            C = x_i.shape[0]
            lds[plane(f["dst"], h, w, f["ws_out"])] = (x_i * y_j).sum(0) / C
        elif kind == 0:                                         # CONV
            h, w, ho, wo, taps, s, off = f["geom"]
            src = lds[plane(f["src"], h, w, f["ws_in"])]
            point = taps == 1 and off == 0
            reduce = ho == wo == 1 and off == 0 and taps == h == w
            separable = not point and not reduce and taps > 3
            hsr = (ho - 1) * s + taps
            if separable:
                # the row pass writes its input rows into the arena's first cells (the
                # kernel's row-sum scratch); rows outside the input are zero rows, rewritten
                # unless the host marked them clean (cgp_net_op.code & HS_CLEAN) — stale
                # data there would reach the column pass, as on the device
                q0, q1 = max(0, -off), min(hsr, h - off)
                for q in range(q0, q1):
                    r = q + off
                    for c in range(wo):
                        base = f["src"] + r * f["ws_in"] + c * s + off
                        lds[hs0 + q * wo + c] = lds[base:base + taps].sum()
                if not f["code"] & HS_CLEAN:
                    lds[hs0:hs0 + q0 * wo] = 0.0
                    lds[hs0 + q1 * wo:hs0 + hsr * wo] = 0.0
                hs = lds[hs0:hs0 + hsr * wo].reshape(hsr, wo).copy()
            else:
                # row pass over the planned slot (reads the halo columns from `lds`)
                hs = np.zeros((hsr, wo))
                for q in range(hsr):
                    r = q + off
                    if not 0 <= r < h:
                        continue
                    for c in range(wo):
                        base = f["src"] + r * f["ws_in"] + c * s + off
                        hs[q, c] = lds[base:base + taps].sum()
            out = np.zeros((ho, wo))
            for r in range(ho):
                out[r] = hs[r * s:r * s + taps].sum(0)
            if f["code"] & FROM_SUM:
                # the previous conv's outputs were never stored: its sums stand for the map
                assert reduce and fused is not None
                out = np.full((1, 1), fused)
            out = f["weight"] * out + f["bias"]
            if reduce and stage.pairs <= 2 and not f["code"] & FROM_SUM:
                # a one-pair reduction leaves its two wave partial sums at cgp_net_args.part
                flat = src.reshape(-1)
                lds[stage.part] = flat[np.arange(flat.size) % 128 < 64].sum() + 1.0
                lds[stage.part + 1] = flat[np.arange(flat.size) % 128 >= 64].sum() + 1.0
            if f.get("relu"):
                vx, vy = var[v]
                out = _relu(out, vx[i], vy[j])
            if f["code"] & SUM:                                 # kept in registers
                assert f["add"] < 0 and f.get("dst2", -1) < 0
                fused = out.sum()
                continue
            if f["add"] >= 0:
                out = out + lds[plane(f["add"], ho, wo, f["ws_out"])]
            lds[plane(f["dst"], ho, wo, f["ws_out"])] = out
            if f.get("dst2", -1) >= 0:
                vx, vy = var[f["var2"]]
                lds[plane(f["dst2"], ho, wo, f["ws_out"])] = _relu(out, vx[i], vy[j])
        elif kind == 1:                                         # RELU
            h, w = f["h"], f["w"]
            vx, vy = var[v]
            out = _relu(lds[plane(f["src"], h, w, f["ws_in"])], vx[i], vy[j])
            if f["add"] >= 0:
                out = out + lds[plane(f["add"], h, w, f["ws_out"])]
            lds[plane(f["dst"], h, w, f["ws_out"])] = out
        else:                                                   # LINEAR
            h, w = f["h"], f["w"]
            out = f["weight"] * lds[plane(f["src"], h, w, f["ws_in"])] + \
                f["bias"] * lds[plane(f["add"], h, w, f["ws_out"])]
            lds[plane(f["dst"], h, w, f["ws_out"])] = out
            if f.get("dst2", -1) >= 0:
                vx, vy = var[f["var2"]]
                lds[plane(f["dst2"], h, w, f["ws_out"])] = _relu(out, vx[i], vy[j])
    return lds[stage.final_slot]


def kernel(net, x, y, same):
    """K through every stage.  One workgroup walks all pairs; a stage with P pairs per
    workgroup gives pair n the arena n % P (each arena keeps its stale cells)."""
    var = variances(net.plan, x, y)
    n1, n2 = x.shape[0], y.shape[0]
    K = np.zeros((n1, n2))
    arenas = [[np.zeros(st.lds_elems) for _ in range(st.pairs)] for st in net.stages]
    n = 0
    for i in range(n1):
        for j in range(n2):
            if same and i == j:
                K[i, i] = var[net.plan.vf][0][i].item()
            elif same and j < i:
                K[i, j] = K[j, i]
            else:
                rec = None
                for s, st in enumerate(net.stages):
                    state = {"in": rec, "out": np.zeros(st.store_stride)}
                    v = run_stage(st, x[i], y[j], var, i, j, arenas[s][n % st.pairs], state)
                    rec = state["out"]
                K[i, j] = v
                n += 1
    return K
