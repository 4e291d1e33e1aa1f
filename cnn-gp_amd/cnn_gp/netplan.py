"""Lowering of a compiled program to the whole-network pair kernel (cgp_net_*).

The layer-by-layer pair pipeline (program.Plan.run_pairs) writes every intermediate
[N1·N2, H, W] map to HBM.  ``NetPlan`` instead lowers the SAME SSA program
(program.compile_program) to a list of ``cgp_net_op`` over LDS slots, executed per pair
by one workgroup (csrc/netfuse.hip).  Semantics per op, with the reference lines:

    MOMENTS  v0 = mean_c x_i·y_j                              kernels.py:44-47
    CONV     w·Σ_window + b [→ ReLU] [+ addend]               kernels.py:92-98, 134-165
    RELU     relu(src) [+ addend]                             kernels.py:134-165
    LINEAR   a·src + b·add   (Sum / Mixture terms)           kernels.py:220-254

Fusion uses rules 1-2 of program.fuse (conv→ReLU epilogue, 2-term Sum folded into its
producer); both are exact (IEEE addition commutes).  A ReLU feeding two consumers and the
input moments stay standalone ops: in LDS they cost no extra memory pass.

Slots.  Every value lives in a slot of its spatial class (H, W): a row-major plane whose
rows are separated by max(HL, HR) zero columns (HL / HR: the widest left / right halo any
conv reading that class needs; row r's right halo and row r+1's left halo share the gap),
row stride ws = W + max(HL, HR), with HL zeros before row 0 and HR after the last row.  Halos are zeroed once per workgroup and never
written, so convs read padding as zeros.  Rows need no halo: the conv's row-sum scratch
carries zero rows instead.  Slots are reused as soon as their value is dead, including
in place (dst == src) — safe because every op reads a pixel before the same thread
writes it, and convs consume their whole input into the scratch before writing.
"""
from __future__ import annotations

import ctypes
import dataclasses
from typing import Optional

import torch

from . import _native as N
from .program import fuse

ALIGN = 2                      # slot bases on 16-byte boundaries (fp64 elements)

# Optional launch timing (bench.py): when a list, every launch appends
# (start event, end event, pairs evaluated) recorded on the launch stream.
TIMING = None
MAX_LDS_BYTES = 160 * 1024


class Unsupported(Exception):
    """The program cannot run on the whole-network kernel (layer path instead)."""


@dataclasses.dataclass
class _Slot:
    base: int                  # element offset of the slot
    origin: int                # element offset of pixel (0, 0)
    cls: tuple                 # (H, W)


def _conv_halo(op):
    """(left, right) zero columns the conv reads beyond its input row."""
    g = op.geom
    w = op.shape_in[1]
    wo = op.shape_out[1]
    left = max(0, -g.offset)
    right = max(0, (wo - 1) * g.stride + g.offset + (g.taps - 1) * g.dilation - (w - 1))
    return left, right


def _zero_code(z):
    """cgp_net_op.zero_halo half-word of (HL, gap): 0 = leave the halos alone."""
    if z is None:
        return 0
    hl, gap = z
    assert 0 <= hl < 256 and 0 < gap < 256
    return hl << 8 | gap


class NetPlan:
    """The whole-network kernel program for one Plan (one model at one input size)."""

    def __init__(self, plan, itemsize: int = 8, dual: bool = True):
        self.plan = plan
        prog, v0, vf = plan.prog, plan.v0, plan.vf
        if plan.final_hw != (1, 1):
            raise Unsupported(f"final map is {plan.final_hw}, not 1x1")
        ops = fuse(prog, v0, vf, True, pre_relu=False, fold_moments=False)
        lib = N.load()
        # 1. per-op checks + geometry codes
        hs_need = 2
        codes = {}
        for k, op in enumerate(ops):
            if op.kind == "conv":
                g = op.geom
                if g.dilation != 1:
                    raise Unsupported("dilated conv")
                (h, w), (ho, wo) = op.shape_in, op.shape_out
                code = lib.cgp_net_geometry(h, w, ho, wo, g.taps, g.stride, g.offset)
                if code < 0:
                    raise Unsupported(f"conv geometry {(h, w, ho, wo, g.taps, g.stride, g.offset)}"
                                      " has no fused instantiation")
                codes[k] = code
                hs_need = max(hs_need, lib.cgp_net_hs_elems(code))
            elif op.kind in ("relu", "add"):
                pass
            else:
                raise Unsupported(f"op {op.kind}")
        # 2. slot classes and their halos
        shapes = prog.shapes
        halo = {}
        for v, shp in shapes.items():
            halo.setdefault(tuple(shp), [0, 0])
        for op in ops:
            if op.kind == "conv":
                lft, rgt = _conv_halo(op)
                hl = halo[tuple(op.shape_in)]
                hl[0] = max(hl[0], lft)
                hl[1] = max(hl[1], rgt)
        # rows share their zero gap: row r's right halo and row r+1's left halo are the
        # same max(HL, HR) columns; the slot adds HL before row 0 and HR after the last
        self.ws = {c: c[1] + max(hl) for c, hl in halo.items()}

        def slot_elems(c):
            n = halo[c][0] + c[0] * self.ws[c] + halo[c][1]
            return (n + ALIGN - 1) // ALIGN * ALIGN

        # 3. lower to a linear op list with explicit LINEAR chains
        lowered = [("moments", v0, None)]
        for k, op in enumerate(ops):
            lowered.append(("op", k, op))
        last = {}
        for idx, (kind, a, op) in enumerate(lowered):
            if kind == "op":
                srcs = ([op.src] if op.src is not None else []) + [t for _, t in op.terms]
                if op.addend is not None:
                    srcs.append(op.addend)
                for s in srcs:
                    last[s] = idx
        last[vf] = len(lowered)
        # 4. slot allocation: first fit over one LDS arena after the row-sum scratch, so
        #    dead slots of one class host values of another (a ResNet's 28x28 slots take
        #    its 14x14 and 7x7 values).  A value may take the slot of a source that dies
        #    at its producer when the class matches (in place, same cells); other slots
        #    of dying values are released only after the producer's output is placed.
        slots: dict = {}
        self.hs = 0
        arena0 = (hs_need + ALIGN - 1) // ALIGN * ALIGN
        top = arena0
        free: list = []                       # sorted disjoint [a, b) element intervals
        dying: list = []
        placements: list = []                 # (slot, index of the producer record)

        def take(n):
            nonlocal top
            for k, (lo, hi) in enumerate(free):
                if hi - lo >= n:
                    if hi - lo == n:
                        del free[k]
                    else:
                        free[k] = (lo + n, hi)
                    return lo
            lo = free.pop()[0] if free and free[-1][1] == top else top
            top = max(top, lo + n)
            return lo

        def give(lo, n):
            free.append((lo, lo + n))
            free.sort()
            merged = []
            for iv in free:
                if merged and merged[-1][1] == iv[0]:
                    merged[-1] = (merged[-1][0], iv[1])
                else:
                    merged.append(iv)
            free[:] = merged

        def alloc(v):
            c = tuple(shapes[v])
            for k, dv in enumerate(dying):
                if slots[dv].cls == c:
                    sl = slots[dying.pop(k)]
                    del slots[dv]
                    break
            else:
                base = take(slot_elems(c))
                sl = _Slot(base, base + halo[c][0], c)
                # a fresh region: its halos are what the zeroing pass below checks (a
                # value taking a dying source's slot in place inherits clean halos —
                # nothing else can write inside a live slot)
                placements.append((sl, len(recs)))
            slots[v] = sl
            return sl

        def release_dead(idx):
            for v in [v for v in slots if last.get(v, -1) == idx and v != vf]:
                if v not in dying:
                    dying.append(v)

        def commit():
            for dv in dying:
                sl = slots.pop(dv)
                give(sl.base, slot_elems(sl.cls))
            dying.clear()

        recs = []           # (NetOp fields dict, var value or None)
        for idx, (kind, a, op) in enumerate(lowered):
            commit()
            if kind == "moments":
                h, w = shapes[v0]
                release_dead(idx)
                d = alloc(v0)
                recs.append((dict(kind=N.CGP_NET_MOMENTS, src=0, dst=d.origin, add=-1,
                                  ws_in=self.ws[(h, w)], ws_out=self.ws[(h, w)], h=h, w=w),
                             None))
                continue
            k = a
            if op.kind == "conv":
                s = slots[op.src]
                ad = slots[op.addend].origin if op.addend is not None else -1
                release_dead(idx)
                d = alloc(op.dst)
                ho, wo = op.shape_out
                relu = op.post == N.CGP_POST_RELU
                recs.append((dict(kind=N.CGP_NET_CONV, code=codes[k], src=s.origin,
                                  dst=d.origin, add=ad, ws_in=self.ws[tuple(op.shape_in)],
                                  ws_out=self.ws[(ho, wo)], relu=int(relu), h=ho, w=wo,
                                  weight=op.geom.weight, bias=op.geom.bias,
                                  geom=(*op.shape_in, ho, wo, op.geom.taps, op.geom.stride,
                                        op.geom.offset)),
                             op.post_var if relu else None))
            elif op.kind == "relu":
                s = slots[op.src]
                ad = slots[op.addend].origin if op.addend is not None else -1
                release_dead(idx)
                d = alloc(op.dst)
                h, w = op.shape_out
                recs.append((dict(kind=N.CGP_NET_RELU, src=s.origin, dst=d.origin, add=ad,
                                  ws_in=self.ws[(h, w)], ws_out=self.ws[(h, w)], relu=1,
                                  h=h, w=w), op.src))
            else:   # add: dst = c0·t0 + c1·t1, then dst = dst + c_k·t_k
                terms = [(1.0 if c is None else float(c), t) for c, t in op.terms]
                h, w = op.shape_out
                srcs = [slots[t].origin for _, t in terms]
                if len(terms) > 2:          # chained: dst must not alias a later term
                    d = alloc(op.dst)
                    release_dead(idx)
                else:
                    release_dead(idx)
                    d = alloc(op.dst)
                base = dict(kind=N.CGP_NET_LINEAR, dst=d.origin, ws_in=self.ws[(h, w)],
                            ws_out=self.ws[(h, w)], h=h, w=w)
                if len(terms) == 1:
                    recs.append((dict(base, src=srcs[0], add=srcs[0], weight=terms[0][0],
                                      bias=0.0), None))
                else:
                    recs.append((dict(base, src=srcs[0], add=srcs[1], weight=terms[0][0],
                                      bias=terms[1][0]), None))
                    for (c, _), so in zip(terms[2:], srcs[2:]):
                        recs.append((dict(base, src=d.origin, add=so, weight=1.0, bias=c),
                                     None))
        final_origin = slots[vf].origin
        commit()
        # 4b. slot halos must read as zeros.  A fresh placement finds them dirty when,
        #     since the previous placement of the same slot (cyclically: the program
        #     repeats for every pair of the workgroup), another placement wrote data on
        #     them; such a slot is cleared by a ZERO op before its producer
        cells = {}
        for sl, _ in placements:
            key = (sl.base, sl.cls)
            if key not in cells:
                h_, w_ = sl.cls
                ws_ = self.ws[sl.cls]
                data = {sl.origin + r * ws_ + q for r in range(h_) for q in range(w_)}
                cells[key] = (data, set(range(sl.base, sl.base + slot_elems(sl.cls))) - data)
        zero_at = {}
        npl = len(placements)
        for t, (sl, ri) in enumerate(placements):
            if max(halo[sl.cls]) == 0:
                continue                      # no conv reads beyond this class's data
            key = (sl.base, sl.cls)
            halo_cells = cells[key][1]
            for back in range(1, npl + 1):
                sl2 = placements[(t - back) % npl][0]
                key2 = (sl2.base, sl2.cls)
                if key2 == key:
                    break
                if halo_cells & cells[key2][0]:
                    zero_at.setdefault(ri, []).append(sl)
                    break
        for ri, sls in zero_at.items():
            assert len(sls) == 1
            sl = sls[0]
            recs[ri][0]["zero"] = (halo[sl.cls][0], self.ws[sl.cls] - sl.cls[1])
        self.n_zero = sum(len(v) for v in zero_at.values())
        # 5. dual outputs: a standalone ReLU of the value the previous op just produced
        #    (a residual block's relu(x) branch input) is written by that op's output
        #    stage as a second result, saving an op, a barrier and an LDS round trip
        if dual:
            folded = []
            for f, v in recs:
                prev = folded[-1][0] if folded else None
                if (f["kind"] == N.CGP_NET_RELU and f["add"] < 0 and prev is not None
                        and prev["kind"] in (N.CGP_NET_CONV, N.CGP_NET_LINEAR)
                        and not prev.get("relu") and prev.get("dst2", -1) < 0
                        and prev["dst"] == f["src"] and (prev["h"], prev["w"]) == (f["h"], f["w"])):
                    prev["dst2"] = f["dst"]
                    prev["var2"] = v
                    if "zero" in f:
                        prev["zero2"] = f["zero"]
                    continue
                folded.append((f, v))
            recs = folded
        for f, _ in recs:
            if f["kind"] == N.CGP_NET_RELU:
                f["code"] = lib.cgp_net_resolution(f["h"], f["w"])
            elif f["kind"] != N.CGP_NET_CONV:
                f["code"] = -1
        self.final_slot = final_origin
        self.hs = 0
        self.lds_elems = top
        self.records = recs
        self.dual = any(f.get("dst2", -1) >= 0 for f, _ in recs)
        self.need_var = {v for _, v in recs if v is not None} | {vf} | \
            {f["var2"] for f, _ in recs if "var2" in f}
        self.n_ops = len(recs)
        if self.lds_elems * itemsize > MAX_LDS_BYTES:
            raise Unsupported(f"LDS footprint {self.lds_elems * itemsize} B")

    def lds_bytes(self, itemsize: int) -> int:
        return self.lds_elems * itemsize

    def _ops_array(self, var):
        arr = (N.NetOp * self.n_ops)()
        for k, (f, v) in enumerate(self.records):
            o = arr[k]
            o.kind = f["kind"]
            o.code = f.get("code", 0)
            o.src, o.dst, o.add = f["src"], f["dst"], f["add"]
            o.ws_in, o.ws_out = f["ws_in"], f["ws_out"]
            o.relu = f.get("relu", 0)
            o.h, o.w = f["h"], f["w"]
            o.div_m, o.div_s = N.make_fastdiv(f["w"])
            o.weight, o.bias = f.get("weight", 0.0), f.get("bias", 0.0)
            o.dst2 = f.get("dst2", -1)
            o.zero_halo = _zero_code(f.get("zero")) | (_zero_code(f.get("zero2")) << 16)
            if v is not None:
                vx, vy = var[v]
                o.var_x, o.var_y = vx.data_ptr(), vy.data_ptr()
            if "var2" in f:
                vx, vy = var[f["var2"]]
                o.var2_x, o.var2_y = vx.data_ptr(), vy.data_ptr()
        return arr

    def prepare(self, x, y, var, n1: int, n2: int, same: bool, flags: int = 0,
                out: Optional[torch.Tensor] = None):
        """Upload the op list for these variance maps; return (launch(stream), out).
        ``out`` may be a row-strided view (e.g. a tile of a larger K): the kernel writes
        K[i, j] at out[i * out.stride(0) + j]."""
        sfx = "f64" if x.dtype == torch.float64 else "f32"
        arr = self._ops_array(var)
        host = torch.frombuffer(bytearray(bytes(arr)), dtype=torch.uint8)
        ops_dev = host.to(x.device)                 # stream-ordered, freed stream-ordered
        if out is None:
            out = torch.empty((n1, n2), dtype=x.dtype, device=x.device)
        if out.shape != (n1, n2) or out.stride(1) != 1 or out.dtype != x.dtype:
            raise ValueError("out must be an [n1, n2] row-major view of the input dtype")
        a = N.NetArgs()
        a.x, a.y, a.out = x.data_ptr(), y.data_ptr(), out.data_ptr()
        if same:
            kd = var[self.plan.vf][0]
            a.kdiag = kd.data_ptr()
        a.ops = ops_dev.data_ptr()
        a.n1, a.n2, a.ldo = n1, n2, out.stride(0)
        a.nops, a.channels, a.h, a.w = self.n_ops, x.shape[1], x.shape[2], x.shape[3]
        a.same, a.final_slot, a.hs, a.lds_elems = int(same), self.final_slot, self.hs, \
            self.lds_elems
        a.flags = flags | (N.CGP_FLAG_NET_DUAL if self.dual else 0)
        fn = getattr(N.load(), f"cgp_net_{sfx}")

        pairs = n1 * (n1 - 1) // 2 if same else n1 * n2

        def launch(stream, a=a, ops_dev=ops_dev, fn=fn):
            if TIMING is not None:
                st = torch.cuda.ExternalStream(stream) if stream else torch.cuda.current_stream()
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                e0.record(st)
                N.check(fn(ctypes.byref(a), stream), "cgp_net")
                e1.record(st)
                TIMING.append((e0, e1, pairs))
            else:
                N.check(fn(ctypes.byref(a), stream), "cgp_net")

        return launch, out

    def run(self, x, y, var, n1: int, n2: int, same: bool, stream, flags: int = 0,
            out: Optional[torch.Tensor] = None):
        """K tile [n1, n2] of the pairs (x_i, y_j).  var: value -> (xx [n1,..], yy [n2,..])
        for every value in ``need_var``."""
        launch, out = self.prepare(x, y, var, n1, n2, same, flags, out)
        launch(stream)
        return out
