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

import collections
import ctypes
import dataclasses
import os
import threading
from typing import Optional

import torch

from . import _native as N
from .program import fuse

ALIGN = 2                      # slot bases on 16-byte boundaries (fp64 elements)

# Optional launch timing (bench.py): when a list, every launch appends
# (start event, end event, pairs evaluated) recorded on the launch stream.
TIMING = None

# Run the library's compiled program for an op list when it holds one (cgp_net_program:
# the reference configs' lowered programs, every offset an immediate).  False forces the
# op-record interpreter (A/B and parity tests of both paths).
USE_PROGRAMS = os.environ.get("CGP_NET_PROGRAMS", "1") != "0"
# a separable conv whose map only the next op's full-map reduction reads keeps its outputs
# in registers and hands the reduction its wave partial sums (cnngp.h CGP_NET_CODE_SUM /
# CGP_NET_CODE_FROM_SUM; one pair per workgroup or half): no map store, no map re-read,
# one barrier less per pair.  CGP_NET_FUSE_REDUCE=0 keeps the two ops apart.
FUSE_REDUCE = os.environ.get("CGP_NET_FUSE_REDUCE", "1") != "0"
MAX_LDS_BYTES = 160 * 1024
# state buffers below this size are allocated without asking for the free memory
SMALL_STATE_BYTES = 512 << 20
# Tile recipes (TileRecipe): a forward's launch sequence kept per (tile shape, stream)
# while its persistent buffers (variance maps, stage states) take at most RECIPE_MAX_BYTES,
# at most RECIPE_SLOTS recipes and RECIPE_TOTAL_BYTES per NetPlan (least recently used
# dropped first: save_K's helper threads each hold the 4-5 tile shapes of a build on
# their own stream).  RECIPE_MAX_BYTES = 0 turns them off.
RECIPE_MAX_BYTES = int(os.environ.get("CGP_RECIPE_MAX_MB", "512")) << 20
RECIPE_SLOTS = 32
RECIPE_TOTAL_BYTES = 4 << 30


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


@dataclasses.dataclass
class Stage:
    """One launch of the whole-network kernel: a contiguous run of the lowered program
    with its own LDS arena (per pair) and pairs per workgroup."""
    records: list
    lds_elems: int
    final_slot: int
    pairs: int
    final: bool
    load_stride: int                   # elements per unit of the incoming state record
    store_stride: int                  # ... of the outgoing one
    part: int = 0                      # LDS cell of a one-pair reduction's partial sums

    @property
    def n_ops(self):
        return len(self.records)

    @property
    def dual(self):
        return any(f.get("dst2", -1) >= 0 for f, _ in self.records)


# pairs per workgroup of a stage whose maps are all at most this many pixels
MULTI_PAIR = ((16, 64), (4, 256))
# pairs per workgroup of the first stage (the full-size maps): 2 runs two one-pair halves
# in one four-wave workgroup (csrc/netfuse.hip net_kernel, NP == 2: units u and u + 1, the
# same image i), 1 one pair on two waves.  Measured on the MI355X (one B = 1024 Kxz tile):
# ConvNet GP +13%, mnist_as_tf / cifar10 +1%, Residual CNN GP even.  CGP_NET_PAIRS0=1
# selects one pair per workgroup.
FIRST_PAIRS = os.environ.get("CGP_NET_PAIRS0", "2")


def first_pairs(n_stages: int) -> int:
    """Pairs per workgroup of the first of n_stages stages."""
    del n_stages
    return 2 if FIRST_PAIRS in ("2", "auto") else 1
MIN_STAGE_OPS = 4                      # a shorter tail is not worth a launch + state
# state buffers: units per launch group (each group runs every stage once, and each launch
# ends in a tail where the last workgroups finish their pairs).  The cap is also clamped
# so that all of a tile's state buffers take at most STATE_FREE_FRAC of the device's free
# memory (NetPlan.chunk_units)
CHUNK_BYTES = int(os.environ.get("CGP_NET_CHUNK_MB", "8192")) << 20
STATE_FREE_FRAC = 0.25


class NetPlan:
    """The whole-network kernel program for one Plan (one model at one input size).

    The program is lowered to one or more stages.  A network whose tail runs on small
    maps (a ResNet's 14x14 and 7x7 blocks) is split where the maps drop to <= 16x16 and
    <= 8x8: those stages run 4 and 16 pairs per workgroup (csrc/netfuse.hip), so a small
    map's op still fills the workgroup's 128 threads.  The maps live across a boundary
    cross it through a per-unit state buffer (CGP_NET_STORE / CGP_NET_LOAD)."""

    def __init__(self, plan, itemsize: int = 8, dual: bool = True, stages: bool = True):
        self.plan = plan
        prog, v0, vf = plan.prog, plan.v0, plan.vf
        if plan.final_hw != (1, 1):
            raise Unsupported(f"final map is {plan.final_hw}, not 1x1")
        ops = fuse(prog, v0, vf, True, pre_relu=False, fold_moments=False)
        lib = N.load()
        self._lib = lib
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
        self._codes = codes
        # 2. slot classes and their halos
        shapes = prog.shapes
        self._shapes = shapes
        halo = {}
        for v, shp in shapes.items():
            halo.setdefault(tuple(shp), [0, 0])
        for op in ops:
            if op.kind == "conv":
                lft, rgt = _conv_halo(op)
                hl = halo[tuple(op.shape_in)]
                hl[0] = max(hl[0], lft)
                hl[1] = max(hl[1], rgt)
        self._halo = halo
        # rows share their zero gap: row r's right halo and row r+1's left halo are the
        # same max(HL, HR) columns; the slot adds HL before row 0 and HR after the last
        self.ws = {c: c[1] + max(hl) for c, hl in halo.items()}
        # 3. a linear op list: the moments, then the fused ops
        lowered = [("moments", v0, None)]
        for k, op in enumerate(ops):
            lowered.append(("op", k, op))
        last = {}
        prod = {v0: 0}
        for idx, (kind, a, op) in enumerate(lowered):
            if kind == "op":
                prod[op.dst] = idx
                for s_ in self._sources(op):
                    last[s_] = idx
        last[vf] = len(lowered)
        # 4. stages, then each stage's slots and records
        multi = stages and not plan.flags & N.CGP_FLAG_EXACT_RELU
        bounds = self._stage_bounds(lowered, multi)
        self.stages = []
        for sidx, (lo, hi, np_) in enumerate(bounds):
            ins = sorted(v for v, pi in prod.items() if pi < lo and last.get(v, -1) >= lo)
            outs = sorted(v for v, pi in prod.items() if pi < hi <= last.get(v, -1)) \
                if hi < len(lowered) else []
            st = self._lower(lowered, lo, hi, np_, ins, outs, last, dual, itemsize)
            # the two-pair workgroup holds cgp_net_units(2) one-pair arenas
            if np_ == 2 and st.lds_elems * itemsize * lib.cgp_net_units(2) > \
                    MAX_LDS_BYTES - lib.cgp_net_static_lds():
                st = self._lower(lowered, lo, hi, 1, ins, outs, last, dual, itemsize)
            self.stages.append(st)
        self.need_var = {vf}
        for st in self.stages:
            self.need_var |= {v for _, v in st.records if v is not None}
            self.need_var |= {f["var2"] for f, _ in st.records if "var2" in f}

    # -- compatibility view of a one-stage program -----------------------------------------
    @property
    def records(self):
        return [r for st in self.stages for r in st.records]

    @property
    def lds_elems(self):
        return max(st.lds_elems * st.pairs for st in self.stages)

    @property
    def final_slot(self):
        return self.stages[-1].final_slot

    @property
    def dual(self):
        return any(st.dual for st in self.stages)

    @property
    def n_ops(self):
        return sum(st.n_ops for st in self.stages)

    hs = 0

    @staticmethod
    def _sources(op):
        srcs = ([op.src] if op.src is not None else []) + [t for _, t in op.terms]
        if op.addend is not None:
            srcs.append(op.addend)
        return srcs

    def _stage_bounds(self, lowered, multi):
        """[(lo, hi, pairs)]: one stage, or the network split where every later op's maps
        fit 4 / 16 pairs per workgroup (compile-time sizes only)."""
        n = len(lowered)
        if not multi:
            return [(0, n, 1)]
        lib, shapes = self._lib, self._shapes
        inf = 1 << 30

        def px(idx):
            kind, _, op = lowered[idx]
            if kind == "moments":
                return inf
            vals = [op.dst] + self._sources(op)
            if op.kind in ("relu", "add"):
                h, w = shapes[op.dst]
                if lib.cgp_net_resolution(h, w) < 0:
                    return inf
            return max(shapes[v][0] * shapes[v][1] for v in vals)

        smax = [0] * (n + 1)
        for idx in range(n - 1, -1, -1):
            smax[idx] = max(px(idx), smax[idx + 1])
        cuts = []
        for pairs, lim in MULTI_PAIR:
            k = next((idx for idx in range(1, n) if smax[idx] <= lim), n)
            cuts.append((k, pairs))
        k16, k4 = cuts[0][0], cuts[1][0]
        bounds = []
        edges = [(0, 1)]
        if k4 < k16:
            edges.append((k4, 4))
        if k16 < n:
            edges.append((k16, 16))
        # a multi-pair stage shorter than MIN_STAGE_OPS stays with its predecessor
        kept = [edges[0]]
        for k, pairs in edges[1:]:
            nxt = next((k2 for k2, _ in edges if k2 > k), n)
            if nxt - k >= MIN_STAGE_OPS:
                kept.append((k, pairs))
        for t, (k, pairs) in enumerate(kept):
            hi = kept[t + 1][0] if t + 1 < len(kept) else n
            bounds.append((k, hi, pairs))
        # the first stage on 2 pairs: two one-pair halves of one workgroup (any op list;
        # __init__ falls back to 1 when twice the arena does not fit the LDS)
        lo0, hi0, _ = bounds[0]
        if first_pairs(len(bounds)) == 2:
            bounds[0] = (lo0, hi0, 2)
        return bounds

    def _lower(self, lowered, lo, hi, pairs, ins, outs, last, dual, itemsize):
        """Slots and records of lowered[lo:hi] (inputs loaded from the incoming state
        record, outputs stored to the outgoing one)."""
        lib, shapes, halo = self._lib, self._shapes, self._halo
        plan = self.plan
        v0, vf = plan.v0, plan.vf
        final = hi == len(lowered)

        def slot_elems(c):
            n = halo[c][0] + c[0] * self.ws[c] + halo[c][1]
            return (n + ALIGN - 1) // ALIGN * ALIGN

        # last use inside this stage: an output is read by its STORE at index hi
        last_s = {v: (hi if v in outs else min(u, hi)) for v, u in last.items()}
        # slot allocation: first fit over one LDS arena after the row-sum scratch, so
        # dead slots of one class host values of another (a ResNet's 28x28 slots take its
        # 14x14 and 7x7 values).  A value may take the slot of a source that dies at its
        # producer when the class matches (in place, same cells); other slots of dying
        # values are released only after the producer's output is placed.
        slots: dict = {}
        hs_need = 2                           # the row-sum scratch this stage's convs need
        for idx in range(lo, hi):
            kind, a, op = lowered[idx]
            if kind == "op" and op.kind == "conv":
                hs_need = max(hs_need, lib.cgp_net_hs_elems(self._codes[a]))
        arena0 = (hs_need + ALIGN - 1) // ALIGN * ALIGN
        top = arena0
        free: list = []                       # sorted disjoint [a, b) element intervals
        dying: list = []
        placements: list = []                 # (slot, index of the producer record)
        recs = []                             # (NetOp fields dict, var value or None)

        def take(n):
            nonlocal top
            for k, (a_, b_) in enumerate(free):
                if b_ - a_ >= n:
                    if b_ - a_ == n:
                        del free[k]
                    else:
                        free[k] = (a_ + n, b_)
                    return a_
            a_ = free.pop()[0] if free and free[-1][1] == top else top
            top = max(top, a_ + n)
            return a_

        def give(a_, n):
            free.append((a_, a_ + n))
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
            for v in [v for v in slots if last_s.get(v, -1) == idx and v != vf]:
                if v not in dying:
                    dying.append(v)

        def commit():
            for dv in dying:
                sl = slots.pop(dv)
                give(sl.base, slot_elems(sl.cls))
            dying.clear()

        # stage inputs
        load_stride = sum(shapes[v][0] * shapes[v][1] for v in ins)
        off = 0
        for v in ins:
            h, w = shapes[v]
            d = alloc(v)
            recs.append((dict(kind=N.CGP_NET_LOAD, src=0, dst=d.origin, add=off,
                              ws_in=self.ws[(h, w)], ws_out=self.ws[(h, w)], h=h, w=w,
                              code=load_stride, state="in"), None))
            off += h * w
        for idx in range(lo, hi):
            kind, a, op = lowered[idx]
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
                s_ = slots[op.src]
                ad = slots[op.addend].origin if op.addend is not None else -1
                release_dead(idx)
                d = alloc(op.dst)
                ho, wo = op.shape_out
                relu = op.post == N.CGP_POST_RELU
                recs.append((dict(kind=N.CGP_NET_CONV, code=self._codes[k], src=s_.origin,
                                  dst=d.origin, add=ad, ws_in=self.ws[tuple(op.shape_in)],
                                  ws_out=self.ws[(ho, wo)], relu=int(relu), h=ho, w=wo,
                                  weight=op.geom.weight, bias=op.geom.bias,
                                  geom=(*op.shape_in, ho, wo, op.geom.taps, op.geom.stride,
                                        op.geom.offset)),
                             op.post_var if relu else None))
            elif op.kind == "relu":
                s_ = slots[op.src]
                ad = slots[op.addend].origin if op.addend is not None else -1
                release_dead(idx)
                d = alloc(op.dst)
                h, w = op.shape_out
                recs.append((dict(kind=N.CGP_NET_RELU, src=s_.origin, dst=d.origin, add=ad,
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
        commit()
        # stage outputs
        store_stride = sum(shapes[v][0] * shapes[v][1] for v in outs)
        off = 0
        for v in outs:
            h, w = shapes[v]
            recs.append((dict(kind=N.CGP_NET_STORE, src=slots[v].origin, dst=0, add=off,
                              ws_in=self.ws[(h, w)], ws_out=self.ws[(h, w)], h=h, w=w,
                              code=store_stride, state="out"), None))
            off += h * w
        final_origin = slots[vf].origin if final else 0
        # halo zeroing: slot halos must read as zeros.  A fresh placement finds them dirty
        # when, since the previous placement of the same slot (cyclically: the stage's
        # ops repeat for every pair of the workgroup), another placement wrote data on
        # them; its producer then zeroes the halo cells first
        cells = {}
        for sl, _ in placements:
            key = (sl.base, sl.cls)
            if key not in cells:
                h_, w_ = sl.cls
                ws_ = self.ws[sl.cls]
                data = {sl.origin + r * ws_ + q for r in range(h_) for q in range(w_)}
                cells[key] = (data, set(range(sl.base, sl.base + slot_elems(sl.cls))) - data)
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
                    recs[ri][0]["zero"] = (halo[sl.cls][0], self.ws[sl.cls] - sl.cls[1])
                    break
        # dual outputs: a standalone ReLU of the value the previous op just produced (a
        # residual block's relu(x) branch input) is written by that op's output stage as
        # a second result, saving an op, a barrier and an LDS round trip
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
        hs_part = self._reduce_cells(recs)
        self._mark_hs_clean(recs, pairs, hs_part)
        self._fuse_reductions(recs, pairs)
        for f, _ in recs:
            # (a two-pair stage runs its ops as one-pair halves: lowered like one pair)
            if f["kind"] == N.CGP_NET_RELU or (f["kind"] == N.CGP_NET_LINEAR and pairs > 2):
                f["code"] = lib.cgp_net_resolution(f["h"], f["w"])
            elif f["kind"] in (N.CGP_NET_MOMENTS, N.CGP_NET_LINEAR):
                f["code"] = -1
        # the kernel's static LDS (cgp_net_static_lds) sits beside the arenas
        if top * itemsize * lib.cgp_net_units(pairs) > MAX_LDS_BYTES - lib.cgp_net_static_lds():
            if pairs == 1:
                raise Unsupported(f"LDS footprint {top * itemsize} B")
        return Stage(records=recs, lds_elems=top, final_slot=final_origin, pairs=pairs,
                     final=final, load_stride=load_stride, store_stride=store_stride,
                     part=hs_part)

    def _hs_cells(self, f):
        """(zero cells, data cells) a separable conv's row pass leaves in the row-sum
        scratch (the arena's first HSR·WO cells: hs row q <-> input row q + off; rows
        outside the input are zero rows), or None for a conv without scratch (1x1,
        full-map reduction, single-pass <= 3 taps: cgp_net_hs_elems() <= 2)."""
        h, w, ho, wo, taps, s, off = f["geom"]
        hs_elems = self._lib.cgp_net_hs_elems(f["code"] & N.CGP_NET_CODE_GEOMETRY)
        if hs_elems <= 2:
            return None
        hsr = (ho - 1) * s + taps
        q0, q1 = max(0, -off), min(hsr, h - off)
        assert hsr * wo == hs_elems, (f["geom"], hs_elems)
        zero = set(range(0, q0 * wo)) | set(range(q1 * wo, hsr * wo))
        return zero, set(range(q0 * wo, q1 * wo))

    def _reduce_cells(self, recs):
        """Where a one-pair full-map reduction puts its two wave partial sums (cgp_net_args.part):
        inside the data rows of every separable conv's row-sum scratch, which each row pass
        rewrites anyway — so the partials never land on a zero row; 0 without separable
        convs."""
        lo, hi = 0, 1 << 30
        for f, _ in recs:
            if f["kind"] == N.CGP_NET_CONV:
                cells = self._hs_cells(f)
                if cells is not None:
                    data = cells[1]
                    lo, hi = max(lo, min(data)), min(hi, max(data) + 1)
        return lo if lo + 2 <= hi else 0

    @staticmethod
    def _fuse_reductions(recs, pairs):
        """CGP_NET_CODE_SUM on a separable conv (no addend, no second output) whose map is
        read only by the next record, a full-map reduction, which gets
        CGP_NET_CODE_FROM_SUM (one pair per workgroup or half only)."""
        if pairs > 2 or not FUSE_REDUCE:
            return
        for k in range(len(recs) - 1):
            f, g = recs[k][0], recs[k + 1][0]
            if f["kind"] != N.CGP_NET_CONV or g["kind"] != N.CGP_NET_CONV:
                continue
            h, w, ho, wo, taps, s_, off = f["geom"]
            point = taps == 1 and off == 0
            full = ho == wo == 1 and off == 0 and taps == h == w
            if taps <= 3 or point or full or f.get("dst2", -1) >= 0 or f["add"] >= 0:
                continue
            gh, gw, gho, gwo, gtaps, _, goff = g["geom"]
            if not (gho == gwo == 1 and goff == 0 and gtaps == gh == gw) or g["src"] != f["dst"]:
                continue
            slot = f["dst"]
            if any(r["src"] == slot or r["add"] == slot or r.get("dst2", -1) == slot
                   for r, _ in recs[k + 2:]):
                continue
            f["code"] |= N.CGP_NET_CODE_SUM
            g["code"] |= N.CGP_NET_CODE_FROM_SUM

    def _mark_hs_clean(self, recs, pairs, hs_part=0):
        """CGP_NET_CODE_HS_CLEAN on every separable conv whose zero rows of the row-sum
        scratch are still zero when it runs: the op list repeats for every pair a
        workgroup walks (LDS is zeroed once at kernel start), so the walk below runs it
        twice — the first pass from the zeroed start, the second from the steady state —
        and a conv is clean only if no data sits on its zero rows in either.  Writers of
        scratch cells: separable row passes (their input rows) and a one-pair full-map
        reduction (its two wave partial sums at cells hs_part, hs_part + 1)."""
        dirty, need = set(), set()
        for _ in range(2):
            for idx, (f, _) in enumerate(recs):
                if f["kind"] != N.CGP_NET_CONV:
                    continue
                cells = self._hs_cells(f)
                if cells is not None:
                    zero, data = cells
                    if zero & dirty:
                        need.add(idx)
                    dirty = (dirty - zero) | data
                else:
                    h, w, ho, wo, taps, s, off = f["geom"]
                    if ho == wo == 1 and off == 0 and taps == h == w and pairs <= 2:
                        dirty |= {hs_part, hs_part + 1}
        for idx, (f, _) in enumerate(recs):
            if f["kind"] == N.CGP_NET_CONV and self._hs_cells(f) is not None and \
                    idx not in need:
                f["code"] |= N.CGP_NET_CODE_HS_CLEAN

    def lds_bytes(self, itemsize: int) -> int:
        return self.lds_elems * itemsize

    def _ops_template(self, sidx, stage, flags, itemsize):
        """Stage ``sidx``'s op records with every field but the variance / state pointers
        filled, built once per (stage, flags, itemsize): the bytes (numpy uint8), the
        uint64 slots of the pointer fields with what each holds — (value, side) of the
        variance maps, or "in" / "out" for the state buffers — and the compiled program
        id (cgp_net_program compares only the non-pointer fields).  A forward per tile then
        copies the bytes and writes the pointers: building the records field by field cost
        ~0.15 ms per mnist_as_tf tile (tools/dropin_probe.py), a quarter of a B = 200
        tile's kernel time."""
        import numpy as np
        key = (sidx, flags, itemsize)
        cache = self.__dict__.setdefault("_templates", {})
        t = cache.get(key)
        if t is not None:
            return t
        arr = self._ops_array(stage, None)
        lib = N.load()
        # the SUM / FROM_SUM contract (cnngp.h), checked on the host copy once per stage
        N.check(lib.cgp_net_validate(ctypes.byref(arr), stage.n_ops, stage.pairs),
                "cgp_net_validate")
        size = ctypes.sizeof(N.NetOp)
        slots, what = [], []
        for k, (f, v) in enumerate(stage.records):
            fields = {}                    # _ops_array's order: a state pointer wins
            if v is not None:
                fields.update(var_x=(v, 0), var_y=(v, 1))
            if "var2" in f:
                fields.update(var2_x=(f["var2"], 0), var2_y=(f["var2"], 1))
            if f.get("state") in ("in", "out"):
                fields["var_x"] = f["state"]
            for name, src in fields.items():
                off = k * size + getattr(N.NetOp, name).offset
                assert off % 8 == 0
                slots.append(off // 8)
                what.append(src)
        fl = flags | (N.CGP_FLAG_NET_DUAL if stage.dual else 0)
        program = lib.cgp_net_program(ctypes.byref(arr), stage.n_ops, stage.pairs, fl,
                                      stage.lds_elems, itemsize) if USE_PROGRAMS else 0
        t = (np.frombuffer(bytes(arr), dtype=np.uint8).copy(), np.asarray(slots, np.int64),
             what, program)
        cache[key] = t
        return t

    def _ops_array(self, stage, var, state_in=None, state_out=None):
        """the stage's op records as a ctypes array; ``var`` None leaves the variance /
        state pointers null (the template of _ops_template)"""
        arr = (N.NetOp * stage.n_ops)()
        for k, (f, v) in enumerate(stage.records):
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
            if var is None:
                continue
            if v is not None:
                vx, vy = var[v]
                o.var_x, o.var_y = vx.data_ptr(), vy.data_ptr()
            if "var2" in f:
                vx, vy = var[f["var2"]]
                o.var2_x, o.var2_y = vx.data_ptr(), vy.data_ptr()
            if f.get("state") == "in":
                o.var_x = state_in.data_ptr()
            elif f.get("state") == "out":
                o.var_x = state_out.data_ptr()
        return arr

    def chunk_units(self, itemsize: int, units: int, device=None) -> int:
        """Units per launch group of a staged program: CHUNK_BYTES of the widest state
        record, clamped so that the state buffers of every stage boundary together take at
        most STATE_FREE_FRAC of the device's free memory; a multiple of 64, at least 64."""
        stride = max(max(st.load_stride, st.store_stride) for st in self.stages)
        chunk = CHUNK_BYTES // (stride * itemsize)
        per_unit = sum(st.load_stride for st in self.stages[1:]) * itemsize
        # the free-memory query (hipMemGetInfo: 0.1-0.5 ms, a B = 200 tile's kernel time)
        # only when the state buffers could be large; below SMALL_STATE_BYTES they fit
        if device is not None and torch.device(device).type == "cuda" and \
                min(chunk, units) * per_unit > SMALL_STATE_BYTES:
            free = torch.cuda.mem_get_info(device)[0]
            chunk = min(chunk, int(free * STATE_FREE_FRAC) // max(1, per_unit))
        return min(max(64, chunk // 64 * 64), units)

    @staticmethod
    def units(n1: int, n2: int, same: bool) -> int:
        """Pair units of a tile: st x st supertiles (upper triangle when same) x st²,
        st = the library's cgp_net_supertile()."""
        st = N.load().cgp_net_supertile()
        nbi, nbj = -(-n1 // st), -(-n2 // st)
        return (nbi * (nbi + 1) // 2 if same else nbi * nbj) * st * st

    def prepare(self, x, y, var, n1: int, n2: int, same: bool, flags: int = 0,
                out: Optional[torch.Tensor] = None, qvar: Optional[dict] = None):
        """Upload the op lists for these variance maps; return (launch(stream), out).
        ``qvar``: the scaled (1/16) x-side maps (program.Plan.run_variances_fused), else they
        are filled here with cgp_scale_batch_f64.
        ``out`` may be a row-strided view (e.g. a tile of a larger K): the kernel writes
        K[i, j] at out[i * out.stride(0) + j]."""
        sfx = "f64" if x.dtype == torch.float64 else "f32"
        if out is None:
            out = torch.empty((n1, n2), dtype=x.dtype, device=x.device)
        if out.shape != (n1, n2) or out.stride(1) != 1 or out.dtype != x.dtype:
            raise ValueError("out must be an [n1, n2] row-major view of the input dtype")
        units = self.units(n1, n2, same)
        multi = len(self.stages) > 1
        chunk = units
        states = [None] * (len(self.stages) + 1)
        if multi:
            chunk = self.chunk_units(x.element_size(), units, x.device)
            for b in range(1, len(self.stages)):
                states[b] = torch.empty((chunk * self.stages[b].load_stride,),
                                        dtype=x.dtype, device=x.device)
        lib = N.load()
        fn = getattr(lib, f"cgp_net_{sfx}")
        launches = []
        keep = []
        # the fp64 closed-form ReLU (csrc/cgp_common.h relu_q_n) reads the x-side variance
        # maps scaled by cgp_net_xvar_scale() = 1/16 (an exact scaling that folds its Newton
        # steps' halvings); the copies are filled on the launch stream before the kernels
        quarters = []
        used = self.quarter_vars(x.dtype, flags)
        if used:
            var = dict(var)
            for v in sorted(used):
                vx, vy = var[v]
                if qvar is not None:           # filled by the variance chain already
                    var[v] = (qvar[v], vy)
                    continue
                q = torch.empty_like(vx)
                quarters.append((vx, q))
                keep.append(q)
                var[v] = (q, vy)
        # every stage's op records in one pinned buffer and one H2D copy.  Pinned +
        # non_blocking: a pageable H2D copy would block the host until the previous tile's
        # kernels drained, leaving the GPU idle while this tile's small launches are issued;
        # the caching host allocator keeps the pinned block until the copy has run
        tmpls = [self._ops_template(sidx, st, flags, x.element_size())
                 for sidx, st in enumerate(self.stages)]
        offs = [0]
        for t in tmpls:
            offs.append(offs[-1] + len(t[0]))
        host = torch.empty((offs[-1],), dtype=torch.uint8, pin_memory=True)
        hb = host.numpy()
        for sidx, (tmpl, slots, what, _) in enumerate(tmpls):
            ptrs = [var[w[0]][w[1]].data_ptr() if isinstance(w, tuple) else
                    (states[sidx] if w == "in" else states[sidx + 1]).data_ptr()
                    for w in what]
            blk = hb[offs[sidx]:offs[sidx + 1]]
            blk[:] = tmpl
            blk.view("<u8")[slots] = ptrs
        ops_dev = host.to(x.device, non_blocking=True)   # stream-ordered, freed stream-ordered
        keep.append(ops_dev)
        for sidx, st in enumerate(self.stages):
            program = tmpls[sidx][3]
            a = N.NetArgs()
            a.x, a.y, a.out = x.data_ptr(), y.data_ptr(), out.data_ptr()
            if same:
                a.kdiag = var[self.plan.vf][0].data_ptr()
            a.ops = ops_dev.data_ptr() + offs[sidx]    # records are 8-byte aligned
            a.n1, a.n2, a.ldo = n1, n2, out.stride(0)
            a.nops, a.channels, a.h, a.w = st.n_ops, x.shape[1], x.shape[2], x.shape[3]
            a.same, a.final_slot, a.hs, a.lds_elems = int(same), st.final_slot, 0, st.lds_elems
            a.part = st.part
            a.flags = flags | (N.CGP_FLAG_NET_DUAL if st.dual else 0)
            a.pairs = st.pairs
            a.final_stage = int(st.final)
            a.program = program
            launches.append(a)

        pairs = n1 * (n1 - 1) // 2 if same else n1 * n2

        if quarters:   # one launch fills every scaled map (cgp_net_xvar_scale: 1/16)
            xscale = lib.cgp_net_xvar_scale()
            nq = len(quarters)
            q_src = (ctypes.c_void_p * nq)(*[N.ptr(s_) for s_, _ in quarters])
            q_dst = (ctypes.c_void_p * nq)(*[N.ptr(q_) for _, q_ in quarters])
            q_n = (ctypes.c_int64 * nq)(*[s_.numel() for s_, _ in quarters])

        def run_all(stream):
            if quarters:
                N.call("cgp_scale_batch_f64", nq, q_src, q_dst, q_n, xscale, stream)
            for u0 in range(0, units, chunk):
                u1 = min(units, u0 + chunk)
                for a in launches:
                    if multi:
                        a.unit_begin, a.unit_end = u0, u1
                    N.check(fn(ctypes.byref(a), stream), "cgp_net")

        def launch(stream, keep=keep, states=states):
            # the op lists were uploaded and the state buffers allocated on torch's current
            # stream: a launch on another stream first waits for that stream, and the
            # caching allocator is told the buffers are in use there, so it cannot hand
            # them out again while the kernels still read them
            cur = torch.cuda.current_stream(x.device)
            if stream and stream != cur.cuda_stream:
                ext = torch.cuda.ExternalStream(stream, device=x.device)
                ext.wait_stream(cur)
                for t in keep + [s for s in states if s is not None]:
                    t.record_stream(ext)
            if TIMING is not None:
                st_ = torch.cuda.ExternalStream(stream) if stream else torch.cuda.current_stream()
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                e0.record(st_)
                run_all(stream)
                e1.record(st_)
                TIMING.append((e0, e1, pairs))
            else:
                run_all(stream)

        launch.args = launches           # TileRecipe rewrites x / y / out per call
        launch.states = states
        return launch, out

    def quarter_vars(self, dtype, flags: int = 0) -> set:
        """Values whose x-side variance maps the fp64 closed-form ReLU reads quartered."""
        # the fp64 closed-form ReLU (relu_q_n) reads its x-side maps scaled by
        # cgp_net_xvar_scale() = 1/16 ("quarter": the round-2 name of the 1/4 scale)
        if dtype != torch.float64 or flags & N.CGP_FLAG_EXACT_RELU:
            return set()
        used = self.__dict__.get("_quarter_used")
        if used is None:                 # asked on every forward: the walk once per plan
            used = set()
            for st in self.stages:
                used |= {v for _, v in st.records if v is not None}
                used |= {f["var2"] for f, _ in st.records if "var2" in f}
            self.__dict__["_quarter_used"] = used
        return set(used)

    def tile_recipe(self, plan, x, y, n1: int, n2: int, same: bool, flags: int, stream):
        """The cached TileRecipe of a forward of this shape on ``stream`` (built on first
        use), or None when its persistent buffers would exceed RECIPE_MAX_BYTES or the
        variance chain cannot run the program (forward then takes the per-call path)."""
        if RECIPE_MAX_BYTES <= 0:
            return None
        key = (n1, n2, bool(same), tuple(x.shape[1:]), x.dtype, x.device, flags, stream)
        lock = self.__dict__.setdefault("_recipe_lock", threading.Lock())
        with lock:
            cache = self.__dict__.setdefault("_recipes", collections.OrderedDict())
            if key in cache:
                cache.move_to_end(key)
                return cache[key]
            rec = TileRecipe.build(self, plan, x, y, n1, n2, same, flags, stream)
            if rec is None:
                return None
            cache[key] = rec
            while len(cache) > RECIPE_SLOTS or (
                    len(cache) > 1 and sum(r.nbytes for r in cache.values()) > RECIPE_TOTAL_BYTES):
                cache.popitem(last=False)
            return rec

    def run(self, x, y, var, n1: int, n2: int, same: bool, stream, flags: int = 0,
            out: Optional[torch.Tensor] = None, qvar: Optional[dict] = None):
        """K tile [n1, n2] of the pairs (x_i, y_j).  var: value -> (xx [n1,..], yy [n2,..])
        for every value in ``need_var``."""
        launch, out = self.prepare(x, y, var, n1, n2, same, flags, out, qvar)
        launch(stream)
        return out


class TileRecipe:
    """One forward's whole launch sequence for a tile shape on one stream, built once and
    replayed: the variance chain (cgp_var_chain_*) into a persistent map buffer, then the
    net stages (cgp_net_*) whose op records point into that buffer — so the records are
    uploaded once, the stage-state buffers are allocated once, and a call only writes the
    images' and the output's addresses into the prebuilt argument structs and issues the
    launches.  save_kernel.py's loop (kernel_save_tools.py:49-58, a forward per tile and a
    synchronous copy back) spent 0.11 ms (ConvNet) to 0.29 ms (mnist_as_tf) of host time
    per B = 200 tile building these (tools/dropin_probe.py), GPU idle meanwhile.

    Replays on one stream are ordered by that stream: the next call's variance chain
    overwrites the maps only after this call's net kernels have read them.  A lock keeps
    each call's launch sequence contiguous when threads share a stream."""

    def __init__(self):
        self.lock = threading.Lock()

    @classmethod
    def build(cls, net, plan, x, y, n1, n2, same, flags, stream):
        from .program import DevPtr
        need = set(net.need_var)
        quarter = net.quarter_vars(x.dtype, flags) & need
        chain = plan._var_chain(need, quarter, x.device)
        if chain is None or chain["lds"] * x.element_size() > 64 * 1024 or \
                x.shape[2] * x.shape[3] > 1024:
            return None
        m2 = 0 if same else n2
        n = n1 + m2
        item = x.element_size()
        vbytes = (n * chain["total"] + n1 * chain["qtotal"]) * item
        units = net.units(n1, n2, same)
        sbytes = sum(units * st.load_stride for st in net.stages[1:]) * item
        if vbytes + sbytes > RECIPE_MAX_BYTES:
            return None
        r = cls()
        r.nbytes = vbytes + sbytes
        r.shape = (n1, n2, tuple(x.shape[1:]), x.dtype, x.device)
        r.same = bool(same)
        r.vbuf = torch.empty((vbytes // item,), dtype=x.dtype, device=x.device)
        a = N.VarArgs()
        a.out, a.ops = r.vbuf.data_ptr(), chain["ops"].data_ptr()
        a.n1, a.n2, a.store_total = n1, m2, chain["total"]
        a.nops, a.channels, a.h, a.w = chain["nops"], x.shape[1], x.shape[2], x.shape[3]
        a.lds_elems, a.scratch = chain["lds"], chain["scratch"]
        r.va = a
        r.var_fn = getattr(N.load(), f"cgp_var_chain_{plan._sfx(x.dtype)}")
        r.chain_ops = chain["ops"]
        var, qvar = {}, {}
        shapes = plan.prog.shapes
        for v, off in chain["store"].items():
            ho, wo = shapes[v]
            px = DevPtr(r.vbuf, n * off * item)
            var[v] = (px, px if same else DevPtr(r.vbuf, (n * off + n1 * ho * wo) * item))
        for v, off in chain["qstore"].items():
            qvar[v] = DevPtr(r.vbuf, (n * chain["total"] + n1 * off) * item)
        out = torch.empty((n1, n2), dtype=x.dtype, device=x.device)
        r.launch, _ = net.prepare(x, y, var, n1, n2, same, flags, out, qvar or None)
        r.args = r.launch.args
        return r

    def run(self, x, y, stream):
        n1, n2, _, _, _ = self.shape
        out = torch.empty((n1, n2), dtype=x.dtype, device=x.device)
        xp, yp, op = x.data_ptr(), y.data_ptr(), out.data_ptr()
        with self.lock:
            self.va.x, self.va.y = xp, yp
            N.check(self.var_fn(self.va, stream), "cgp_var_chain")
            for a in self.args:
                a.x, a.y, a.out, a.ldo = xp, yp, op, n2
            self.launch(stream)
        return out
