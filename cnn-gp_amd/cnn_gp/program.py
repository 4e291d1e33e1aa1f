"""Compile an NNGP module tree into a fused device program and run it.

The reference evaluates ``Sequential.propagate`` recursively (cnn_gp/kernels.py:184-187),
issuing 3 ``F.conv2d`` + a bias pass per Conv2d and ~14 pointwise ops per ReLU on the
whole [N1·N2, 1, H, W] covariance tensor.  Here the tree is flattened once into SSA form

    v0 = moments(x, y)               kernels.py:44-49
    v  = conv(u, geometry)           kernels.py:92-98
    v  = relu(u)                     kernels.py:134-165
    v  = add[(coef, u), ...]         Sum (kernels.py:252-254) / Mixture (:220-225)

and then split into two device pipelines:

* the VARIANCE pipeline runs every op, unfused, on the per-image maps [xx | yy]
  ((N1 + N2) maps — negligible next to the N1·N2 pair maps) and keeps the variances
  of every value a ReLU consumes;
* the PAIR pipeline runs on the N1·N2 maps with ops fused so each HBM pass does the
  most work:  [ReLU|moments] → Conv → [ReLU] → [+ addend]  is ONE kernel
  (cgp_conv_*), a ReLU not adjacent to a single-use conv is cgp_relu_* (+ addend),
  and only sums that cannot be folded into their producer run as cgp_axpby_*.

Fusion changes no arithmetic: each fused stage performs exactly the operations of the
op it replaces (a + b == b + a in IEEE, so folding a Sum into either branch is exact).
"""
from __future__ import annotations

import dataclasses
from typing import Optional

import torch

from . import _native as N


# ------------------------------------------------------------------------------------
# IR
# ------------------------------------------------------------------------------------
@dataclasses.dataclass
class ConvGeom:
    taps: int
    offset: int
    stride: int
    dilation: int
    weight: float       # the kernel buffer's value (fp32-rounded unless built in fp64)
    bias: float
    extent: int = 0     # the reference kernel's edge (k + 1 for an even "same" kernel)


@dataclasses.dataclass
class Op:
    kind: str                              # 'conv' | 'relu' | 'add' | 'moments'
    dst: int
    src: Optional[int] = None
    geom: Optional[ConvGeom] = None
    shape_in: tuple = (0, 0)
    shape_out: tuple = (0, 0)
    terms: list = dataclasses.field(default_factory=list)   # add: [(coef|None, value)]
    # fusion (pair pipeline only)
    pre: int = N.CGP_PRE_NONE
    pre_var: Optional[int] = None          # value whose variances feed the PRE ReLU
    post: int = N.CGP_POST_NONE
    post_var: Optional[int] = None
    addend: Optional[int] = None


class Program:
    """Flattened SSA program for one module tree at one input size."""

    def __init__(self):
        self.ops: list[Op] = []
        self.shapes: dict[int, tuple] = {}
        self.n_values = 0

    def new_value(self, shape) -> int:
        v = self.n_values
        self.n_values += 1
        self.shapes[v] = tuple(shape)
        return v


def conv_geometry(mod) -> ConvGeom:
    """Conv2d.__init__'s padding rules (kernels.py:71-88) as tap offsets."""
    k, d, s = int(mod.kernel_size), int(mod.dilation), int(mod.stride)
    pad = int(mod.padding)
    offset = -pad + (d if mod.kernel_has_row_of_zeros else 0)
    kern = mod.kernel.detach().to("cpu", torch.float64).reshape(mod.kernel.shape[-2:])
    w = float(kern[-1, -1])
    want = torch.full_like(kern, w)
    if mod.kernel_has_row_of_zeros:
        want[0, :] = 0.
        want[:, 0] = 0.
    if tuple(mod.kernel.shape[:2]) != (1, 1) or not torch.equal(kern, want):
        # the HIP kernels run the reference's constant box kernel (kernels.py:75-87); a
        # buffer edited to anything else has no device path
        raise NotImplementedError(
            "Conv2d.kernel must be the constant var_weight/k² box (kernels.py:75-87), with "
            "the zero first row and column of an even 'same' kernel; got a buffer of shape "
            f"{tuple(mod.kernel.shape)} that is not")
    return ConvGeom(taps=k, offset=offset, stride=s, dilation=d, weight=w,
                    extent=k + 1 if mod.kernel_has_row_of_zeros else k,
                    bias=float(mod.var_bias))


def conv_out_hw(mod, h: int, w: int):
    """F.conv2d output size for Conv2d `mod` (kernel extent k+1 for even 'same')."""
    k, d, s, p = int(mod.kernel_size), int(mod.dilation), int(mod.stride), int(mod.padding)
    keff = k + 1 if mod.kernel_has_row_of_zeros else k
    ho = (h + 2 * p - d * (keff - 1) - 1) // s + 1
    wo = (w + 2 * p - d * (keff - 1) - 1) // s + 1
    if ho <= 0 or wo <= 0:
        raise RuntimeError(f"Conv2d(kernel_size={k}, stride={s}, padding={p}, dilation={d}) "
                           f"produces an empty output from a {h}x{w} input")
    return ho, wo


def _emit(prog: Program, mod, v: int) -> int:
    """Append the ops of `mod` applied to value v; return the output value."""
    from . import kernels as K
    if isinstance(mod, K.Conv2d):
        h, w = prog.shapes[v]
        ho, wo = conv_out_hw(mod, h, w)
        out = prog.new_value((ho, wo))
        prog.ops.append(Op("conv", out, src=v, geom=conv_geometry(mod), shape_in=(h, w),
                           shape_out=(ho, wo)))
        return out
    if isinstance(mod, K.ReLU):
        out = prog.new_value(prog.shapes[v])
        prog.ops.append(Op("relu", out, src=v, shape_in=prog.shapes[v],
                           shape_out=prog.shapes[v]))
        return out
    if isinstance(mod, K.Sequential):
        for m in mod.mods:
            v = _emit(prog, m, v)
        return v
    if isinstance(mod, (K.Sum, K.Mixture)):
        outs = [_emit(prog, m, v) for m in mod.mods]
        shp = {prog.shapes[o] for o in outs}
        if len(shp) != 1:
            raise RuntimeError(f"{type(mod).__name__} branches disagree on spatial size: {shp}")
        if isinstance(mod, K.Sum):
            if len(outs) == 1:
                return outs[0]          # 0 + kp == kp
            terms = [(None, o) for o in outs]
        else:
            props = mod.proportions()
            terms = [(props[i], o) for i, o in enumerate(outs)]
        out = prog.new_value(shp.pop())
        prog.ops.append(Op("add", out, terms=terms, shape_in=prog.shapes[out],
                           shape_out=prog.shapes[out]))
        return out
    if isinstance(mod, K.NNGPKernel):
        raise TypeError(f"no device lowering for {type(mod).__name__}")
    raise TypeError(f"not an NNGP kernel module: {type(mod).__name__}")


def compile_program(model, h: int, w: int) -> tuple:
    """Returns (Program, v0, v_final)."""
    prog = Program()
    v0 = prog.new_value((h, w))
    vf = _emit(prog, model, v0)
    return prog, v0, vf


# ------------------------------------------------------------------------------------
# fusion for the pair pipeline
# ------------------------------------------------------------------------------------
def _uses(ops, final):
    u = {}
    for op in ops:
        srcs = [op.src] if op.src is not None else []
        srcs += [t for _, t in op.terms]
        if op.addend is not None:
            srcs.append(op.addend)
        for s in srcs:
            u[s] = u.get(s, 0) + 1
    u[final] = u.get(final, 0) + 1
    return u


def fuse(prog: Program, v0: int, vf: int, enable: bool = True, pre_relu: bool = True,
         fold_moments: bool = True) -> list:
    """Return the fused op list for the pair pipeline (prog.ops is left untouched).
    ``pre_relu`` / ``fold_moments`` enable rules 3 / 4 (the whole-network kernel keeps
    standalone ReLU and moments ops: in LDS they cost no extra memory pass)."""
    ops = [dataclasses.replace(o, terms=list(o.terms)) for o in prog.ops]
    if not enable:
        return ops
    producer = lambda ops_, v: next((i for i, o in enumerate(ops_) if o.dst == v), None)  # noqa

    # 1. conv -> relu  ==> conv(post=RELU)
    changed = True
    while changed:
        changed = False
        uses = _uses(ops, vf)
        for ri, r in enumerate(ops):
            if r.kind != "relu" or r.addend is not None:
                continue
            pi = producer(ops, r.src)
            if pi is None:
                continue
            c = ops[pi]
            if c.kind == "conv" and c.post == N.CGP_POST_NONE and c.addend is None \
                    and uses.get(r.src, 0) == 1:
                c.post, c.post_var, c.dst = N.CGP_POST_RELU, r.src, r.dst
                del ops[ri]
                changed = True
                break

    # 2. plain 2-term Sum folded into the producer of one term as its epilogue addend
    changed = True
    while changed:
        changed = False
        uses = _uses(ops, vf)
        for ai, a in enumerate(ops):
            if a.kind != "add" or len(a.terms) != 2 or any(c is not None for c, _ in a.terms):
                continue
            (_, t0), (_, t1) = a.terms
            for cand, other in ((t1, t0), (t0, t1)):
                pi = producer(ops, cand)
                if pi is None or ops[pi].kind not in ("conv", "relu") or \
                        ops[pi].addend is not None or uses.get(cand, 0) != 1:
                    continue
                oi = producer(ops, other)
                if oi is not None and oi > pi:
                    continue                    # the addend must exist before the producer
                if cand == other:
                    continue
                ops[pi].addend, ops[pi].dst = other, a.dst
                del ops[ai]
                changed = True
                break
            if changed:
                break

    # 3. relu -> conv  ==> conv(pre=RELU) when the relu output has no other consumer
    changed = pre_relu
    while changed:
        changed = False
        uses = _uses(ops, vf)
        for ci, c in enumerate(ops):
            if c.kind != "conv" or c.pre != N.CGP_PRE_NONE:
                continue
            ri = producer(ops, c.src)
            if ri is None:
                continue
            r = ops[ri]
            if r.kind == "relu" and r.addend is None and uses.get(c.src, 0) == 1:
                c.pre, c.pre_var, c.src = N.CGP_PRE_RELU, r.src, r.src
                c.shape_in = r.shape_in
                del ops[ri]
                changed = True
                break

    # 4. the input moments folded into a single consuming conv
    uses = _uses(ops, vf)
    if fold_moments and uses.get(v0, 0) == 1 and vf != v0:
        for c in ops:
            if c.kind == "conv" and c.src == v0 and c.pre == N.CGP_PRE_NONE:
                c.pre = N.CGP_PRE_MOMENTS
                break
    return ops


def needed_variances(ops) -> set:
    need = set()
    for o in ops:
        if o.kind == "relu":
            need.add(o.src)
        if o.pre == N.CGP_PRE_RELU:
            need.add(o.pre_var)
        if o.post == N.CGP_POST_RELU:
            need.add(o.post_var)
    return need


# ------------------------------------------------------------------------------------
# execution
# ------------------------------------------------------------------------------------
def _adjacent(x, y) -> bool:
    """y's elements start where x's end (one allocation, x then y), both contiguous."""
    return (x.is_contiguous() and y.is_contiguous() and x.dtype == y.dtype
            and y.data_ptr() == x.data_ptr() + x.numel() * x.element_size())



class DevPtr:
    """A device address inside ``base`` (kept alive by the handle, like a view would be):
    what the launch records need of a variance map, without building a tensor view."""
    __slots__ = ("base", "off")

    def __init__(self, base: torch.Tensor, off: int):
        self.base, self.off = base, off

    def data_ptr(self) -> int:
        return self.base.data_ptr() + self.off

class Plan:
    """A compiled model at one input geometry: the variance program and the fused pair
    program.  Cached per (H, W, fuse) on the model."""

    def __init__(self, model, h: int, w: int, enable_fusion: bool = True,
                 exact_relu: bool = False):
        self.flags = N.CGP_FLAG_EXACT_RELU if exact_relu else 0
        self.prog, self.v0, self.vf = compile_program(model, h, w)
        self.pair_ops = fuse(self.prog, self.v0, self.vf, enable_fusion)
        self.need_var = needed_variances(self.pair_ops)
        fh, fw = self.prog.shapes[self.vf]
        self.final_hw = (fh, fw)
        self.moments_fused = any(o.pre == N.CGP_PRE_MOMENTS for o in self.pair_ops)

    # -- helpers -----------------------------------------------------------------------
    @staticmethod
    def _sfx(dtype):
        if dtype == torch.float64:
            return "f64"
        if dtype == torch.float32:
            return "f32"
        raise TypeError(f"unsupported dtype {dtype} (float32 or float64)")

    def _last_use(self, ops, extra_final):
        last = {}
        for idx, o in enumerate(ops):
            srcs = ([o.src] if o.src is not None else []) + [t for _, t in o.terms]
            if o.addend is not None:
                srcs.append(o.addend)
            for s in srcs:
                last[s] = idx
        last[extra_final] = len(ops)
        return last

    # -- variance pipeline --------------------------------------------------------------
    def run_variances(self, xx0, yy0, n1, n2, same, stream, need=None):
        """Per-image variance maps of every value a ReLU reads (or of ``need``).
        xx0/yy0: [n, H, W]."""
        sfx = self._sfx(xx0.dtype)
        dev = xx0.device
        vals = {self.v0: (xx0, yy0)}
        need = self.need_var if need is None else need
        ops = self.prog.ops
        last = self._last_use(ops, self.vf)
        keep = {}
        if self.v0 in need:
            keep[self.v0] = vals[self.v0]
        for idx, op in enumerate(ops):
            ho, wo = op.shape_out
            if op.kind == "conv":
                xin, yin = vals[op.src]
                buf = torch.empty((n1 + n2, ho, wo), dtype=xx0.dtype, device=dev)
                g = op.geom
                h, w = op.shape_in
                # xx and yy may live in different allocations: launch per block, or once
                # over both when they are adjacent (every value after the first is)
                parts = ((xin, buf[:n1], n1), (yin, buf[n1:], n2))
                if _adjacent(xin, yin):
                    parts = ((xin, buf, n1 + n2),)
                for src, dst, n in parts:
                    a = N.ConvArgs()
                    a.in_, a.out = N.ptr(src), N.ptr(dst)
                    a.nmaps, a.n1, a.n2 = n, n, 1
                    a.h, a.w, a.ho, a.wo = h, w, ho, wo
                    a.taps, a.offset, a.stride, a.dilation = g.taps, g.offset, g.stride, g.dilation
                    a.weight, a.bias = g.weight, g.bias
                    N.check(getattr(N.load(), f"cgp_conv_{sfx}")(a, stream), "cgp_conv")
                out = (buf[:n1], buf[n1:])
            elif op.kind == "relu":
                xin, yin = vals[op.src]
                buf = torch.empty((n1 + n2, ho, wo), dtype=xx0.dtype, device=dev)
                N.call(f"cgp_var_relu_{sfx}", N.ptr(xin), N.ptr(yin), n1, n2, ho * wo,
                       int(same), N.ptr(buf[:n1]), N.ptr(buf[n1:]), stream)
                out = (buf[:n1], buf[n1:])
            elif op.kind == "add":
                buf = torch.empty((n1 + n2, ho, wo), dtype=xx0.dtype, device=dev)
                outx, outy = buf[:n1], buf[n1:]
                whole = all(_adjacent(*vals[t]) for _, t in op.terms)
                for part, o, n in (((None, buf, n1 + n2),) if whole else
                                   ((0, outx, n1), (1, outy, n2))):
                    first = True
                    for coef, t in op.terms:
                        src = vals[t][0] if part is None else vals[t][part]
                        if first:
                            alpha = 1.0 if coef is None else coef
                            N.call(f"cgp_axpby_{sfx}", alpha, N.ptr(src), 0.0, None, N.ptr(o),
                                   n * ho * wo, stream)
                            first = False
                        else:
                            beta = 1.0 if coef is None else coef
                            N.call(f"cgp_axpby_{sfx}", 1.0, N.ptr(o), beta, N.ptr(src), N.ptr(o),
                                   n * ho * wo, stream)
                out = (outx, outy)
            else:
                raise AssertionError(op.kind)
            vals[op.dst] = out
            if op.dst in need:
                keep[op.dst] = out
            # free what no later op reads
            for v in [v for v in vals if last.get(v, -1) <= idx and v != op.dst]:
                del vals[v]
        return keep

    # -- the same program in one launch (cgp_var_chain_*) --------------------------------
    def _var_chain(self, need, quarter, dev):
        """cgp_var_op records of the variance program (cached per need/quarter/device):
        LDS slots by first fit over the values' live ranges, store offsets per image.
        None when the program has an op the chain kernel lacks (a Sum of > 4 terms)."""
        key = (frozenset(need), frozenset(quarter), str(dev))
        cache = self.__dict__.setdefault("_var_chains", {})
        if key in cache:
            return cache[key]
        ops = self.prog.ops
        shapes = self.prog.shapes
        last = self._last_use(ops, self.vf)
        free = []                                  # (start, size) free LDS ranges
        top = [0]
        slot = {}

        def alloc(v):
            size = shapes[v][0] * shapes[v][1]
            size += size & 1                       # 16-byte aligned fp64 slots
            for k, (st, sz) in enumerate(free):
                if sz >= size:
                    free[k] = (st + size, sz - size)
                    slot[v] = st
                    return st
            slot[v] = top[0]
            top[0] += size
            return slot[v]

        def release(v):
            size = shapes[v][0] * shapes[v][1]
            free.append((slot.pop(v), size + (size & 1)))

        store, qstore, total, qtotal = {}, {}, 0, 0

        def stored(v):
            nonlocal total, qtotal
            if v not in need:
                return -1, -1
            hw = shapes[v][0] * shapes[v][1]
            store[v], total = total, total + hw
            if v in quarter:
                qstore[v], qtotal = qtotal, qtotal + hw
            return store[v], qstore.get(v, -1)

        recs = []
        h, w = shapes[self.v0]
        r = N.VarOp(kind=N.CGP_VAR_MOMENTS, dst=alloc(self.v0), h=h, w=w, ho=h, wo=w)
        r.src[:] = [-1, -1, -1, -1]
        r.store, r.qstore = stored(self.v0)
        recs.append(r)
        for idx, op in enumerate(ops):
            srcs = [op.src] if op.kind in ("conv", "relu") else [t for _, t in op.terms]
            # the chain kernel covers at most kVarE·kBlock = 1024 elements per pass, over
            # both the row pass (h·wo) and the output (ho·wo): a conv padded beyond "same"
            # grows its map past the input's, so the input size alone does not bound it
            (hi_, wi_), (ho_, wo_) = shapes[srcs[0]], op.shape_out
            if len(srcs) > 4 or max(hi_ * wo_, ho_ * wo_, hi_ * wi_) > 1024:
                cache[key] = None
                return None
            r = N.VarOp(dst=alloc(op.dst))
            r.src[:] = [slot[s] for s in srcs] + [-1] * (4 - len(srcs))
            (r.h, r.w), (r.ho, r.wo) = shapes[srcs[0]], op.shape_out
            if op.kind == "conv":
                g = op.geom
                r.kind = N.CGP_VAR_CONV
                r.taps, r.offset, r.stride, r.dilation = g.taps, g.offset, g.stride, g.dilation
                r.weight, r.bias = g.weight, g.bias
            elif op.kind == "relu":
                r.kind = N.CGP_VAR_HALF
            else:
                r.kind = N.CGP_VAR_SUM
                r.coef[:] = [1.0 if c is None else float(c) for c, _ in op.terms] + \
                    [0.0] * (4 - len(op.terms))
            r.store, r.qstore = stored(op.dst)
            recs.append(r)
            for s in set(srcs):
                if last.get(s, -1) <= idx and s in slot:
                    release(s)
            if last.get(op.dst, -1) <= idx and op.dst != self.vf:
                release(op.dst)
        # the convs' row-sum scratch after the slots: [h][wo] of the largest conv
        scratch = top[0]
        hs = max([r.h * r.wo for r in recs if r.kind == N.CGP_VAR_CONV] + [2])
        top[0] += hs + (hs & 1)
        arr = (N.VarOp * len(recs))(*recs)
        host = torch.frombuffer(bytearray(bytes(arr)), dtype=torch.uint8).pin_memory()
        chain = dict(ops=host.to(dev, non_blocking=True), nops=len(recs), lds=top[0],
                     scratch=scratch,
                     store=store, qstore=qstore, total=total, qtotal=qtotal)
        cache[key] = chain
        return chain

    def run_variances_fused(self, x, y, n1, n2, same, stream, need, quarter=(), views=True):
        """run_variances in one launch.  Returns (var, qvar): var[v] = (xx [n1,..],
        yy [n2,..]) for v in need (yy is xx when same), qvar[v] = xx scaled by
        cgp_net_xvar_scale() (1/16 from ABI 9; "quarter" is the round-2 name) for v in quarter;
        None when the chain kernel cannot run this program.  ``views=False`` gives
        DevPtr handles (data_ptr() only) instead of tensor views: a forward only needs the
        maps' addresses, and ~90 views cost ~0.1 ms of host time per ResNet tile."""
        need = set(need)
        quarter = set(quarter) & need
        chain = self._var_chain(need, quarter, x.device)
        # the chain kernel holds maps of up to 4·256 pixels per workgroup in 64 KB of LDS
        if chain is None or chain["lds"] * x.element_size() > 64 * 1024 or \
                x.shape[2] * x.shape[3] > 1024:
            return None
        m2 = 0 if same else n2
        n = n1 + m2
        out = torch.empty((n * chain["total"] + n1 * chain["qtotal"],), dtype=x.dtype,
                          device=x.device)
        a = N.VarArgs()
        a.x, a.y, a.out, a.ops = x.data_ptr(), y.data_ptr(), out.data_ptr(), \
            chain["ops"].data_ptr()
        a.n1, a.n2, a.store_total = n1, m2, chain["total"]
        a.nops, a.channels, a.h, a.w = chain["nops"], x.shape[1], x.shape[2], x.shape[3]
        a.lds_elems, a.scratch = chain["lds"], chain["scratch"]
        N.check(getattr(N.load(), f"cgp_var_chain_{self._sfx(x.dtype)}")(a, stream),
                "cgp_var_chain")
        shapes = self.prog.shapes
        var, qvar = {}, {}
        if not views:
            item = out.element_size()
            for v, off in chain["store"].items():
                ho, wo = shapes[v]
                px = DevPtr(out, n * off * item)
                var[v] = (px, px if same else DevPtr(out, (n * off + n1 * ho * wo) * item))
            for v, off in chain["qstore"].items():
                qvar[v] = DevPtr(out, (n * chain["total"] + n1 * off) * item)
            return var, qvar
        for v, off in chain["store"].items():
            ho, wo = shapes[v]
            blk = out[n * off:n * (off + ho * wo)].view(n, ho, wo)
            var[v] = (blk[:n1], blk[:n1] if same else blk[n1:])
        for v, off in chain["qstore"].items():
            ho, wo = shapes[v]
            base = n * chain["total"] + n1 * off
            qvar[v] = out[base:base + n1 * ho * wo].view(n1, ho, wo)
        return var, qvar

    # -- pair pipeline ------------------------------------------------------------------
    def run_pairs(self, x, y, xy0, var, n1, n2, same, diag, stream, probe=None):
        """Runs the fused pair program; returns the final [nmaps, fh, fw] tensor.
        x, y: images [n, C, H, W] (for the fused moments); xy0: the initial pair maps
        (None when the moments are fused into the first conv).  ``probe(idx, op, launch)``
        (optional) is called after each op with a closure that re-launches it, so a
        benchmark can time single kernels on live data."""
        sfx = self._sfx(x.dtype)
        lib = N.load()
        dev = x.device
        nmaps = n1 if diag else n1 * n2
        vals = {}
        if xy0 is not None:
            vals[self.v0] = xy0
        ops = self.pair_ops
        last = self._last_use(ops, self.vf)
        C = x.shape[1]
        for idx, op in enumerate(ops):
            ho, wo = op.shape_out
            if op.kind == "conv":
                out = torch.empty((nmaps, ho, wo), dtype=x.dtype, device=dev)
                g = op.geom
                h, w = op.shape_in
                a = N.ConvArgs()
                if op.pre == N.CGP_PRE_MOMENTS:
                    a.in_, a.in_y, a.channels = N.ptr(x), N.ptr(y), C
                else:
                    a.in_ = N.ptr(vals[op.src])
                a.out = N.ptr(out)
                a.addend = N.ptr(vals[op.addend]) if op.addend is not None else None
                if op.pre == N.CGP_PRE_RELU:
                    vx, vy = var[op.pre_var]
                    a.pre_xx, a.pre_yy = N.ptr(vx), N.ptr(vy)
                if op.post == N.CGP_POST_RELU:
                    vx, vy = var[op.post_var]
                    a.post_xx, a.post_yy = N.ptr(vx), N.ptr(vy)
                a.pre, a.post = op.pre, op.post
                a.nmaps, a.n1, a.n2 = nmaps, n1, n2
                a.h, a.w, a.ho, a.wo = h, w, ho, wo
                a.taps, a.offset, a.stride, a.dilation = g.taps, g.offset, g.stride, g.dilation
                a.same, a.diag = int(same), int(diag)
                a.weight, a.bias = g.weight, g.bias
                a.flags = self.flags
                fn = getattr(lib, f"cgp_conv_{sfx}")
                launch = (lambda fn=fn, a=a: N.check(fn(a, stream), "cgp_conv"))
            elif op.kind == "relu":
                out = torch.empty((nmaps, ho, wo), dtype=x.dtype, device=dev)
                vx, vy = var[op.src]
                r = N.ReluArgs()
                r.xy, r.out = N.ptr(vals[op.src]), N.ptr(out)
                r.addend = N.ptr(vals[op.addend]) if op.addend is not None else None
                r.xx, r.yy = N.ptr(vx), N.ptr(vy)
                r.nmaps, r.n1, r.n2 = nmaps, n1, n2
                r.hw, r.same, r.diag = ho * wo, int(same), int(diag)
                r.flags = self.flags
                fn = getattr(lib, f"cgp_relu_{sfx}")
                launch = (lambda fn=fn, r=r: N.check(fn(r, stream), "cgp_relu"))
            elif op.kind == "add":
                out = torch.empty((nmaps, ho, wo), dtype=x.dtype, device=dev)
                n = nmaps * ho * wo
                srcs = [(coef, vals[t]) for coef, t in op.terms]

                def launch(srcs=srcs, out=out, n=n):
                    for k, (coef, src) in enumerate(srcs):
                        c = 1.0 if coef is None else coef
                        if k == 0:
                            N.call(f"cgp_axpby_{sfx}", c, N.ptr(src), 0.0, None, N.ptr(out), n,
                                   stream)
                        else:
                            N.call(f"cgp_axpby_{sfx}", 1.0, N.ptr(out), c, N.ptr(src),
                                   N.ptr(out), n, stream)
            else:
                raise AssertionError(op.kind)
            launch()
            if probe is not None:
                probe(idx, op, launch)
            vals[op.dst] = out
            for v in [v for v in vals if last.get(v, -1) <= idx and v != op.dst]:
                del vals[v]
        return vals[self.vf]
