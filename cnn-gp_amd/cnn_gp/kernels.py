"""Drop-in NNGP kernel modules (reference: cnn_gp/kernels.py), evaluated on MI355X.

Same constructors, attributes and call surface as the reference —
``Sequential(*mods)(x, y=None, same=None, diag=False)`` — but ``forward`` runs a fused
device program (program.py) through libcnngp.so instead of torch ops.  Tensors are
storage only: no torch compute runs on the pair maps.
"""
from __future__ import annotations

import os
from typing import Optional

import numpy as np
import torch
import torch.nn as nn

from . import _native as N
from .program import Plan

# the whole-network path computes the per-image variance maps with one cgp_var_chain launch
# (CGP_VAR_CHAIN=0: the layer-by-layer variance pipeline, one launch per op)
VAR_CHAIN = os.environ.get("CGP_VAR_CHAIN", "1") != "0"

__all__ = ("NNGPKernel", "Conv2d", "ReLU", "Sequential", "Mixture", "Sum", "resnet_block")


def _stream_handle(device):
    return torch.cuda.current_stream(device).cuda_stream


def _to_device(t: torch.Tensor, device) -> torch.Tensor:
    if t.device != device:
        t = t.to(device, non_blocking=True)
    return t.contiguous()


class _ImageVariances:
    """Variance maps of one image set for one Gram build (NNGPKernel.image_variances):
    var[v] = [N, h, w] maps of every value the whole-network kernel reads, qvar[v] their
    x-side copies scaled by cgp_net_xvar_scale() = 1/16 (fp64 closed-form ReLU), key =
    (H, W, dtype, plan flags)."""

    __slots__ = ("images", "var", "qvar", "key")

    def __init__(self, images, var, qvar, key):
        self.images, self.var, self.qvar, self.key = images, var, qvar, key

    def __len__(self):
        return len(self.images)


# bumped by every change an NNGPKernel's structure key could see (attribute sets and
# deletes, add_module / register_buffer, .to() / .double() / .cuda() through _apply):
# _structure_key reuses its last walk while the generation is unchanged
_GENERATION = [0]


class NNGPKernel(nn.Module):
    """Base class; ``forward`` mirrors kernels.py:18-57."""

    def __setattr__(self, name, value):
        _GENERATION[0] += 1
        super().__setattr__(name, value)

    def __delattr__(self, name):
        _GENERATION[0] += 1
        super().__delattr__(name)

    def add_module(self, name, module):
        _GENERATION[0] += 1
        super().add_module(name, module)

    def register_buffer(self, name, tensor, persistent=True):
        _GENERATION[0] += 1
        super().register_buffer(name, tensor, persistent)

    def _apply(self, fn, *args, **kwargs):
        _GENERATION[0] += 1
        out = super()._apply(fn, *args, **kwargs)
        _GENERATION[0] += 1
        return out

    def _plan(self, h: int, w: int) -> Plan:
        cache = self.__dict__.setdefault("_cgp_plans", {})
        fusion = getattr(self, "_cgp_fusion", True)
        exact = getattr(self, "_cgp_exact_relu", False)
        key = (h, w, fusion, exact, self._structure_key())
        wver = self._weights_version()
        if self.__dict__.get("_cgp_wver") != wver:
            # a Conv2d weight buffer changed in place (load_state_dict, mul_, .data = …):
            # the reference reads self.kernel on every call (kernels.py:92-97), so every
            # plan built from the old weights goes
            cache.clear()
            self.__dict__["_cgp_wver"] = wver
        plan = cache.get(key)
        if plan is None:
            plan = Plan(self, h, w, enable_fusion=fusion, exact_relu=exact)
            cache[key] = plan
        return plan

    def _structure_key(self):
        """Changes whenever a hyper-parameter the program depends on changes.  Asked on
        every forward (the plan cache's key): ``modules()`` over the 114-module ResNets
        cost a quarter of a millisecond per call, as long as a B = 200 tile's kernels
        (bench.py ``dropin``).  So the last key is reused while no NNGPKernel has changed
        since (_GENERATION; a tree with a Mixture is walked every time, its logits can
        change in place), and the walk itself goes by hand (pre-order, attributes read
        from the instance dicts)."""
        memo = self.__dict__.get("_cgp_skey")
        if memo is not None and memo[0] == _GENERATION[0]:
            return memo[1]
        gen = _GENERATION[0]
        mixture = False
        key = []
        bufs = []
        stack = [self]
        while stack:
            m = stack.pop()
            d = m.__dict__
            if isinstance(m, Conv2d):
                # host-side attributes only: reading the (device) buffer would sync
                key.append(("c", d["kernel_size"], d["stride"], d["padding"], d["dilation"],
                            float(d["var_weight"]), float(d["var_bias"]),
                            d["_buffers"]["kernel"].dtype))
                bufs.append(d["_buffers"]["kernel"])
            elif isinstance(m, Mixture):
                mixture = True
                key.append(("m", tuple(m.proportions())))
            else:
                key.append((type(m).__name__, len(d.get("mods", ()))))
            stack.extend(reversed(d["_modules"].values()))
        key = tuple(key)
        self.__dict__["_cgp_bufs"] = (gen, bufs)
        if not mixture:
            self.__dict__["_cgp_skey"] = (gen, key)     # not through __setattr__
        return key

    def _weights_version(self):
        """(version counter, address) of every Conv2d weight buffer in the tree, read on
        the host (no sync): in-place edits bump a tensor's version without touching
        __setattr__, so the structure key alone cannot see them."""
        memo = self.__dict__.get("_cgp_bufs")
        if memo is None or memo[0] != _GENERATION[0]:
            self.__dict__.pop("_cgp_skey", None)
            self._structure_key()
            memo = self.__dict__["_cgp_bufs"]
        return tuple((b._version, b.data_ptr()) for b in memo[1])

    def set_fusion(self, enabled: bool):
        """Enable/disable op fusion in the pair pipeline (for A/B tests; default on)."""
        for m in self.modules():
            m.__dict__["_cgp_fusion"] = bool(enabled)
        return self

    def set_fused_network(self, enabled: bool):
        """Run off-diagonal forwards on the whole-network kernel (csrc/netfuse.hip: one
        workgroup carries a pair's map through every layer in LDS; default) or on the
        layer-by-layer pipeline (one HBM pass per fused op).  Models the fused kernel
        has no instantiation for use the layer path either way."""
        for m in self.modules():
            m.__dict__["_cgp_netfuse"] = bool(enabled)
        return self

    def _net_plan(self, plan, itemsize):
        """The NetPlan of ``plan`` or None (unsupported program / disabled)."""
        if not getattr(self, "_cgp_netfuse", True):
            return None
        key = ("_net", itemsize)
        if key not in plan.__dict__:
            from .netplan import NetPlan, Unsupported
            try:
                plan.__dict__[key] = NetPlan(plan, itemsize)
            except Unsupported:
                plan.__dict__[key] = None
        return plan.__dict__[key]

    def set_exact_relu(self, enabled: bool):
        """Evaluate the ReLU map op by op exactly like the reference (correctly rounded
        1/sqrt, sqrt, acos, division) instead of the closed form (default; within 1e-14 of
        the exact map, see csrc/relu_poly.h).  For parity studies; ~2x slower."""
        for m in self.modules():
            m.__dict__["_cgp_exact_relu"] = bool(enabled)
        return self

    def forward(self, x, y=None, same=None, diag=False):
        """[N1,C,H,W] × [N2,C,H,W] -> kernel [N1,N2] (or [N1] when diag)."""
        if y is None:                                            # kernels.py:23-26
            assert same is None
            y = x
            same = True
        assert not diag or len(x) == len(y), (
            "diagonal kernels must operate with data of equal length")
        assert 4 == len(x.size())
        assert 4 == len(y.size())
        assert x.size(1) == y.size(1)
        assert x.size(2) == y.size(2)
        assert x.size(3) == y.size(3)
        same = bool(same)
        diag = bool(diag)
        if x.dtype not in (torch.float32, torch.float64):
            raise TypeError(f"cnn_gp kernels compute in float32 or float64, got {x.dtype}")
        out_device = x.device
        if len(x) == 0 or len(y) == 0:
            # the reference's torch ops return the empty [N1, N2] / [N1] result for an empty
            # batch (conv2d on a zero-size batch); there is nothing to evaluate
            return torch.empty((len(x),) if diag else (len(x), len(y)), dtype=x.dtype,
                               device=out_device)
        if x.device.type == "cuda":
            dev = x.device
        else:
            if not torch.cuda.is_available():
                raise RuntimeError("cnn_gp on MI355X needs a HIP device: no GPU is visible "
                                   "(there is no CPU path)")
            dev = torch.device("cuda", torch.cuda.current_device())
        with torch.cuda.device(dev):
            xd = _to_device(x, dev)
            yd = xd if y is x else _to_device(y.to(x.dtype), dev)
            r = self._run(xd, yd, same, diag, _stream_handle(dev))
        return r.to(out_device) if out_device != dev else r

    def _run(self, x, y, same, diag, stream):
        n1, c, h, w = x.shape
        n2 = y.shape[0]
        plan = self._plan(h, w)
        sfx = Plan._sfx(x.dtype)
        lib = N.load()
        net = None if diag else self._net_plan(plan, x.element_size())
        if net is not None and VAR_CHAIN:
            # the same launches from a recipe built once per tile shape and stream (record
            # upload, state buffers and argument structs done once; netplan.TileRecipe)
            rec = net.tile_recipe(plan, x, y, n1, n2, same, plan.flags, stream)
            if rec is not None:
                return rec.run(x, y, stream)
            # every variance map in one launch (cgp_var_chain_*), scaled (1/16) x-side copies
            # included (kernels.py:44-49 moments, then the program on each image)
            fused = plan.run_variances_fused(x, y, n1, n2, same, stream, net.need_var,
                                             net.quarter_vars(x.dtype, plan.flags),
                                             views=False)
            if fused is not None:
                var, qvar = fused
                return net.run(x, y, var, n1, n2, same, stream, plan.flags, qvar=qvar)
        # per-image variances of the inputs (kernels.py:48-49)
        var0 = torch.empty((n1 + n2, h, w), dtype=x.dtype, device=x.device)
        N.check(getattr(lib, f"cgp_moments_var_{sfx}")(N.ptr(x), N.ptr(y), n1, n2, c, h * w,
                                                        N.ptr(var0[:n1]), N.ptr(var0[n1:]),
                                                        stream), "cgp_moments_var")
        if net is not None:                                      # whole-network kernel
            var = plan.run_variances(var0[:n1], var0[n1:], n1, n2, same, stream,
                                     need=net.need_var)
            return net.run(x, y, var, n1, n2, same, stream, plan.flags)
        var = plan.run_variances(var0[:n1], var0[n1:], n1, n2, same, stream)
        xy0 = None
        if not plan.moments_fused:
            nmaps = n1 if diag else n1 * n2
            xy0 = torch.empty((nmaps, h, w), dtype=x.dtype, device=x.device)
            N.check(getattr(lib, f"cgp_moments_xy_{sfx}")(N.ptr(x), N.ptr(y), n1, n2, c, h * w,
                                                           int(diag), N.ptr(xy0), stream),
                    "cgp_moments_xy")
        out = plan.run_pairs(x, y, xy0, var, n1, n2, same, diag, stream)
        if plan.final_hw != (1, 1):                              # kernels.py:53-57
            raise RuntimeError(f"the model's output is {plan.final_hw[0]}x{plan.final_hw[1]}"
                               " per pair, not 1x1: add a final Conv2d covering the map")
        return out.view(n1) if diag else out.view(n1, n2)

    # ---- Gram builds: every image's variance maps once per build -------------------
    # The reference (and forward above) recomputes the per-image variance recursion
    # (kernels.py:44-49, then every layer on the same/diag path) for both image blocks of
    # every tile: a Gram build over B-row tiles of N images does it about 2N/B times per
    # image.  image_variances() runs the whole-network program's variance chain once over
    # an image set; tile_from_variances() evaluates one tile from slices of two such sets.
    # Nothing is kept between builds (the caller holds the maps for one build).

    def image_variances(self, x: torch.Tensor, max_bytes: Optional[int] = None):
        """The variance maps every whole-network tile of images ``x`` ([N, C, H, W], on the
        device) reads, computed in one launch: an object for tile_from_variances, or None
        when the model runs on the layer path (shapes netfuse lacks, CGP_VAR_CHAIN=0, maps
        the chain kernel cannot hold) or the maps would take more than ``max_bytes``
        (default: a quarter of the device's free memory) -- callers then fall back to
        forward() per tile."""
        if x.device.type != "cuda" or x.dtype not in (torch.float32, torch.float64) or \
                x.dim() != 4 or not VAR_CHAIN:
            return None
        n, _, h, w = x.shape
        plan = self._plan(h, w)
        net = self._net_plan(plan, x.element_size())
        if net is None:
            return None
        quarter = net.quarter_vars(x.dtype, plan.flags)
        chain = plan._var_chain(set(net.need_var), set(quarter) & set(net.need_var), x.device)
        if chain is None:
            return None
        size = n * (chain["total"] + chain["qtotal"]) * x.element_size()
        if max_bytes is None:
            max_bytes = torch.cuda.mem_get_info(x.device)[0] // 4
        if size > max_bytes:
            return None
        x = x.contiguous()
        with torch.cuda.device(x.device):
            fused = plan.run_variances_fused(x, x, n, n, True, _stream_handle(x.device),
                                             net.need_var, quarter)
        if fused is None:
            return None
        var, qvar = fused
        return _ImageVariances(x, {v: xx for v, (xx, _) in var.items()}, dict(qvar),
                               (h, w, x.dtype, plan.flags, self._weights_version()))

    def tile_from_variances(self, vx: "_ImageVariances", i0: int, i1: int,
                            vy: "_ImageVariances", j0: int, j1: int, same: bool,
                            out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """K[i0:i1, j0:j1] of vx's images against vy's, equal to
        forward(vx.images[i0:i1], vy.images[j0:j1], same, False) (same: a diagonal tile,
        the same rows of one set).  ``out``: an [i1 - i0, j1 - j0] row-major view of the
        images' dtype to write into (e.g. a tile of the Gram matrix)."""
        if vx.key != vy.key:
            raise ValueError("tile_from_variances: the two image sets were prepared for "
                             "different shapes, dtypes or ReLU modes")
        if same and (vx is not vy or (i0, i1) != (j0, j1)):
            raise ValueError("a diagonal tile takes the same rows of one image set")
        # the kernel indexes the sliced maps by the tile's extents: they must be in range
        if not (0 <= i0 < i1 <= len(vx) and 0 <= j0 < j1 <= len(vy)):
            raise ValueError(f"tile rows [{i0}, {i1}) x cols [{j0}, {j1}) outside the image "
                             f"sets ({len(vx)}, {len(vy)})")
        h, w, dtype, flags, wver = vx.key
        plan = self._plan(h, w)
        if plan.flags != flags:
            raise ValueError("tile_from_variances: the model's ReLU mode changed since "
                             "image_variances")
        if self._weights_version() != wver:
            raise ValueError("tile_from_variances: a Conv2d weight buffer changed since "
                             "image_variances (bind the image sets again)")
        net = self._net_plan(plan, torch.empty((), dtype=dtype).element_size())
        x, y = vx.images[i0:i1], vy.images[j0:j1]
        var = {v: (m[i0:i1], vy.var[v][j0:j1]) for v, m in vx.var.items()}
        qvar = {v: q[i0:i1] for v, q in vx.qvar.items()}
        with torch.cuda.device(x.device):
            return net.run(x, y, var, i1 - i0, j1 - j0, same, _stream_handle(x.device),
                           flags, out=out, qvar=qvar or None)

    def layers(self):
        return 0


class Conv2d(NNGPKernel):
    """kernels.py:60-98 — constant k×k kernel of value var_weight/k², plus var_bias."""

    def __init__(self, kernel_size, stride=1, padding="same", dilation=1,
                 var_weight=1., var_bias=0., in_channel_multiplier=1,
                 out_channel_multiplier=1):
        super().__init__()
        self.kernel_size = kernel_size
        self.stride = stride
        self.dilation = dilation
        self.var_weight = var_weight
        self.var_bias = var_bias
        self.kernel_has_row_of_zeros = False
        self._padding_arg = padding
        if padding == "same":
            self.padding = dilation * (kernel_size // 2)
            self.kernel_has_row_of_zeros = kernel_size % 2 == 0
        else:
            self.padding = padding
        # the reference's kernel buffer: default dtype (float32), so model.double()
        # yields float32-rounded weights — kept for identical numerics and for
        # .cuda()/.double() semantics
        side = kernel_size + 1 if self.kernel_has_row_of_zeros else kernel_size
        kernel = torch.ones(1, 1, side, side)
        if self.kernel_has_row_of_zeros:
            kernel[:, :, 0, :] = 0.
            kernel[:, :, :, 0] = 0.
        self.register_buffer("kernel", kernel * (self.var_weight / self.kernel_size ** 2))
        self.in_channel_multiplier = in_channel_multiplier
        self.out_channel_multiplier = out_channel_multiplier

    def layers(self):
        return 1

    def extra_repr(self):
        return (f"kernel_size={self.kernel_size}, stride={self.stride}, "
                f"padding={self.padding}, dilation={self.dilation}, "
                f"var_weight={self.var_weight}, var_bias={self.var_bias}")


class ReLU(NNGPKernel):
    """kernels.py:128-165 — the arc-cosine covariance map (device: relu_cov)."""
    f32_tiny = np.finfo(np.float32).tiny

    def layers(self):
        return 0


class Sequential(NNGPKernel):
    """kernels.py:178-200."""

    def __init__(self, *mods):
        super().__init__()
        self.mods = mods
        for idx, mod in enumerate(mods):
            self.add_module(str(idx), mod)

    def layers(self):
        return sum(mod.layers() for mod in self.mods)


class Mixture(NNGPKernel):
    """kernels.py:203-229 — softmax(logit)-weighted sum of branches."""

    def __init__(self, mods, logit_proportions=None):
        super().__init__()
        self.mods = mods
        for idx, mod in enumerate(mods):
            self.add_module(str(idx), mod)
        if logit_proportions is None:
            logit_proportions = torch.zeros(len(mods))
        self.logit = nn.Parameter(logit_proportions)

    def proportions(self):
        """softmax of the logits in their own dtype (kernels.py:221), as floats."""
        with torch.no_grad():
            lg = self.logit.detach().cpu()
            return [float(v) for v in torch.softmax(lg, dim=0)]

    def layers(self):
        return max(mod.layers() for mod in self.mods)


class Sum(NNGPKernel):
    """kernels.py:246-260 — elementwise sum of the branches' outputs."""

    def __init__(self, mods):
        super().__init__()
        self.mods = mods
        for idx, mod in enumerate(mods):
            self.add_module(str(idx), mod)

    def layers(self):
        return max(mod.layers() for mod in self.mods)


def resnet_block(stride=1, projection_shortcut=False, multiplier=1):
    """kernels.py:274-296."""
    if stride == 1 and not projection_shortcut:
        return Sum([
            Sequential(),
            Sequential(
                ReLU(),
                Conv2d(3, stride=stride, in_channel_multiplier=multiplier,
                       out_channel_multiplier=multiplier),
                ReLU(),
                Conv2d(3, in_channel_multiplier=multiplier, out_channel_multiplier=multiplier),
            )
        ])
    return Sequential(
        ReLU(),
        Sum([
            Conv2d(1, stride=stride, in_channel_multiplier=multiplier // stride,
                   out_channel_multiplier=multiplier),
            Sequential(
                Conv2d(3, stride=stride, in_channel_multiplier=multiplier // stride,
                       out_channel_multiplier=multiplier),
                ReLU(),
                Conv2d(3, in_channel_multiplier=multiplier, out_channel_multiplier=multiplier),
            )
        ]),
    )

