"""ctypes binding of libcnngp.so (include/cnngp.h).

The library is built in-tree (``cnn-gp_amd/lib/libcnngp.so``, see csrc/Makefile or
``__graft_entry__.build()``).  There is no fallback: if the library is missing or fails
to load, every compute call raises ``RuntimeError`` naming the problem.
"""
from __future__ import annotations

import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("CNNGP_LIB",
                          os.path.join(os.path.dirname(_HERE), "lib", "libcnngp.so"))

CGP_ABI_VERSION = 11
CGP_FLAG_EXACT_RELU = 1
CGP_FLAG_GENERIC_CONV = 2
CGP_FLAG_NET_DUAL = 4
CGP_PRE_NONE, CGP_PRE_RELU, CGP_PRE_MOMENTS = 0, 1, 2
CGP_POST_NONE, CGP_POST_RELU = 0, 1
CGP_NET_CONV, CGP_NET_RELU, CGP_NET_MOMENTS, CGP_NET_LINEAR = 0, 1, 2, 3
CGP_NET_LOAD, CGP_NET_STORE = 4, 5
CGP_NET_CODE_HS_CLEAN = 0x100
CGP_NET_CODE_SUM = 0x200         # conv: outputs summed for the next op's reduction (cnngp.h)
CGP_NET_CODE_FROM_SUM = 0x400    # reduction: reads the previous conv's partial sums
CGP_NET_CODE_GEOMETRY = 0xff
CGP_VAR_MOMENTS, CGP_VAR_CONV, CGP_VAR_HALF, CGP_VAR_SUM = 0, 1, 2, 3

_vp = ctypes.c_void_p
_i64 = ctypes.c_int64
_i32 = ctypes.c_int32
_f64 = ctypes.c_double


class ConvArgs(ctypes.Structure):
    """Mirror of cgp_conv_args (include/cnngp.h)."""
    _fields_ = [
        ("in_", _vp), ("in_y", _vp), ("out", _vp), ("addend", _vp),
        ("pre_xx", _vp), ("pre_yy", _vp), ("post_xx", _vp), ("post_yy", _vp),
        ("nmaps", _i64), ("n1", _i64), ("n2", _i64),
        ("h", _i32), ("w", _i32), ("ho", _i32), ("wo", _i32),
        ("taps", _i32), ("offset", _i32), ("stride", _i32), ("dilation", _i32),
        ("channels", _i32), ("pre", _i32), ("post", _i32), ("same", _i32), ("diag", _i32),
        ("maps_per_block", _i32), ("flags", _i32), ("reserved", _i32),
        ("weight", _f64), ("bias", _f64),
    ]


class ReluArgs(ctypes.Structure):
    """Mirror of cgp_relu_args (include/cnngp.h)."""
    _fields_ = [
        ("xy", _vp), ("out", _vp), ("addend", _vp), ("xx", _vp), ("yy", _vp),
        ("nmaps", _i64), ("n1", _i64), ("n2", _i64),
        ("hw", _i32), ("same", _i32), ("diag", _i32), ("flags", _i32),
    ]


class NetOp(ctypes.Structure):
    """Mirror of cgp_net_op (include/cnngp.h)."""
    _fields_ = [
        ("kind", _i32), ("code", _i32), ("src", _i32), ("dst", _i32), ("add", _i32),
        ("ws_in", _i32), ("ws_out", _i32), ("relu", _i32), ("h", _i32), ("w", _i32),
        ("div_m", ctypes.c_uint32), ("div_s", ctypes.c_uint32),
        ("dst2", _i32), ("zero_halo", _i32),
        ("weight", _f64), ("bias", _f64), ("var_x", _vp), ("var_y", _vp),
        ("var2_x", _vp), ("var2_y", _vp),
    ]


class VarOp(ctypes.Structure):
    """Mirror of cgp_var_op (include/cnngp.h)."""
    _fields_ = [
        ("kind", _i32), ("dst", _i32), ("src", _i32 * 4),
        ("h", _i32), ("w", _i32), ("ho", _i32), ("wo", _i32),
        ("taps", _i32), ("offset", _i32), ("stride", _i32), ("dilation", _i32),
        ("store", _i64), ("qstore", _i64),
        ("weight", _f64), ("bias", _f64), ("coef", _f64 * 4),
    ]


class VarArgs(ctypes.Structure):
    """Mirror of cgp_var_args (include/cnngp.h)."""
    _fields_ = [
        ("x", _vp), ("y", _vp), ("out", _vp), ("ops", _vp),
        ("n1", _i64), ("n2", _i64), ("store_total", _i64),
        ("nops", _i32), ("channels", _i32), ("h", _i32), ("w", _i32),
        ("lds_elems", _i32), ("scratch", _i32),
    ]


class NetArgs(ctypes.Structure):
    """Mirror of cgp_net_args (include/cnngp.h)."""
    _fields_ = [
        ("x", _vp), ("y", _vp), ("out", _vp), ("kdiag", _vp), ("ops", _vp),
        ("n1", _i64), ("n2", _i64), ("ldo", _i64),
        ("nops", _i32), ("channels", _i32), ("h", _i32), ("w", _i32),
        ("same", _i32), ("final_slot", _i32), ("hs", _i32), ("lds_elems", _i32),
        ("flags", _i32), ("pairs", _i32), ("unit_begin", _i64), ("unit_end", _i64),
        ("final_stage", _i32), ("program", _i32), ("part", _i32),
    ]


def make_fastdiv(d: int):
    """(m, s) of the multiply-high divisor the kernels use (cgp_common.h FastDiv)."""
    s = 0
    while (1 << s) < d:
        s += 1
    m = (((1 << 32) * ((1 << s) - d)) // d + 1) & 0xFFFFFFFF
    return m, s


# name -> (restype, argtypes)
SIGNATURES = {
    "cgp_abi_version": (_i32, []),
    "cgp_net_xvar_scale": (ctypes.c_double, []),
    "cgp_last_error": (ctypes.c_char_p, []),
    "cgp_conv_args_size": (ctypes.c_size_t, []),
    "cgp_relu_args_size": (ctypes.c_size_t, []),
    "cgp_device_count": (_i32, []),
    "cgp_selftest": (_i32, []),
    "cgp_moments_xy_f64": (_i32, [_vp, _vp, _i64, _i64, _i32, _i32, _i32, _vp, _vp]),
    "cgp_moments_xy_f32": (_i32, [_vp, _vp, _i64, _i64, _i32, _i32, _i32, _vp, _vp]),
    "cgp_moments_var_f64": (_i32, [_vp, _vp, _i64, _i64, _i32, _i32, _vp, _vp, _vp]),
    "cgp_moments_var_f32": (_i32, [_vp, _vp, _i64, _i64, _i32, _i32, _vp, _vp, _vp]),
    "cgp_conv_f64": (_i32, [ctypes.POINTER(ConvArgs), _vp]),
    "cgp_conv_f32": (_i32, [ctypes.POINTER(ConvArgs), _vp]),
    "cgp_relu_f64": (_i32, [ctypes.POINTER(ReluArgs), _vp]),
    "cgp_relu_f32": (_i32, [ctypes.POINTER(ReluArgs), _vp]),
    "cgp_var_relu_f64": (_i32, [_vp, _vp, _i64, _i64, _i32, _i32, _vp, _vp, _vp]),
    "cgp_var_relu_f32": (_i32, [_vp, _vp, _i64, _i64, _i32, _i32, _vp, _vp, _vp]),
    "cgp_axpby_f64": (_i32, [_f64, _vp, _f64, _vp, _vp, _i64, _vp]),
    "cgp_axpby_f32": (_i32, [_f64, _vp, _f64, _vp, _vp, _i64, _vp]),
    "cgp_scale_batch_f64": (_i32, [_i32, _vp, _vp, _vp, _f64, _vp]),
    "cgp_cast_f32_f64": (_i32, [_vp, _vp, _i64, _vp]),
    "cgp_transpose_f64": (_i32, [_vp, _i64, _i64, _vp, _vp]),
    "cgp_chol_solve_f64": (_i32, [_vp, _i64, _i64, _vp, _i64, _i64, _f64,
                                  ctypes.POINTER(_i64), _vp]),
    "cgp_chol_last_phases": (_i32, [_vp, ctypes.POINTER(_f64)]),
    "cgp_chol_solve_f64_timed": (_i32, [_vp, _i64, _i64, _vp, _i64, _i64, _f64,
                                        ctypes.POINTER(_i64), ctypes.POINTER(_f64), _vp]),
    "cgp_gemm_f64": (_i32, [_vp, _vp, _vp, _i64, _i64, _i64, _vp]),
    "cgp_sym_mirror_f64": (_i32, [_vp, _i64, _i64, _vp, _vp]),
    "cgp_sym_residual_f64": (_i32, [_vp, _i64, _i64, _vp, _vp, _vp, _i64, _i64, _vp, _vp]),
    "cgp_argmax_rows_f64": (_i32, [_vp, _i64, _i64, _vp, _vp]),
    "cgp_pred_var_f64": (_i32, [_vp, _i64, _i64, _vp, _i64, _i64, _vp, _vp, _vp]),
    "cgp_net_geometry": (_i32, [_i32] * 7),
    "cgp_net_hs_elems": (_i32, [_i32]),
    "cgp_net_supertile": (_i32, []),
    "cgp_net_units": (_i32, [_i32]),
    "cgp_net_resolution": (_i32, [_i32, _i32]),
    "cgp_net_op_size": (ctypes.c_size_t, []),
    "cgp_net_args_size": (ctypes.c_size_t, []),
    "cgp_net_occupancy": (_i32, [_i32, _i32, _i32, _i32]),
    "cgp_net_program": (_i32, [_vp, _i32, _i32, _i32, _i32, _i32]),
    "cgp_net_validate": (_i32, [_vp, _i32, _i32]),
    "cgp_net_static_lds": (_i32, []),
    "cgp_net_f64": (_i32, [ctypes.POINTER(NetArgs), _vp]),
    "cgp_net_f32": (_i32, [ctypes.POINTER(NetArgs), _vp]),
    "cgp_var_op_size": (ctypes.c_size_t, []),
    "cgp_var_args_size": (ctypes.c_size_t, []),
    "cgp_var_chain_f64": (_i32, [ctypes.POINTER(VarArgs), _vp]),
    "cgp_var_chain_f32": (_i32, [ctypes.POINTER(VarArgs), _vp]),
}

_lib = None
_lib_err = None
_lock = threading.Lock()


def load():
    """Load (once) and return the ctypes library; raise RuntimeError if unavailable."""
    global _lib, _lib_err
    with _lock:
        if _lib is not None:
            return _lib
        if _lib_err is not None:
            raise RuntimeError(_lib_err)
        if not os.path.exists(LIB_PATH):
            _lib_err = (f"libcnngp.so not found at {LIB_PATH}: build it with "
                        "`python -c 'import __graft_entry__ as g; g.build()'` or "
                        "`make -C cnn-gp_amd/csrc` (no CPU fallback exists)")
            raise RuntimeError(_lib_err)
        try:
            lib = ctypes.CDLL(LIB_PATH)
        except OSError as e:
            _lib_err = f"failed to load {LIB_PATH}: {e}"
            raise RuntimeError(_lib_err) from e
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        if lib.cgp_abi_version() != CGP_ABI_VERSION:
            _lib_err = "libcnngp.so ABI version mismatch (rebuild it)"
            raise RuntimeError(_lib_err)
        if lib.cgp_conv_args_size() != ctypes.sizeof(ConvArgs) or \
                lib.cgp_relu_args_size() != ctypes.sizeof(ReluArgs) or \
                lib.cgp_net_op_size() != ctypes.sizeof(NetOp) or \
                lib.cgp_net_args_size() != ctypes.sizeof(NetArgs) or \
                lib.cgp_var_op_size() != ctypes.sizeof(VarOp) or \
                lib.cgp_var_args_size() != ctypes.sizeof(VarArgs):
            _lib_err = "libcnngp.so argument struct layout differs from _native.py"
            raise RuntimeError(_lib_err)
        _lib = lib
        return lib


def check(rc: int, what: str):
    if rc != 0:
        msg = load().cgp_last_error().decode(errors="replace")
        raise RuntimeError(f"{what} failed (code {rc}): {msg}")


def call(name: str, *args):
    lib = load()
    check(getattr(lib, name)(*args), name)


def ptr(t):
    """Device pointer of a torch tensor (None -> NULL)."""
    return None if t is None else ctypes.c_void_p(t.data_ptr())
