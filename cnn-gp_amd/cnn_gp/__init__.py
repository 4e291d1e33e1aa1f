"""cnn_gp on MI355X — drop-in for the reference package's kernel/tile/solve surface.

``from cnn_gp import Conv2d, ReLU, Sequential, Sum, resnet_block`` works as in the
reference's configs (configs/*.py:2-16); ``model(x, x2, same, diag)`` evaluates the
NNGP kernel with hand-written HIP kernels (libcnngp.so).
"""
from . import kernels, data, kernel_save_tools, solve, gram
from .kernels import *  # noqa: F401,F403
from .data import *  # noqa: F401,F403
from .kernel_save_tools import *  # noqa: F401,F403
from .solve import *  # noqa: F401,F403

__all__ = kernels.__all__ + data.__all__ + kernel_save_tools.__all__ + solve.__all__
