"""Architecture specs of the reference configs, restated for the oracle — TEST
INFRASTRUCTURE ONLY (see oracle/nngp_oracle.py's header for the import rule).

Each function restates one /root/reference/configs/*.py ``initial_model`` as a nested
oracle spec.  ``resnet_block`` restates cnn_gp/kernels.py:274-296.
"""
from __future__ import annotations


def conv(kernel_size, stride=1, padding="same", dilation=1, var_weight=1.0, var_bias=0.0):
    return ("conv", dict(kernel_size=kernel_size, stride=stride, padding=padding,
                         dilation=dilation, var_weight=var_weight, var_bias=var_bias))


RELU = ("relu",)


def seq(*mods):
    return ("seq", list(mods))


def resnet_block(stride=1, projection_shortcut=False):
    """kernels.py:274-296 (channel multipliers do not affect the kernel)."""
    if stride == 1 and not projection_shortcut:
        return ("sum", [seq(), seq(RELU, conv(3, stride=stride), RELU, conv(3))])
    return seq(RELU, ("sum", [conv(1, stride=stride),
                              seq(conv(3, stride=stride), RELU, conv(3))]))


def mnist_paper_convnet_gp():
    """configs/mnist_paper_convnet_gp.py:16-30."""
    var_bias, var_weight = 7.86, 2.79
    layers = []
    for _ in range(7):
        layers += [conv(7, padding="same", var_weight=var_weight * 7 ** 2, var_bias=var_bias),
                   RELU]
    return seq(*layers, conv(28, padding=0, var_weight=var_weight, var_bias=var_bias))


def mnist_paper_residual_cnn_gp():
    """configs/mnist_paper_residual_cnn_gp.py:30-45 (sums after the ReLU, as published)."""
    var_bias, var_weight = 4.69, 7.27
    blocks = [("sum", [seq(), seq(conv(4, padding="same", var_weight=var_weight * 4 ** 2,
                                       var_bias=var_bias), RELU)]) for _ in range(8)]
    return seq(*blocks,
               conv(4, padding="same", var_weight=var_weight * 4 ** 2, var_bias=var_bias),
               RELU,
               conv(28, padding=0, var_weight=var_weight, var_bias=var_bias))


def _resnet_body():
    mods = [conv(3)]
    for stride in (1, 2, 2):
        mods.append(resnet_block(stride=stride, projection_shortcut=True))
        mods += [resnet_block(stride=1, projection_shortcut=False) for _ in range(4)]
    return mods


def mnist_as_tf():
    """configs/mnist_as_tf.py:20-49 (identical architecture in configs/mnist.py:16-45)."""
    return seq(*_resnet_body(), conv(7, padding=0), RELU, conv(1, padding=0))


def cifar10():
    """configs/cifar10.py:16-47."""
    return seq(*_resnet_body(), conv(8, padding=0), conv(1, padding=0), RELU,
               conv(1, padding=0))


CONFIGS = {
    "mnist_paper_convnet_gp": mnist_paper_convnet_gp,
    "mnist_paper_residual_cnn_gp": mnist_paper_residual_cnn_gp,
    "mnist_as_tf": mnist_as_tf,
    "mnist": mnist_as_tf,
    "cifar10": cifar10,
}

# input geometry of each config (channels, side)
GEOMETRY = {
    "mnist_paper_convnet_gp": (1, 28),
    "mnist_paper_residual_cnn_gp": (1, 28),
    "mnist_as_tf": (1, 28),
    "mnist": (1, 28),
    "cifar10": (3, 32),
}
