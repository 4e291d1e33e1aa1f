"""The ResNet-GP body shared by configs/mnist.py, mnist_as_tf.py and cifar10.py
(reference configs/mnist_as_tf.py:20-42): a 3x3 stem and three stages of five
resnet_blocks, the first of each stage a projection block (strides 1, 2, 2)."""
from cnn_gp import Conv2d, resnet_block


def resnet_body():
    mods = [Conv2d(kernel_size=3)]
    for stage, stride in enumerate((1, 2, 2)):
        mult = 2 ** stage
        mods.append(resnet_block(stride=stride, projection_shortcut=True, multiplier=mult))
        mods += [resnet_block(stride=1, projection_shortcut=False, multiplier=mult)
                 for _ in range(4)]
    return mods
