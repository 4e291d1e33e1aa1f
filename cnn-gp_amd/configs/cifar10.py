"""ResNet-GP on CIFAR-10 (reference configs/cifar10.py): 3x32x32 inputs, final 8x8 conv
then two 1x1 convs around a ReLU."""
from cnn_gp import Conv2d, ReLU, Sequential

from ._resnet import resnet_body

train_range = range(40000)
validation_range = range(40000, 50000)
test_range = range(50000, 60000)

kernel_batch_size = 350

dataset_name = "CIFAR10"
model_name = "ResNet"
in_channels = 3
dataset = "CIFAR10"
transforms = []
epochs = 0

initial_model = Sequential(
    *resnet_body(),
    Conv2d(kernel_size=8, padding=0, in_channel_multiplier=4, out_channel_multiplier=4),
    Conv2d(kernel_size=1, padding=0, in_channel_multiplier=4, out_channel_multiplier=4),
    ReLU(),
    Conv2d(kernel_size=1, padding=0, in_channel_multiplier=4),
)
