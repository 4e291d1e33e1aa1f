"""ResNet-GP on MNIST, splits 50k/10k/10k (reference configs/mnist.py); the
architecture is the one of mnist_as_tf."""
from cnn_gp import Conv2d, ReLU, Sequential

from ._resnet import resnet_body

train_range = range(50000)
validation_range = range(50000, 60000)
test_range = range(60000, 70000)

dataset_name = "MNIST"
model_name = "ResNet"
dataset = "MNIST"
transforms = []
epochs = 0
in_channels = 1
out_channels = 10

initial_model = Sequential(
    *resnet_body(),
    Conv2d(kernel_size=7, padding=0, in_channel_multiplier=4, out_channel_multiplier=4),
    ReLU(),
    Conv2d(kernel_size=1, padding=0, in_channel_multiplier=4),
)
