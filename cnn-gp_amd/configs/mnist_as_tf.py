"""ResNet-GP on MNIST with the original TensorFlow experiments' splits
(reference configs/mnist_as_tf.py)."""
from cnn_gp import Conv2d, ReLU, Sequential

from ._resnet import resnet_body

train_range = range(5000, 55000)
validation_range = list(range(55000, 60000)) + list(range(0, 5000))
test_range = range(60000, 70000)

dataset_name = "MNIST"
model_name = "ResNet"
dataset = "MNIST"
transforms = []
epochs = 0
in_channels = 1
out_channels = 10

# the final 7x7 conv replaces average pooling; no nonlinearity before it
initial_model = Sequential(
    *resnet_body(),
    Conv2d(kernel_size=7, padding=0, in_channel_multiplier=4, out_channel_multiplier=4),
    ReLU(),
    Conv2d(kernel_size=1, padding=0, in_channel_multiplier=4),
)
