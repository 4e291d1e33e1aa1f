"""The best random-searched residual CNN GP of the paper (reference
configs/mnist_paper_residual_cnn_gp.py).  As published, each residual branch is summed
AFTER its ReLU (the reference replicates that choice, and so does this config)."""
from cnn_gp import Conv2d, ReLU, Sequential, Sum

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

var_bias = 4.69
var_weight = 7.27


def _branch():
    return Sequential(Conv2d(kernel_size=4, padding="same", var_weight=var_weight * 4 ** 2,
                             var_bias=var_bias), ReLU())


initial_model = Sequential(
    *[Sum([Sequential(), _branch()]) for _ in range(8)],
    Conv2d(kernel_size=4, padding="same", var_weight=var_weight * 4 ** 2, var_bias=var_bias),
    ReLU(),
    Conv2d(kernel_size=28, padding=0, var_weight=var_weight, var_bias=var_bias),
)
