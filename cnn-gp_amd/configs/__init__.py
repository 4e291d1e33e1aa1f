"""Experiment configs restated for the MI355X build (reference: configs/*.py).

Same module attributes as the reference (``initial_model``, ``train_range``,
``validation_range``, ``test_range``, ``dataset_name``, ...), built from this package's
``cnn_gp`` classes.  ``dataset`` names the local-file reader instead of a torchvision
class (this build never downloads).
"""
