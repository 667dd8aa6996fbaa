"""Model families of the harness."""
from .mnist_tp import LayerConfig, MnistTPLayer, patchify  # noqa: F401
