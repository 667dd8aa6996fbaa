"""Data layer: DP sharding and synthetic MNIST-shaped data."""
from .preprocess import split_data, synthetic_mnist  # noqa: F401
