"""DP data sharding (reference data/data_parallel_preprocess.py:3-59) and the
synthetic stand-in for the MNIST file the reference does not ship
(.MISSING_LARGE_BLOBS:1 lists data/MNISTdata.hdf5).
"""
from __future__ import annotations

import numpy as np


def split_data(x_train, y_train, mp_size: int, dp_size: int, rank: int):
    """Contiguous, un-shuffled split across DP groups; every MP rank of a DP
    group gets the same block (``dp_group_idx = rank // mp_size``).  Returns views.
    Works on NumPy arrays and torch tensors alike (slicing along axis 0)."""
    data_size = x_train.shape[0]
    split_size = data_size // dp_size
    dp_group_idx = rank // mp_size
    start_idx = dp_group_idx * split_size
    end_idx = (dp_group_idx + 1) * split_size
    return x_train[start_idx:end_idx], y_train[start_idx:end_idx]


def synthetic_mnist(n: int = 60000, seed: int = 0, feature_dim: int = 784, classes: int = 10):
    """MNIST-shaped synthetic data: ``x`` (n, 784) float32 in [0, 1), ``y`` (n,) int32.

    Labels are a deterministic function of the pixels (argmax of a fixed random
    projection) so a model can actually learn them."""
    rng = np.random.default_rng(seed)
    x = rng.random((n, feature_dim), dtype=np.float32)
    proj = np.random.default_rng(seed + 1).standard_normal((feature_dim, classes)).astype(np.float32)
    y = np.argmax(x @ proj, axis=1).astype(np.int32)
    return x, y
