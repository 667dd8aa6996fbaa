"""DP sharding (reference tests/test_data_split.py): serial, one process
simulating every rank.  Same cases: (mp, dp) = (2,1), (1,2), (2,2), (2,4) on
8 samples of 2x2 float64 with 2-vector labels."""
import numpy as np
import pytest

from data.data_parallel_preprocess import split_data

X = np.arange(1.0, 33.0).reshape(8, 2, 2)
Y = np.arange(1.0, 17.0).reshape(8, 2)


def _expected_blocks(mp, dp):
    per = X.shape[0] // dp
    return {r: (X[(r // mp) * per:(r // mp + 1) * per], Y[(r // mp) * per:(r // mp + 1) * per])
            for r in range(mp * dp)}


@pytest.mark.parametrize("mp,dp", [(2, 1), (1, 2), (2, 2), (2, 4)])
def test_split(mp, dp):
    for rank, (ex, ey) in _expected_blocks(mp, dp).items():
        gx, gy = split_data(x_train=X, y_train=Y, mp_size=mp, dp_size=dp, rank=rank)
        assert gx.shape[0] * dp == X.shape[0]
        assert gy.shape[0] * dp == Y.shape[0]
        np.testing.assert_allclose(gx, ex)
        np.testing.assert_allclose(gy, ey)


def test_mp_ranks_share_block_and_views():
    gx0, _ = split_data(X, Y, mp_size=2, dp_size=2, rank=2)
    gx1, _ = split_data(X, Y, mp_size=2, dp_size=2, rank=3)
    assert np.shares_memory(gx0, X)  # views, no copy (reference semantics)
    np.testing.assert_array_equal(gx0, gx1)
    np.testing.assert_array_equal(gx0, X[4:])


def test_synthetic_mnist_shape():
    from collective_communication_mpi_amd.data import synthetic_mnist

    x, y = synthetic_mnist(512, seed=3)
    assert x.shape == (512, 784) and x.dtype == np.float32
    assert y.shape == (512,) and y.dtype == np.int32 and 0 <= y.min() and y.max() < 10
