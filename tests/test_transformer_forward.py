"""fc_o forward collects (reference tests/test_transformer_forward.py): exactly
4 ranks; each rank holds a NON-contiguous last-axis slice of a (4, 8, 8)
float64 tensor and the collect must rebuild the whole tensor, dtype preserved."""
import numpy as np
import pytest

from collective_communication_mpi_amd import MPI
from model.func_impl import naive_collect_forward_input, naive_collect_forward_output

GLOBAL = np.arange(4 * 8 * 8, dtype=np.float64).reshape(4, 8, 8)


def _shard():
    comm = MPI.COMM_WORLD
    r = comm.Get_rank()
    assert comm.Get_size() == 4, "this test needs exactly 4 ranks"
    k = GLOBAL.shape[2] // 4
    return comm, GLOBAL[:, :, r * k:(r + 1) * k]


@pytest.mark.mpi
@pytest.mark.parametrize("fn,kw", [(naive_collect_forward_input, "x"), (naive_collect_forward_output, "out")])
def test_collect_forward(fn, kw):
    comm, x = _shard()
    assert not x.flags.c_contiguous
    got = fn(**{kw: x, "mp_comm": comm, "mp_size": 4})
    assert got.dtype == x.dtype
    np.testing.assert_allclose(got, GLOBAL)
