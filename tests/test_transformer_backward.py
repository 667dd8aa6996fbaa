"""fc_o backward collects (reference tests/test_transformer_backward.py): exactly 4 ranks.

* backward_output: rank r gets columns [2r, 2r+2) of a (1, 4, 8) gradient;
* backward_x: each rank's (1, 3, 8) grad_x is rank r's slice of a (4, 3, 8)
  tensor; the result is the sum over ranks split into 4 blocks of width 2."""
import numpy as np
import pytest

from collective_communication_mpi_amd import MPI
from model.func_impl import naive_collect_backward_output, naive_collect_backward_x


@pytest.mark.mpi
def test_fc2_naive_mp_backward_output_3d():
    r = MPI.COMM_WORLD.Get_rank()
    g = np.arange(32).reshape(1, 4, 8).astype(np.float64)
    out = naive_collect_backward_output(output_grad=g, mp_group_idx=r, mp_size=4)
    assert out.dtype == g.dtype
    np.testing.assert_allclose(out, g[:, :, 2 * r:2 * r + 2])


@pytest.mark.mpi
def test_fc2_naive_mp_backward_x_3d():
    comm = MPI.COMM_WORLD
    r = comm.Get_rank()
    assert comm.Get_size() == 4, "this test needs exactly 4 ranks"
    full = np.arange(4 * 3 * 8).reshape(4, 3, 8).astype(np.float64)
    out = naive_collect_backward_x(grad_x=full[r:r + 1], mp_comm=comm, mp_size=4)
    assert out.dtype == np.float64
    np.testing.assert_allclose(out, full.sum(axis=0, keepdims=True)[:, :, 2 * r:2 * r + 2])
