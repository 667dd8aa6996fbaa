"""2-D grid (reference tests/test_get_info.py): exactly 8 ranks, mp=4, dp=2.

Run: ``scripts/mpirun -n 8 python -m pytest tests/test_get_info.py --with-mpi``
(tests/test_reference_suite.py does this from a plain pytest run)."""
import numpy as np
import pytest

from collective_communication_mpi_amd import MPI
from model.func_impl import get_info

MP, DP = 4, 2
ROWS = np.arange(80).reshape(8, 10)


def _run(fc_layer, in_dim, out_dim, want_in, want_out):
    comm = MPI.COMM_WORLD
    rank = comm.Get_rank()
    assert comm.Get_size() == MP * DP, "this test needs exactly 8 ranks"
    mp_idx, dp_idx, mp_comm, dp_comm, pin, pout = get_info(
        comm=comm, rank=rank, mp_size=MP, dp_size=DP, fc_layer=fc_layer, in_dim=in_dim, out_dim=out_dim)
    assert (mp_idx, dp_idx) == (rank % MP, rank // MP)
    assert (pin, pout) == (want_in, want_out)
    mine = ROWS[rank]
    mp_sum = np.empty_like(mine)
    dp_sum = np.empty_like(mine)
    mp_comm.Allreduce(mine, mp_sum, op=MPI.SUM)
    dp_comm.Allreduce(mine, dp_sum, op=MPI.SUM)
    # mp group = the 4 consecutive ranks of this replica; dp group = ranks with equal mp_idx
    np.testing.assert_allclose(mp_sum, ROWS[dp_idx * MP:(dp_idx + 1) * MP].sum(axis=0))
    np.testing.assert_allclose(dp_sum, ROWS[mp_idx::MP].sum(axis=0))


@pytest.mark.mpi
def test_fc_q():
    _run("fc_q", 768, 256, 768, 256 // 4)


@pytest.mark.mpi
def test_fc_o():
    _run("fc_o", 256, 10, 256 // 4, 10)


@pytest.mark.mpi
def test_bad_layer_raises_everywhere():
    with pytest.raises(ValueError):
        get_info(MPI.COMM_WORLD, MPI.COMM_WORLD.Get_rank(), MP, DP, "fc_x", 8, 8)
