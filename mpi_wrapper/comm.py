"""Reference module path ``mpi_wrapper.comm`` (mpi_wrapper/comm.py)."""
from collective_communication_mpi_amd import mpi as MPI  # noqa: F401
from collective_communication_mpi_amd.comm import Communicator  # noqa: F401
