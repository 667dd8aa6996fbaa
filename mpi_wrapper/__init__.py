"""Reference import path ``from mpi_wrapper import Communicator`` (mpi_wrapper/__init__.py:1)."""
from collective_communication_mpi_amd.comm import Communicator  # noqa: F401
