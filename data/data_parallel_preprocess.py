"""Reference import path ``data.data_parallel_preprocess`` (data/data_parallel_preprocess.py)."""
from collective_communication_mpi_amd.data.preprocess import split_data, synthetic_mnist  # noqa: F401
