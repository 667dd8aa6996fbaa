"""collective_communication_mpi_amd — MI355X-native collective communication
library and 2-D (DP x TP) training harness.

Capabilities of the teaching reference ``anaykulkarni/collective-communication-mpi``
(mpi4py + NumPy) re-designed for AMD Instinct MI355X (gfx950 / CDNA4):

* ``mpi``       — mpi4py-compatible ``MPI`` namespace over a C++ shared-memory host plane
* ``Communicator`` — reference API + byte accounting, CPU and GPU buffers
* ``device``    — hand-written CDNA4 collectives over IPC-mapped xGMI peer memory,
                  RCCL library baseline, RCCL-P2P ring / RHD schedules
* ``parallel``  — mp-major DP x TP grid, naive + Megatron TP collects, DP grad buckets
* ``models``    — TP transformer layer on MNIST-shaped data (MFMA bf16 GEMMs)
* ``launch``    — ``mpirun``-compatible launcher (``scripts/mpirun``)
"""
from . import mpi  # noqa: F401
from . import mpi as MPI  # noqa: F401
from .comm import Communicator  # noqa: F401
from .data.preprocess import split_data, synthetic_mnist  # noqa: F401
from .parallel.layout import (  # noqa: F401
    get_info,
    naive_collect_backward_output,
    naive_collect_backward_x,
    naive_collect_forward_input,
    naive_collect_forward_output,
)

__version__ = "0.1.0"
