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
import os as _os

# Kernel arguments in device memory: every kernel's first argument fetch then comes from HBM /
# L2 instead of the host-side kernarg pool.  Measured on the fused attention kernel (one launch
# per forward step): 1.1-1.2 us less per launch (profiles/r6_attn/README.md).  Read by the HIP
# runtime at its initialisation, so it must be set before the first GPU call; an explicit
# setting wins.
_os.environ.setdefault("HIP_FORCE_DEV_KERNARG", "1")

from . import mpi  # noqa: E402,F401
from . import mpi as MPI  # noqa: E402,F401
from .comm import Communicator  # noqa: E402,F401
from .data.preprocess import split_data, synthetic_mnist  # noqa: E402,F401
from .parallel.layout import (  # noqa: E402,F401
    get_info,
    naive_collect_backward_output,
    naive_collect_backward_x,
    naive_collect_forward_input,
    naive_collect_forward_output,
)

__version__ = "0.1.0"
