"""Reference import path ``model.func_impl`` (model/func_impl.py)."""
from collective_communication_mpi_amd.parallel.layout import (  # noqa: F401
    get_info,
    naive_collect_backward_output,
    naive_collect_backward_x,
    naive_collect_forward_input,
    naive_collect_forward_output,
)
