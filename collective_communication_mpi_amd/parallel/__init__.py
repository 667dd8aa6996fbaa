"""Parallel layout: mp-major 2-D (DP x TP) rank grid, TP collects, DP grad sync,
Megatron-style tensor-parallel layers and bucketed data parallelism for any torch model."""
from .layout import (  # noqa: F401
    get_info,
    naive_collect_backward_output,
    naive_collect_backward_x,
    naive_collect_forward_input,
    naive_collect_forward_output,
    device_group_for,
)
from .ddp import DistributedDataParallel, ddp_wrap  # noqa: F401,E402
from .tensor_parallel import (  # noqa: F401,E402
    ColumnParallelLinear,
    ParallelSwiGLUMLP,
    RowParallelLinear,
    all_reduce,
    all_reduce_,
    copy_to_tensor_parallel_region,
    gather_from_tensor_parallel_region,
    reduce_from_tensor_parallel_region,
    scatter_to_tensor_parallel_region,
)
