"""Parallel layout: mp-major 2-D (DP x TP) rank grid, TP collects, DP grad sync."""
from .layout import (  # noqa: F401
    get_info,
    naive_collect_backward_output,
    naive_collect_backward_x,
    naive_collect_forward_input,
    naive_collect_forward_output,
    device_group_for,
)
