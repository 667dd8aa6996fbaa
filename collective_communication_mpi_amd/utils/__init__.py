"""Tracing, timing and small helpers."""
from .trace import TRACE, trace_call  # noqa: F401
