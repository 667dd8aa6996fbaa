"""Loader for the in-tree native extensions (builds them on first use if absent).

``_host`` (C++ shared-memory plane) has no GPU dependency.  ``_device`` (HIP
kernels + device communicator) is loaded only after ``torch`` so that it binds
to the HIP runtime / RCCL that torch already mapped into the process (same
SONAMEs), never to a second copy.
"""
from __future__ import annotations

import importlib
import os
import sys

_host_mod = None
_device_mod = None


def host():
    global _host_mod
    if _host_mod is None:
        from . import _build

        if os.environ.get("CCMPI_NO_AUTOBUILD") != "1":
            _build.build_host()
        _host_mod = importlib.import_module(f"{__package__}._host")
    return _host_mod


def device():
    """Return the `_device` extension; raises if it cannot be loaded."""
    global _device_mod
    if _device_mod is None:
        import torch  # noqa: F401  - must be loaded first (shared HIP runtime)
        from . import _build

        if os.environ.get("CCMPI_NO_AUTOBUILD") != "1":
            _build.build_device()
        _device_mod = importlib.import_module(f"{__package__}._device")
    return _device_mod


def device_available() -> bool:
    try:
        import torch

        return bool(torch.cuda.is_available()) and device() is not None
    except Exception:  # pragma: no cover - reported by callers
        return False
