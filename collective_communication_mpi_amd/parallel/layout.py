"""2-D parallel layout helpers (reference model/func_impl.py:1-187), MI355X-native.

Same signatures and results as the reference:

* ``get_info`` — mp-major grid: ``mp_idx = rank % mp``, ``dp_idx = rank // mp``
  (func_impl.py:53-54); ``mp_comm = comm.Split(color=dp_idx, key=mp_idx)``,
  ``dp_comm = comm.Split(color=mp_idx, key=dp_idx)`` (:57-62); fc_q/k/v are
  column-parallel ``(in, out//mp)``, fc_o row-parallel ``(in//mp, out)`` (:65-72).
  Splits are cached per (comm, mp, dp) so repeated per-layer calls do not
  re-split (all ranks call in the same order, so the cache stays collective).
* ``naive_collect_forward_input/output`` — last-axis all-gather (:76-109).
* ``naive_collect_backward_output`` — zero-copy last-axis slice (:111-147).
* ``naive_collect_backward_x`` — last-axis reduce-scatter (:150-187).

Host (NumPy) inputs take buffer collectives of the native host plane: one
contiguous all-gather into a ``(p, B, S, k)`` buffer + concatenate, and one
``Reduce_scatter_block`` of the ``(p, B, S, in/p)`` packed gradient (instead of
pickled object all-gather / all-to-all).  Shapes are agreed first with a tiny
object all-gather, so ragged inputs still take the (reference) object path.
Device (CUDA tensor) inputs use the hand-written device collectives plus the
``interleave_lastaxis`` / ``deinterleave_lastaxis`` HIP kernels.
"""
from __future__ import annotations

import sys
from typing import Dict, Tuple

import numpy as np

_split_cache: Dict[Tuple, Tuple] = {}
_device_groups: Dict[int, object] = {}


def _is_device(x) -> bool:
    torch = sys.modules.get("torch")
    return torch is not None and isinstance(x, torch.Tensor) and x.is_cuda


def _host_comm(comm):
    """Underlying host communicator of a Communicator or a raw Comm."""
    return getattr(comm, "comm", comm)


def device_group_for(comm):
    """DeviceGroup of a Communicator (``.dev``) or of a raw host Comm (cached)."""
    if hasattr(comm, "dev") and hasattr(comm, "total_bytes_transferred"):
        return comm.dev
    key = id(comm)
    g = _device_groups.get(key)
    if g is None:
        from ..device import DeviceGroup

        g = DeviceGroup(comm)
        _device_groups[key] = g
    return g


def get_info(
    comm,
    rank: int,
    mp_size: int,
    dp_size: int,
    fc_layer: str,
    in_dim: int,
    out_dim: int,
):
    """Return ``(mp_idx, dp_idx, mp_comm, dp_comm, part_in_dim, part_out_dim)``.

    ``comm`` may be a raw ``MPI.Comm`` or a ``Communicator``; the returned
    communicators are of the same kind.  Layer validation happens before any
    communication so a bad ``fc_layer`` fails on every rank alike.
    """
    if fc_layer in ("fc_q", "fc_k", "fc_v"):
        part_in_dim, part_out_dim = in_dim, out_dim // mp_size
    elif fc_layer == "fc_o":
        part_in_dim, part_out_dim = in_dim // mp_size, out_dim
    else:
        raise ValueError(f"Invalid fc_layer: {fc_layer}.")
    mp_idx = rank % mp_size
    dp_idx = rank // mp_size
    key = (id(comm), rank, mp_size, dp_size)
    hit = _split_cache.get(key)
    if hit is None:
        mp_comm = comm.Split(color=dp_idx, key=mp_idx)
        dp_comm = comm.Split(color=mp_idx, key=dp_idx)
        _split_cache[key] = (comm, mp_comm, dp_comm)
    else:
        _, mp_comm, dp_comm = hit
    return mp_idx, dp_idx, mp_comm, dp_comm, part_in_dim, part_out_dim


# --------------------------------------------------------------------------
# host helpers
# --------------------------------------------------------------------------
def _host_allgather_lastaxis(x: np.ndarray, mp_comm) -> np.ndarray:
    hc = _host_comm(mp_comm)
    sig = (tuple(x.shape), x.dtype.str)
    sigs = hc.allgather(sig)
    if all(s == sig for s in sigs) and hasattr(hc, "Allgather") and x.dtype != object:
        p = len(sigs)
        xc = np.ascontiguousarray(x)
        buf = np.empty((p,) + x.shape, dtype=x.dtype)
        hc.Allgather(xc, buf)
        return np.concatenate(list(buf), axis=2)
    return np.concatenate(hc.allgather(x), axis=2)


def _host_reduce_scatter_lastaxis(g: np.ndarray, mp_comm, mp_size: int) -> np.ndarray:
    hc = _host_comm(mp_comm)
    sig = (tuple(g.shape), g.dtype.str)
    sigs = hc.allgather(sig)
    if all(s == sig for s in sigs) and g.shape[2] % mp_size == 0 and hasattr(hc, "Reduce_scatter_block"):
        from .. import mpi as MPI

        try:
            MPI.dtype_code(g.dtype)
            packed = np.ascontiguousarray(np.stack(np.split(g, mp_size, axis=2)))
            out = np.empty(packed.shape[1:], dtype=g.dtype)
            hc.Reduce_scatter_block(packed, out, MPI.SUM)
            return out
        except TypeError:
            pass
    chunks = np.split(g, mp_size, axis=2)
    return np.sum(hc.alltoall(chunks), axis=0)


# --------------------------------------------------------------------------
# device helpers
# --------------------------------------------------------------------------
def _dev_allgather_lastaxis(x, mp_comm, mp_size: int):
    """(.., k) shards -> (.., p*k): one device kernel pulls every peer's rows straight
    into the strided destination (no staging buffer, no interleave pass)."""
    import torch

    g = device_group_for(mp_comm)
    p = g.size
    xc = x.contiguous()
    k = xc.shape[-1]
    rows = xc.numel() // max(k, 1)
    out = torch.empty(tuple(xc.shape[:-1]) + (p * k,), dtype=xc.dtype, device=xc.device)
    rb = k * xc.element_size()
    if p == 1:
        out.copy_(xc)
    elif rb % 16 == 0:
        g.allgather_lastaxis(xc, out, rows, rb)
    else:  # rows not 16-B multiples: contiguous all-gather + interleave kernel
        stage = torch.empty((p,) + tuple(xc.shape), dtype=xc.dtype, device=xc.device)
        g.allgather(xc.reshape(-1), stage.reshape(-1))
        g.D.interleave_lastaxis(stage.data_ptr(), out.data_ptr(), rows, p, rb,
                                torch.cuda.current_stream(xc.device).cuda_stream)
    return out


def _dev_reduce_scatter_lastaxis(gx, mp_comm, mp_size: int):
    """(.., p*k) partial sums -> (.., k) reduced shard: one kernel reads each peer's
    strided last-axis slice and sums in registers (no pack pass)."""
    import torch

    g = device_group_for(mp_comm)
    p = g.size
    gc = gx.contiguous()
    n = gc.shape[-1]
    if n % p:
        raise ValueError("last axis must be divisible by mp_size")
    k = n // p
    rows = gc.numel() // max(n, 1)
    out = torch.empty(tuple(gc.shape[:-1]) + (k,), dtype=gc.dtype, device=gc.device)
    if p == 1:
        out.copy_(gc)
    elif (k * gc.element_size()) % 16 == 0:
        g.reduce_scatter_lastaxis(gc, out, rows, k)
    else:
        packed = torch.empty((p,) + tuple(gc.shape[:-1]) + (k,), dtype=gc.dtype, device=gc.device)
        g.D.deinterleave_lastaxis(gc.data_ptr(), packed.data_ptr(), rows, p, k * gc.element_size(),
                                  torch.cuda.current_stream(gc.device).cuda_stream)
        g.reduce_scatter(packed.reshape(-1), out.reshape(-1))
    return out


# --------------------------------------------------------------------------
# public API (reference names and argument order)
# --------------------------------------------------------------------------
def naive_collect_forward_input(x, mp_comm, mp_size: int):
    """fc_o forward input: ``(B, S, part_in)`` shards -> ``(B, S, part_in * mp)``."""
    if _is_device(x):
        return _dev_allgather_lastaxis(x, mp_comm, mp_size)
    return _host_allgather_lastaxis(x, mp_comm)


def naive_collect_forward_output(out, mp_comm, mp_size: int):
    """fc_o forward output: ``(B, S, part_out)`` shards -> ``(B, S, part_out * mp)``."""
    if _is_device(out):
        return _dev_allgather_lastaxis(out, mp_comm, mp_size)
    return _host_allgather_lastaxis(out, mp_comm)


def naive_collect_backward_output(output_grad, mp_group_idx: int, mp_size: int):
    """Local shard of the fc_o output gradient: a zero-copy last-axis view."""
    part_out_dim = output_grad.shape[2] // mp_size
    start_idx = mp_group_idx * part_out_dim
    return output_grad[:, :, start_idx:start_idx + part_out_dim]


def naive_collect_backward_x(grad_x, mp_comm, mp_size: int):
    """Reduce-scatter of fc_o's ``grad_x`` along the last axis:
    ``(B, S, in)`` on every rank -> summed ``(B, S, in // mp)`` shard ``mp_idx``."""
    if _is_device(grad_x):
        return _dev_reduce_scatter_lastaxis(grad_x, mp_comm, mp_size)
    return _host_reduce_scatter_lastaxis(grad_x, mp_comm, mp_size)
