"""Data parallelism: flat parameter/gradient storage and bucketed gradient
all-reduce overlapped with the backward pass.

The reference only shards data across DP groups (data_parallel_preprocess.py:45-59)
and builds ``dp_comm`` (func_impl.py:61-62); "we simply just split the batch"
(README.md:177).  Here the DP group also synchronises gradients:

* every parameter lives in one flat fp32 master buffer (+ a bf16 compute copy
  + AdamW moments); gradients live in one flat fp32 buffer allocated from the
  DP device group's *symmetric heap*, so bucket all-reduces run zero-copy
  (no staging) with the hand-written fan-out two-shot kernel over all xGMI links;
* the layout is in backward order, so each bucket is a contiguous range that
  becomes ready as soon as its layer's weight-gradient GEMMs are issued;
* ``GradBuckets.ready(i)`` records an event on the compute stream and launches
  bucket ``i``'s all-reduce on a dedicated communication stream: the collective
  overlaps the remaining backward GEMMs; ``wait()`` joins before the optimizer.
* the 1/dp average is folded into the fused AdamW kernel (one pass over the
  flat buffers that also refreshes the bf16 compute copy).
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional, Sequence, Tuple

import torch

from .. import _native

_ALIGN = 64  # elements: keeps every parameter view 256-B aligned


class FlatParams:
    """Flat fp32 master weights + bf16 compute copy + AdamW moments.

    ``transposed`` names 2-D parameters that also keep a TRANSPOSED bf16 copy
    (``param16_t``), refreshed by the same fused AdamW / cast kernels, so the
    backward GEMMs that consume W^T need no per-step transpose launch."""

    def __init__(self, specs: Sequence[Tuple[str, Tuple[int, ...]]], device, grad_alloc=None,
                 transposed: Sequence[str] = ()):
        self.specs = list(specs)
        self.offsets: Dict[str, Tuple[int, int, Tuple[int, ...]]] = {}
        off = 0
        for name, shape in self.specs:
            n = 1
            for s in shape:
                n *= int(s)
            self.offsets[name] = (off, n, tuple(shape))
            off += (n + _ALIGN - 1) // _ALIGN * _ALIGN
        self.numel = max(off, _ALIGN)
        self.device = torch.device(device)
        self.p32 = torch.zeros(self.numel, dtype=torch.float32, device=self.device)
        self.p16 = torch.zeros(self.numel, dtype=torch.bfloat16, device=self.device)
        self.g = grad_alloc(self.numel) if grad_alloc else torch.zeros(self.numel, dtype=torch.float32,
                                                                          device=self.device)
        self.g.zero_()
        self.m = torch.zeros_like(self.p32)
        self.v = torch.zeros_like(self.p32)
        self.step_count = 0
        self._step_dev: Optional[torch.Tensor] = None  # two "steps done" slots for recorded steps
        self._step_par = 0
        self.grad_dirty = False  # g holds values a step has not consumed (AdamW zeroes what it reads)
        self.p16_t: Dict[str, torch.Tensor] = {}
        for name in transposed:
            off, n, shape = self.offsets[name]
            if len(shape) != 2:
                raise ValueError(f"transposed copy needs a 2-D parameter, {name} is {shape}")
            self.p16_t[name] = torch.zeros((shape[1], shape[0]), dtype=torch.bfloat16, device=self.device)
        self._tregions = [(self.offsets[nm][0], self.offsets[nm][2][0], self.offsets[nm][2][1], t.data_ptr())
                          for nm, t in self.p16_t.items()]

    def view(self, buf: torch.Tensor, name: str) -> torch.Tensor:
        off, n, shape = self.offsets[name]
        return buf[off:off + n].view(shape)

    def param(self, name):
        return self.view(self.p32, name)

    def param16(self, name):
        return self.view(self.p16, name)

    def grad(self, name):
        return self.view(self.g, name)

    def range_of(self, names: Sequence[str]) -> Tuple[int, int]:
        lo = min(self.offsets[n][0] for n in names)
        hi = max(self.offsets[n][0] + (self.offsets[n][1] + _ALIGN - 1) // _ALIGN * _ALIGN for n in names)
        return lo, hi

    def param16_t(self, name):
        """[cols, rows] bf16 copy of a 2-D parameter (see ``transposed``)."""
        return self.p16_t[name]

    def refresh_bf16(self) -> None:
        _native.device().cast_bf16(self.p32.data_ptr(), self.p16.data_ptr(), self.numel,
                                   torch.cuda.current_stream(self.device).cuda_stream, self._tregions)

    def device_step(self) -> torch.Tensor:
        """The device-side step counter (two int32 slots of "steps done", used alternately),
        seeded from ``step_count``.  An AdamW launched with ``device_step=True`` reads
        t - 1 from slot ``p`` and writes t to slot ``p ^ 1`` (``p`` flips per call), so the
        alternating pair of recorded training steps (HIP graphs or launch plans) replays with
        the right bias corrections; ``sync_step()`` brings ``step_count`` back."""
        if self._step_dev is None:
            self._step_dev = torch.zeros(2, dtype=torch.int32, device=self.device)
        self._step_dev.fill_(self.step_count)
        self._step_par = 0
        return self._step_dev

    def sync_step(self) -> int:
        """step_count <- the device counter (after graph replays)."""
        if self._step_dev is not None:
            newest = int(torch.argmax(self._step_dev).item())     # the slots alternate; the newer is larger
            self.step_count = int(self._step_dev[newest].item())
            self._step_par = newest
        return self.step_count

    def adamw(self, lr: float, betas=(0.9, 0.999), eps: float = 1e-8, weight_decay: float = 0.0,
              grad_scale: float = 1.0, device_step: bool = False) -> None:
        self.step_count += 1
        if device_step and self._step_dev is None:
            raise RuntimeError("adamw(device_step=True): call device_step() first (outside any capture)")
        _native.device().adamw_step(self.p32.data_ptr(), self.g.data_ptr(), self.m.data_ptr(), self.v.data_ptr(),
                                    self.p16.data_ptr(), self.numel, lr, betas[0], betas[1], eps, weight_decay,
                                    self.step_count, grad_scale, torch.cuda.current_stream(self.device).cuda_stream,
                                    self._tregions, True,
                                    step_dev=self._step_dev.data_ptr() if device_step else 0,
                                    step_parity=self._step_par if device_step else 0)
        if device_step:
            self._step_par ^= 1
        self.grad_dirty = False


class GradBuckets:
    """Bucketed DP gradient all-reduce on a side stream."""

    def __init__(self, flat: FlatParams, dp_group, buckets: Sequence[Sequence[str]], algo: str = "auto",
                 overlap: bool = True):
        self.flat = flat
        self.dp = dp_group  # DeviceGroup or None (dp == 1)
        self.ranges = [flat.range_of(b) for b in buckets]
        self.algo = algo
        self.overlap = overlap
        # side stream at NORMAL priority: measured (profiles/r2_overlap, 2 ranks, 4 Llama-3-8B
        # layers) a high-priority bucket stream hid 0% of the all-reduce -- its spinning CTAs are
        # dispatched ahead of the GEMM tiles and wait for the peer's bucket -- vs 35% at normal
        # priority; CCMPI_DP_STREAM_PRIORITY=-1 restores the high-priority stream
        prio = int(os.environ.get("CCMPI_DP_STREAM_PRIORITY", "0"))
        # > 2 ranks sharing one GPU (test setup): no side stream -- one extra stream per
        # process oversubscribes the hardware queues (see DeviceGroup.start)
        crowded = dp_group is not None and dp_group.shared_device and dp_group.ranks_per_device > 2
        self.stream = torch.cuda.Stream(device=flat.device, priority=prio) \
            if (dp_group is not None and overlap and not crowded) else None
        self.events: List[torch.cuda.Event] = [torch.cuda.Event() for _ in self.ranges]
        self.launched = 0

    def ready(self, i: int) -> None:
        if self.dp is None or self.dp.size == 1:
            return
        lo, hi = self.ranges[i]
        seg = self.flat.g[lo:hi]
        if self.stream is None:
            self.dp.allreduce(seg, seg, "SUM", self.algo)
            return
        ev = self.events[i]
        ev.record(torch.cuda.current_stream(self.flat.device))
        self.stream.wait_event(ev)
        with torch.cuda.stream(self.stream):
            self.dp.allreduce(seg, seg, "SUM", self.algo, max_blocks=self.dp.overlap_blocks)
        self.launched += 1

    def wait(self) -> None:
        if self.stream is not None:
            torch.cuda.current_stream(self.flat.device).wait_stream(self.stream)
