"""Data-parallel gradient synchronisation for any torch model: gradients live in
flat, byte-capped buckets and each bucket is all-reduced as soon as autograd has
produced all of its gradients, on a communication stream that overlaps the rest
of the backward pass.

The reference only shards the data (data_parallel_preprocess.py:45-59) and
builds ``dp_comm`` (func_impl.py:61-62).  ``DistributedDataParallel`` adds the
gradient all-reduce on that DP communicator:

* buckets are filled in reverse parameter-registration order (roughly the order
  backward produces gradients) up to ``bucket_bytes`` each; xGMI is
  point-to-point, so a bucket must be large enough to keep all 7 links busy
  (default 64 MiB: ~9 MiB per link in flight at 8 ranks) and small enough that
  the first all-reduce starts early in the backward;
* every parameter's ``.grad`` is a view into its bucket (allocated from the DP
  device group's symmetric heap on the GPU, so the hand-written two-shot
  kernel runs zero-copy), so autograd accumulates straight into the buckets;
* a post-accumulate-grad hook counts a bucket's ready gradients; the last one
  records an event on the compute stream and launches the bucket's all-reduce
  on a high-priority side stream (its workgroups are dispatched ahead of the
  backward GEMM tiles queued behind them);
* ``finish()`` (call after ``backward()``, before the optimizer) launches
  buckets whose parameters got no gradient, joins the side stream and applies
  the 1/dp average;
* ``schedule``: ``"overlap"`` (the above), ``"deferred"`` (every bucket all-reduced
  in ``finish``, back to back on the compute stream at the group's full CTA budget:
  no collective CTAs beside the backward's GEMMs), or ``"auto"`` (default): the
  first synchronising steps run each schedule in turn, the device time between
  consecutive ``finish`` calls is compared (max over ranks) and the faster schedule
  is kept -- overlap can then never make a step slower than not overlapping
  (``schedule_choice`` records both times);
* gradient sinks (``grad_sink=True``, CUDA): the framework's own layers
  (tensor_parallel: Column/RowParallelLinear, ParallelSwiGLUMLP) write their weight
  gradients straight into the bucket views from the dW GEMM and notify the bucket
  themselves -- autograd then has no gradient tensor to accumulate, which saves
  an extra read-read-write pass over every such gradient (16 GB of bf16 per
  Llama-3-8B step).  Other parameters go through AccumulateGrad and the hook.

CPU tensors are reduced by the C++ host plane (the reference's CPU setting).
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional

import torch

from .layout import _host_comm, device_group_for


class _Bucket:
    __slots__ = ("params", "buf", "pending", "launched", "reduced", "event", "sinks")

    def __init__(self, params, buf):
        self.params = params
        self.buf = buf
        self.pending = len(params)
        self.launched = False
        self.reduced = False  # its all-reduce was issued this backward (the view is no longer ours)
        self.event = None
        self.sinks = []


class _GradSink:
    """Where a layer's backward writes a parameter's gradient (``param._ccmpi_grad_sink``):
    ``begin()`` returns (bucket view, accumulate?) -- overwrite after ``zero_grad`` (or when
    the user dropped ``.grad``), add when accumulating micro-batches -- and ``done()``
    counts the parameter ready in its bucket, exactly like the post-accumulate hook."""

    __slots__ = ("ddp", "param", "view", "fresh", "reported", "scale")

    def __init__(self, ddp, param, view, scale: float = 1.0):
        self.ddp, self.param, self.view, self.fresh, self.reported = ddp, param, view, True, False
        # the DP average folded into the producing GEMM (alpha = 1/p): no scaling pass over
        # the reduced bucket afterwards
        self.scale = scale

    def begin(self):
        q = self.param
        if q.grad is None or q.grad.data_ptr() != self.view.data_ptr():
            # grad dropped (zero_grad) or replaced: the bucket view is the gradient again, and
            # it is overwritten -- a user-supplied gradient is kept, scaled like everything the
            # sink adds to it (the DDP average rides in every contribution, not in finish)
            if q.grad is not None:
                if self.scale != 1.0:
                    torch.mul(q.grad.view_as(self.view), self.scale, out=self.view)
                else:
                    self.view.copy_(q.grad.view_as(self.view))
                self.fresh = False
            else:
                self.fresh = True
            q.grad = self.view
        acc = not self.fresh
        self.fresh = False
        return self.view, acc

    def done(self):
        self.reported = True
        self.ddp._ready(self.param)


class DistributedDataParallel(torch.nn.Module):
    """Wraps ``module``; ``comm`` is the DP communicator (Communicator or host Comm)."""

    def __init__(self, module: torch.nn.Module, comm, bucket_bytes: Optional[int] = None, algo: str = "auto",
                 average: bool = True, overlap: bool = True, broadcast_params: bool = True, grad_sink="auto",
                 max_blocks: Optional[int] = None, schedule: Optional[str] = None):
        super().__init__()
        schedule = schedule or os.environ.get("CCMPI_DP_SCHEDULE", "auto")
        if schedule not in ("overlap", "deferred", "auto"):
            raise ValueError(f"DistributedDataParallel: schedule {schedule!r} not in overlap/deferred/auto")
        # auto: trial steps (the first of each schedule is a warm-up), then the faster one
        self._trial = (["overlap"] * 3 + ["deferred"] * 3) if schedule == "auto" else []
        self.schedule = self._trial[0] if self._trial else schedule
        self.schedule_choice: Optional[dict] = None
        self._trial_events: List = []
        if bucket_bytes is None:
            # bucket sweep (profiles/r2_overlap/buckets.md): per-call cost makes buckets
            # below ~64 MiB expensive (16 MiB: 2.3x the comm time of 416 MiB buckets)
            bucket_bytes = int(os.environ.get("CCMPI_DP_BUCKET_MB", "64")) << 20
        self.module = module
        self.comm = comm
        self.hc = _host_comm(comm)
        self.p = self.hc.Get_size()
        self.algo = algo
        self.average = average
        self.require_backward_grad_sync = True  # False: buckets fill but are not reduced (no_sync)
        self.max_blocks = max_blocks  # CTA budget of the bucket all-reduces (None: the group's overlap_blocks)
        params = [q for q in module.parameters() if q.requires_grad]
        if not params:
            raise ValueError("DistributedDataParallel: the module has no trainable parameters")
        dev = params[0].device
        self.device = dev
        self.dev = device_group_for(comm) if dev.type == "cuda" and self.p > 1 else None
        if broadcast_params and self.p > 1:
            self._broadcast_params(params)
        # ---- buckets: reverse registration order, <= bucket_bytes, one dtype each
        self.buckets: List[_Bucket] = []
        self._view_of: Dict[int, torch.Tensor] = {}
        cur: List[torch.nn.Parameter] = []
        cur_bytes = 0
        for q in reversed(params):
            nb = q.numel() * q.element_size()
            if cur and (cur_bytes + nb > bucket_bytes or q.dtype != cur[0].dtype):
                self._make_bucket(cur)
                cur, cur_bytes = [], 0
            cur.append(q)
            cur_bytes += nb
        if cur:
            self._make_bucket(cur)
        self._bucket_of: Dict[int, _Bucket] = {id(q): b for b in self.buckets for q in b.params}
        # > 2 ranks sharing one GPU (test setup): no side stream (DeviceGroup.start)
        crowded = self.dev is not None and self.dev.shared_device and self.dev.ranks_per_device > 2
        self.stream = (torch.cuda.Stream(device=dev, priority=-1)
                       if (dev.type == "cuda" and overlap and self.p > 1 and not crowded) else None)
        self._hooks = [q.register_post_accumulate_grad_hook(self._on_grad) for q in params]
        self._late: List = []  # (param, scaled gradient) that arrived after its bucket's all-reduce started
        # grad_sink: "auto" = on CUDA; True also on the CPU (the host plane; tests)
        if grad_sink is True or (grad_sink == "auto" and dev.type == "cuda"):
            # the weights of the framework's TP layers, whose backward delivers dW itself;
            # every other parameter (biases, norms, embeddings, foreign modules) keeps the
            # AccumulateGrad + hook path
            from .tensor_parallel import ColumnParallelLinear, RowParallelLinear

            capable = {id(m.weight) for m in module.modules() if isinstance(m, (ColumnParallelLinear, RowParallelLinear))}
            for b in self.buckets:
                for q in b.params:
                    if id(q) in capable:
                        sk = _GradSink(self, q, self._view_of[id(q)],
                                       1.0 / self.p if (self.average and self.p > 1) else 1.0)
                        q._ccmpi_grad_sink = sk
                        b.sinks.append(sk)
                        self._hooks.append(q.register_hook(self._sink_pre_hook(q, sk, b)))

    # ------------------------------------------------------------------ setup
    def _broadcast_params(self, params) -> None:
        """Rank 0's parameters everywhere (the replicas start identical)."""
        with torch.no_grad():
            for q in params:
                if q.is_cuda:
                    t = q.data.contiguous()
                    self.dev.bcast(t, 0)
                    if t.data_ptr() != q.data.data_ptr():
                        q.data.copy_(t)
                else:
                    q.data.copy_(torch.as_tensor(self.hc.bcast(q.data.numpy() if self.hc.Get_rank() == 0 else None)))

    def _make_bucket(self, params) -> None:
        n = sum(q.numel() for q in params)
        dt = params[0].dtype
        if self.dev is not None:
            buf = self.dev.empty(n, dt)   # symmetric heap: zero-copy device collectives
            buf.zero_()
        else:
            buf = torch.zeros(n, dtype=dt, device=params[0].device)
        off = 0
        for q in params:
            q.grad = buf[off:off + q.numel()].view_as(q)
            self._view_of[id(q)] = q.grad
            off += q.numel()
        self.buckets.append(_Bucket(params, buf))

    # --------------------------------------------------------------- forward
    def forward(self, *args, **kwargs):
        return self.module(*args, **kwargs)

    # --------------------------------------------------------------- backward
    def _sink_pre_hook(self, q, sk: "_GradSink", b: "_Bucket"):
        """Gradient hook of a sink parameter: a contribution that reaches the weight through
        autograd (another use of the weight -- a penalty term, a foreign op) instead of the
        layer's sink.  Autograd runs the weight's AccumulateGrad after every producer's
        backward, so the layer's sink (if any) has delivered already.  The contribution is
        scaled like the sink's (1/p, the DDP average in every summand); if the bucket's
        all-reduce is already in flight it must not touch the bucket view: it is kept aside
        and all-reduced on its own in ``finish``."""

        def hook(g):
            if g is None:
                return None  # only the layer's sink produced this weight's gradient
            if sk.reported and b.reduced:
                self._late.append((q, g * sk.scale if sk.scale != 1.0 else g.clone()))
                q.grad = None  # AccumulateGrad then stores a fresh tensor; _on_grad restores the view
                return g
            return g * sk.scale if sk.scale != 1.0 else g

        return hook

    def _on_grad(self, q) -> None:
        v = self._view_of[id(q)]
        sk = getattr(q, "_ccmpi_grad_sink", None)
        if sk is not None and sk.reported:
            # the layer delivered this gradient itself: autograd still runs the post-accumulate
            # hook for the parameter (it was counted already); a late contribution was set
            # aside by the gradient hook -- re-attach the bucket view
            q.grad = v
            return
        if q.grad is None:
            q.grad = v  # no contribution at all
            if sk is not None and sk.fresh:
                v.zero_()  # a sink view nothing wrote this step reads as zero
                sk.fresh = False
        elif q.grad is not v and q.grad.data_ptr() != v.data_ptr():
            # the user dropped the grad (zero_grad(set_to_none=True)), or a sink parameter
            # reached only through autograd after DDP.zero_grad: autograd made a fresh tensor
            # -- move it into the bucket and re-attach the view
            v.copy_(q.grad)
            q.grad = v
        if sk is not None:
            sk.fresh = False  # the bucket view now holds this step's gradient (already 1/p-scaled)
        self._ready(q)

    def _ready(self, q) -> None:
        b = self._bucket_of[id(q)]
        b.pending -= 1
        if b.pending < 0:
            raise RuntimeError("DistributedDataParallel: a parameter produced two gradients in one backward "
                               "(shared weight?) -- build DDP with grad_sink=False")
        if b.pending == 0:
            self._launch(b)

    def _launch(self, b: _Bucket) -> None:
        if b.launched or self.p == 1 or not self.require_backward_grad_sync:
            b.launched = True
            return
        if self.schedule == "deferred" and not self._finishing:
            return  # all-reduced by finish(), after the backward
        b.launched = True
        b.reduced = True
        if self.dev is None:  # host plane
            from .. import mpi as MPI

            self.hc.Allreduce(MPI.IN_PLACE, b.buf.numpy(), op=MPI.SUM)
            return
        if self.schedule == "deferred":
            # nothing else runs: the compute stream and the full CTA budget
            self.dev.allreduce(b.buf, b.buf, "SUM", self.algo, max_blocks=self.dev.max_blocks, symmetric=True)
            return
        if self.stream is None:
            self.dev.allreduce(b.buf, b.buf, "SUM", self.algo, symmetric=True)
            return
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.device))
        self.stream.wait_event(ev)
        with torch.cuda.stream(self.stream):  # beside the backward: the overlap CTA budget
            self.dev.allreduce(b.buf, b.buf, "SUM", self.algo, max_blocks=self._blocks(),
                               symmetric=True)

    def _blocks(self) -> int:
        """CTA budget of a bucket all-reduce: ``max_blocks`` (default: the group's
        ``overlap_blocks``), never above the group's ``overlap_cap``."""
        return min(self.max_blocks or self.dev.overlap_blocks, getattr(self.dev, "overlap_cap", 1 << 30))

    _finishing = False

    def finish(self) -> None:
        """Complete the gradient synchronisation (after backward, before the step)."""
        self._finishing = True
        try:
            for b in self.buckets:  # parameters that received no gradient this step (deferred: all)
                if not b.launched:
                    for sk in b.sinks:
                        if sk.fresh:  # no gradient since zero_grad: the view must read as zero
                            sk.view.zero_()
                            sk.fresh = False
                    self._launch(b)
        finally:
            self._finishing = False
        if self.stream is not None:
            torch.cuda.current_stream(self.device).wait_stream(self.stream)
        if self._late:
            # contributions that reached sink weights after their bucket's all-reduce started
            # (already 1/p-scaled): every rank has the same list (same model code), each one
            # is all-reduced on its own and added to the reduced bucket view
            for q, g in self._late:
                g = g.contiguous()
                if self.dev is None:
                    from .. import mpi as MPI

                    self.hc.Allreduce(MPI.IN_PLACE, g.numpy(), op=MPI.SUM)
                else:
                    self.dev.allreduce(g, g, "SUM", self.algo)
                self._view_of[id(q)].add_(g.view_as(self._view_of[id(q)]))
            self._late = []
        if self.average and self.p > 1 and self.require_backward_grad_sync:
            # (no_sync micro-batches: the local sums keep accumulating, the synchronising
            # backward reduces and averages all of them at once).  Every contribution to a
            # sink parameter is already scaled by 1/p (the GEMM's alpha, or the gradient
            # hook): only the others are scaled here (norms, biases, embeddings: ~1 GB of a
            # Llama-3-8B's 16 GB)
            for b in self.buckets:
                if not b.sinks:
                    b.buf.mul_(1.0 / self.p)
                    continue
                sunk = {id(sk.param) for sk in b.sinks}
                for q in b.params:
                    if id(q) not in sunk:
                        self._view_of[id(q)].mul_(1.0 / self.p)
        for b in self.buckets:
            b.pending = len(b.params)
            b.launched = False
            b.reduced = False
            for sk in b.sinks:
                sk.reported = False
                sk.param.grad = sk.view
        if self._trial and self.require_backward_grad_sync and self.p > 1 and self.dev is not None:
            self._trial_step()

    def _trial_step(self) -> None:
        """``schedule="auto"``: an event at the end of every synchronising step; step k ran
        ``_trial[k]``.  After the last trial step: the median device time between
        consecutive events of each schedule (its first step, the switch, excluded), max over
        ranks (a host all-reduce: every rank takes the same decision), and the faster
        schedule kept."""
        ev = torch.cuda.Event(enable_timing=True)
        ev.record(torch.cuda.current_stream(self.device))
        self._trial_events.append(ev)
        k = len(self._trial_events) - 1
        if k + 1 < len(self._trial):
            self.schedule = self._trial[k + 1]
            return
        from .. import mpi as MPI

        ev.synchronize()
        evs = self._trial_events
        gaps = [evs[i - 1].elapsed_time(evs[i]) for i in range(1, len(evs))]
        self.schedule_choice = pick_schedule(self._trial, gaps, lambda v: self.hc.allreduce(v, op=MPI.MAX))
        self.schedule = self.schedule_choice["chosen"]
        self._trial, self._trial_events = [], []

    def zero_grad(self, set_to_none: bool = False) -> None:
        """Zero the gradients and re-attach every ``.grad`` view (``set_to_none`` is ignored).
        Gradients with a sink are not written: their ``.grad`` is set to None instead, so the
        next backward overwrites the bucket view -- through the layer's sink, or through
        AccumulateGrad and ``_on_grad`` (a weight reached by another op) -- and ``finish``
        zeroes the ones it did not reach and re-attaches the views."""
        for b in self.buckets:
            sunk = {id(sk.param) for sk in b.sinks}
            if not sunk:
                b.buf.zero_()
            else:
                for q in b.params:
                    if id(q) not in sunk:
                        self._view_of[id(q)].zero_()
                for sk in b.sinks:
                    sk.fresh = True
            for q in b.params:
                q.grad = None if id(q) in sunk else self._view_of[id(q)]

    def allreduce_all(self, max_blocks: Optional[int] = None) -> None:
        """All-reduce every bucket now, back to back on the current stream (the comm-only
        time of the overlap measurement; no averaging).  ``max_blocks``: the CTA budget
        (default: the overlap budget)."""
        if self.dev is None or self.p == 1:
            return
        for b in self.buckets:
            self.dev.allreduce(b.buf, b.buf, "SUM", self.algo, max_blocks=max_blocks or self._blocks(),
                               symmetric=True)

    @property
    def bucket_sizes(self) -> List[int]:
        return [b.buf.numel() * b.buf.element_size() for b in self.buckets]


def pick_schedule(trial: List[str], gaps_ms: List[float], agree_max) -> dict:
    """The ``schedule="auto"`` decision.  ``trial[k]``: the schedule step k ran;
    ``gaps_ms[k - 1]``: device time from the end of step k - 1 to the end of step k.  A
    step whose predecessor ran another schedule (the first of each, a warm-up or the
    switch) is not counted; per schedule the median, max over ranks (``agree_max``, so
    every rank decides the same), the smaller wins (ties: overlap)."""
    times: Dict[str, List[float]] = {}
    for k in range(1, len(trial)):
        if trial[k] == trial[k - 1] and k - 1 < len(gaps_ms):
            times.setdefault(trial[k], []).append(gaps_ms[k - 1])
    med = {s: agree_max(sorted(v)[len(v) // 2]) for s, v in sorted(times.items(), key=lambda kv: kv[0] != "overlap")}
    chosen = min(med, key=med.get) if med else "overlap"
    return {"chosen": chosen, **{f"{s}_ms": round(v, 3) for s, v in med.items()}}


def ddp_wrap(module: torch.nn.Module, comm, **kw) -> DistributedDataParallel:
    return DistributedDataParallel(module, comm, **kw)


__all__ = ["DistributedDataParallel", "ddp_wrap", "pick_schedule"]
