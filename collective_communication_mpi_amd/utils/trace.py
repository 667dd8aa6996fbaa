"""Structured per-collective tracing (off by default).

``CCMPI_TRACE=1`` makes every device collective:

* open a roctx range named ``ccmpi.<op>.<algo>.<bytes>B`` (torch.cuda.nvtx maps to
  roctx on ROCm, so the ranges appear in ``rocprofv3 --marker-trace``);
* record a pair of hipEvents around the launch on the collective's stream.

``TRACE.report()`` (also registered ``atexit`` when ``CCMPI_TRACE_FILE`` is set)
resolves the events and prints / dumps one record per call: op, algo, bytes,
device time, algbw and busbw (NCCL-tests conventions).  This replaces the
reference's only metrics, ``MPI.Wtime`` deltas and ``total_bytes_transferred``
(mpi-test.py:59-72, comm.py:7), with measured device-side numbers.
"""
from __future__ import annotations

import atexit
import json
import os
import sys
import threading
from typing import List, Optional

_BUS = {"allreduce": lambda p: 2 * (p - 1) / p, "allgather": lambda p: (p - 1) / p,
        "reduce_scatter": lambda p: (p - 1) / p, "alltoall": lambda p: (p - 1) / p, "bcast": lambda p: 1.0}


class _Trace:
    def __init__(self) -> None:
        self.enabled = os.environ.get("CCMPI_TRACE", "0") not in ("0", "")
        self.records: List[dict] = []
        self._pending: List[tuple] = []
        self._lock = threading.Lock()
        if self.enabled:  # summary on stderr at exit, or JSON lines to CCMPI_TRACE_FILE
            atexit.register(self.report, os.environ.get("CCMPI_TRACE_FILE"))

    def begin(self, op: str, algo: str, nbytes: int, ranks: int, stream) -> Optional[tuple]:
        if not self.enabled:
            return None
        import torch

        name = f"ccmpi.{op}.{algo}.{nbytes}B"
        torch.cuda.nvtx.range_push(name)
        if torch.cuda.is_current_stream_capturing():
            # inside a HIP graph capture an event record becomes a graph node whose
            # timestamps cannot be read back: keep the range, skip the timing
            return (op, algo, nbytes, ranks, None, None, stream)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record(stream)
        return (op, algo, nbytes, ranks, s, e, stream)

    def end(self, tok: Optional[tuple]) -> None:
        if tok is None:
            return
        import torch

        torch.cuda.nvtx.range_pop()
        if tok[4] is None:
            return
        tok[5].record(tok[6])
        with self._lock:
            self._pending.append(tok)
            drain = len(self._pending) >= 4096
        if drain:  # bound the pending events of long runs: resolve the completed ones
            self.flush(completed_only=True)

    def flush(self, completed_only: bool = False) -> None:
        with self._lock:
            if completed_only:
                pend = [t for t in self._pending if t[5].query()]
                done = {id(t) for t in pend}
                self._pending = [t for t in self._pending if id(t) not in done]
            else:
                pend, self._pending = self._pending, []
        for op, algo, nbytes, ranks, s, e, _ in pend:
            e.synchronize()
            ms = s.elapsed_time(e)
            algbw = nbytes / (ms * 1e-3) / 1e9 if ms > 0 else 0.0
            self.records.append({"op": op, "algo": algo, "bytes": nbytes, "ranks": ranks, "ms": round(ms, 4),
                                 "algbw_GBps": round(algbw, 3),
                                 "busbw_GBps": round(algbw * _BUS.get(op, lambda p: 1.0)(ranks), 3)})

    def report(self, path: Optional[str] = None, file=sys.stderr) -> List[dict]:
        self.flush()
        if path:
            with open(path if "{pid}" not in path else path.format(pid=os.getpid()), "w") as f:
                for r in self.records:
                    f.write(json.dumps(r) + "\n")
        else:
            agg = {}
            for r in self.records:
                k = (r["op"], r["algo"])
                a = agg.setdefault(k, [0, 0, 0.0])
                a[0] += 1
                a[1] += r["bytes"]
                a[2] += r["ms"]
            for (op, algo), (n, b, ms) in sorted(agg.items()):
                print(f"[ccmpi trace] {op:15s} {algo:13s} calls={n:6d} bytes={b:14d} device_ms={ms:10.3f} "
                      f"algbw={b / max(ms, 1e-9) / 1e6:9.2f} GB/s", file=file)
        return self.records


TRACE = _Trace()


def trace_call(op: str):
    """Decorator for DeviceGroup collectives: (self, src, ...) with an ``algo`` kwarg/positional."""
    def deco(fn):
        import inspect

        sig = inspect.signature(fn)

        def wrapped(self, *args, **kw):
            if not TRACE.enabled:
                return fn(self, *args, **kw)
            bound = sig.bind(self, *args, **kw)
            bound.apply_defaults()
            src = args[0]
            nbytes = src.numel() * src.element_size()
            algo = bound.arguments.get("algo", "default")
            if op == "allreduce" and algo == "auto":  # record the algorithm actually chosen
                algo = f"auto->{self.pick_allreduce(nbytes)}"
            tok = TRACE.begin(op, str(algo), nbytes, self.size, self.torch.cuda.current_stream(self.device))
            try:
                return fn(self, *args, **kw)
            finally:
                TRACE.end(tok)
        wrapped.__name__ = fn.__name__
        wrapped.__doc__ = fn.__doc__
        return wrapped
    return deco
