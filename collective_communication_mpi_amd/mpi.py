"""mpi4py-compatible ``MPI`` namespace backed by the framework's native host plane.

The reference imports ``from mpi4py import MPI`` everywhere (mpi_wrapper/comm.py:1,
model/func_impl.py:2, mpi-test.py:1, tests/*.py).  mpi4py and libmpi are not
part of this framework: this module exposes the subset of mpi4py's API that
the reference (and typical teaching code like it) uses, implemented by the C++
shared-memory runtime in ``csrc/host`` (``_host`` extension):

* ``COMM_WORLD`` / ``COMM_SELF`` / ``COMM_NULL``, ``Comm.Get_rank/Get_size``;
* buffer ("uppercase") P2P: ``Send/Recv/Isend/Irecv/Sendrecv``, ``Probe/Iprobe``;
* buffer collectives: ``Barrier, Bcast, Allreduce, Reduce, Allgather(v),
  Gather(v), Scatter(v), Reduce_scatter_block, Reduce_scatter, Alltoall(v),
  Scan, Exscan``;
* object ("lowercase", pickle) versions: ``send/recv/isend/irecv/sendrecv,
  bcast, allgather, alltoall, gather, scatter, allreduce, reduce, barrier``;
* ``Split(color, key)``, ``Dup``, ``Free``; ops ``SUM PROD MIN MAX LAND LOR
  LXOR BAND BOR BXOR REPLACE``; ``Wtime``; ``Request.Wait/Test/Waitall/Waitany``;
  ``IN_PLACE``; ``UNDEFINED``; ``ANY_SOURCE``/``ANY_TAG``/``PROC_NULL``.

Launch with ``scripts/mpirun -n N python ...`` (or Hydra ``mpiexec``, or
``torchrun``: the runtime reads PMI_*/OMPI_*/RANK env vars).
"""
from __future__ import annotations

import pickle
import sys
import threading
import time as _time
from typing import Any, Iterable, List, Optional, Sequence

import numpy as np

from . import _native

_h = _native.host()
# METH_FASTCALL entry points (csrc/host/fastcall.cpp) for plain contiguous
# buffers; each returns NotImplemented when the general path is needed
_fsend, _frecv, _fisend, _firecv = _h.fsend, _h.frecv, _h.fisend, _h.firecv
_fwait, _ftest, _fwaitall, _fsendrecv = _h.fwait, _h.ftest, _h.fwaitall, _h.fsendrecv
_fbarrier, _fbcast, _fallreduce, _fallgather = _h.fbarrier, _h.fbcast, _h.fallreduce, _h.fallgather
_falltoall, _freduce_scatter_block = _h.falltoall, _h.freduce_scatter_block
_NI = NotImplemented

ANY_SOURCE = _h.ANY_SOURCE
ANY_TAG = _h.ANY_TAG
PROC_NULL = _h.PROC_NULL
UNDEFINED = -32766
SUCCESS = 0
THREAD_SINGLE, THREAD_FUNNELED, THREAD_SERIALIZED, THREAD_MULTIPLE = 0, 1, 2, 3
VERSION, SUBVERSION = 3, 1


class _InPlace:
    def __repr__(self) -> str:
        return "MPI.IN_PLACE"


IN_PLACE = _InPlace()
BOTTOM = None


# --------------------------------------------------------------------------
# datatypes & ops
# --------------------------------------------------------------------------
DT_I8, DT_U8, DT_I16, DT_U16, DT_I32, DT_U32, DT_I64, DT_U64 = range(8)
DT_F16, DT_BF16, DT_F32, DT_F64, DT_BOOL, DT_C64, DT_C128, DT_BYTE = range(8, 16)

_NP2DT = {
    np.dtype(np.int8): DT_I8, np.dtype(np.uint8): DT_U8,
    np.dtype(np.int16): DT_I16, np.dtype(np.uint16): DT_U16,
    np.dtype(np.int32): DT_I32, np.dtype(np.uint32): DT_U32,
    np.dtype(np.int64): DT_I64, np.dtype(np.uint64): DT_U64,
    np.dtype(np.float16): DT_F16, np.dtype(np.float32): DT_F32,
    np.dtype(np.float64): DT_F64, np.dtype(np.bool_): DT_BOOL,
    np.dtype(np.complex64): DT_C64, np.dtype(np.complex128): DT_C128,
}


_DT_CACHE: dict = {}


def dtype_code(dt) -> int:
    """Native dtype code for a numpy dtype (``"bfloat16"`` for bf16 payloads)."""
    code = _DT_CACHE.get(dt) if isinstance(dt, np.dtype) else None
    if code is not None:
        return code
    if isinstance(dt, str) and dt == "bfloat16":
        return DT_BF16
    d = np.dtype(dt)
    if d.byteorder not in ("=", "|"):
        d = d.newbyteorder("=")
    try:
        code = _NP2DT[d]
    except KeyError:
        raise TypeError(f"MPI: unsupported buffer dtype {dt!r}") from None
    if isinstance(dt, np.dtype):
        _DT_CACHE[dt] = code
    return code


class Datatype:
    """Minimal mpi4py Datatype: only used in ``[buf, MPI.INT]`` buffer specs."""

    def __init__(self, name: str, np_dtype) -> None:
        self.name = name
        self.np_dtype = np.dtype(np_dtype) if np_dtype is not None else None

    def Get_size(self) -> int:
        return self.np_dtype.itemsize if self.np_dtype is not None else 1

    size = property(Get_size)

    def __repr__(self) -> str:
        return f"MPI.{self.name}"


CHAR = Datatype("CHAR", np.int8)
SIGNED_CHAR = CHAR
BYTE = Datatype("BYTE", np.uint8)
SHORT = Datatype("SHORT", np.int16)
INT = Datatype("INT", np.int32)
LONG = Datatype("LONG", np.int64)
LONG_LONG = LONG
UNSIGNED = Datatype("UNSIGNED", np.uint32)
UNSIGNED_LONG = Datatype("UNSIGNED_LONG", np.uint64)
FLOAT = Datatype("FLOAT", np.float32)
DOUBLE = Datatype("DOUBLE", np.float64)
BOOL = Datatype("BOOL", np.bool_)
C_BOOL = BOOL
INT8_T, INT16_T, INT32_T, INT64_T = CHAR, SHORT, INT, LONG
UINT8_T = BYTE
COMPLEX = Datatype("COMPLEX", np.complex64)
DOUBLE_COMPLEX = Datatype("DOUBLE_COMPLEX", np.complex128)


class Op:
    """Reduction operator; ``code`` indexes the native kernel table."""

    def __init__(self, name: str, code: int, py) -> None:
        self.name, self.code, self._py = name, code, py

    def __call__(self, a, b):
        return self._py(a, b)

    def __eq__(self, other) -> bool:
        return isinstance(other, Op) and other.code == self.code

    def __hash__(self) -> int:
        return hash(("MPI.Op", self.code))

    def __repr__(self) -> str:
        return f"MPI.{self.name}"


def _elem(fn_np, fn_py):
    def f(a, b):
        if isinstance(a, np.ndarray) or isinstance(b, np.ndarray):
            return fn_np(a, b)
        return fn_py(a, b)
    return f


SUM = Op("SUM", 0, lambda a, b: a + b)
PROD = Op("PROD", 1, lambda a, b: a * b)
MIN = Op("MIN", 2, _elem(np.minimum, min))
MAX = Op("MAX", 3, _elem(np.maximum, max))
LAND = Op("LAND", 4, _elem(np.logical_and, lambda a, b: a and b))
LOR = Op("LOR", 5, _elem(np.logical_or, lambda a, b: a or b))
LXOR = Op("LXOR", 6, _elem(np.logical_xor, lambda a, b: bool(a) != bool(b)))
BAND = Op("BAND", 7, lambda a, b: a & b)
BOR = Op("BOR", 8, lambda a, b: a | b)
BXOR = Op("BXOR", 9, lambda a, b: a ^ b)
REPLACE = Op("REPLACE", 10, lambda a, b: b)
NO_OP = Op("NO_OP", 10, lambda a, b: a)
OPS = (SUM, PROD, MIN, MAX, LAND, LOR, LXOR, BAND, BOR, BXOR, REPLACE)


class MPIException(RuntimeError):
    """Mirrors ``mpi4py.MPI.Exception`` (exported under that name at the end)."""

    def __init__(self, msg: str = "", code: int = 1) -> None:
        super().__init__(msg)
        self.error_code = code

    def Get_error_code(self) -> int:
        return self.error_code


# --------------------------------------------------------------------------
# buffer specs
# --------------------------------------------------------------------------
class _Buf:
    __slots__ = ("arr", "obj", "dt", "counts", "displs")

    def __init__(self, arr, dt: int, counts=None, displs=None) -> None:
        self.arr, self.obj, self.dt, self.counts, self.displs = arr, arr, dt, counts, displs

    @property
    def nbytes(self) -> int:
        return self.arr.nbytes

    @property
    def itemsize(self) -> int:
        return self.arr.itemsize


def _as_array(x, writable: bool):
    torch = sys.modules.get("torch")  # never import torch from the host plane
    if torch is not None and isinstance(x, torch.Tensor):
        if x.device.type != "cpu":
            raise TypeError("MPI: this call takes host buffers; CUDA tensors work with Allreduce, Allgather, "
                            "Reduce_scatter_block, Alltoall and Bcast (and with Communicator)")
        x = x.detach().numpy()
    if isinstance(x, (bytes, bytearray, memoryview)):
        a = np.frombuffer(x, dtype=np.uint8)
        if writable and not a.flags.writeable:
            raise ValueError("MPI: receive buffer is read-only")
        return a
    if not isinstance(x, np.ndarray):
        x = np.asarray(x)
    if not x.flags.c_contiguous:
        if writable:
            raise ValueError("MPI: receive buffers must be C-contiguous")
        x = np.ascontiguousarray(x)
    if writable and not x.flags.writeable:
        raise ValueError("MPI: receive buffer is read-only")
    return x


def _parse(spec, writable: bool) -> Optional[_Buf]:
    """Accept ``arr``, ``[arr, Datatype]``, ``[arr, count, Datatype]`` or
    ``[arr, (counts, displs), Datatype]`` / ``[arr, counts, displs, Datatype]``."""
    if type(spec) is np.ndarray:  # fast path: a plain contiguous NumPy buffer (the common case)
        f = spec.flags
        if f.c_contiguous and (f.writeable or not writable):
            code = _DT_CACHE.get(spec.dtype)
            if code is not None:
                return _Buf(spec, code)
    if spec is None or spec is IN_PLACE:
        return None
    counts = displs = None
    dtype = None
    if isinstance(spec, (list, tuple)):
        parts = list(spec)
        arr = parts[0]
        rest = parts[1:]
        if rest and isinstance(rest[-1], Datatype):
            dtype = rest.pop()
        if len(rest) == 1:
            if isinstance(rest[0], (list, tuple)) and len(rest[0]) == 2 and isinstance(rest[0][0], (list, tuple, np.ndarray)):
                counts, displs = rest[0]
            elif isinstance(rest[0], (list, tuple, np.ndarray)):
                counts = rest[0]
        elif len(rest) == 2:
            counts, displs = rest
    else:
        arr = spec
    a = _as_array(arr, writable)
    if dtype is not None and dtype.np_dtype is not None and a.dtype != dtype.np_dtype:
        a = a.view(dtype.np_dtype) if a.dtype.itemsize * a.size % dtype.np_dtype.itemsize == 0 else a
    try:
        dt = dtype_code(a.dtype)
    except TypeError:
        dt = DT_BYTE
    if counts is not None:
        counts = [int(c) for c in np.asarray(counts).ravel()]
    if displs is not None:
        displs = [int(d) for d in np.asarray(displs).ravel()]
    return _Buf(a, dt, counts, displs)


def _cuda(*xs) -> bool:
    """True when a buffer argument is a CUDA tensor (CUDA-aware-MPI calls)."""
    torch = sys.modules.get("torch")
    return torch is not None and any(isinstance(x, torch.Tensor) and x.is_cuda for x in xs)


def _raw(b: Optional[_Buf]):
    return None if b is None else b.arr


# --------------------------------------------------------------------------
# status / requests
# --------------------------------------------------------------------------
class Status:
    def __init__(self) -> None:
        self.source = ANY_SOURCE
        self.tag = ANY_TAG
        self.count = 0  # bytes
        self.error = SUCCESS

    def _set(self, st) -> None:
        self.source, self.tag, self.count = int(st[0]), int(st[1]), int(st[2])

    def Get_source(self) -> int:
        return self.source

    def Get_tag(self) -> int:
        return self.tag

    def Get_error(self) -> int:
        return self.error

    def Get_count(self, datatype: Optional[Datatype] = None) -> int:
        size = datatype.Get_size() if datatype is not None else 1
        return self.count // size

    Get_elements = Get_count


class Request:
    """Wraps a native request and keeps its buffer alive until completion.
    ``_native`` is an int handle (fast path, fastcall.cpp) or a pybind11 request."""

    __slots__ = ("_comm", "_native", "_keep", "_decode", "_done", "_result")

    def __init__(self, comm: "Comm", native, keep, decode=None) -> None:
        self._comm, self._native, self._keep, self._decode = comm, native, keep, decode
        self._done = native is None
        self._result = None

    def _finish(self, status: Optional[Status]):
        if self._native is not None and not self._done:
            n = self._native
            st = _fwait(n) if type(n) is int else self._comm._hc.wait(n)
            if type(n) is int:
                self._native = st  # keep the status for a later Get_status
            self._done = True
            if status is not None:
                status._set(st)
            if self._decode is not None:
                self._result = self._decode()
            self._keep = None
        elif status is not None and self._native is not None:
            status._set(self._native if type(self._native) is tuple else self._native.status)
        return self._result

    def Wait(self, status: Optional[Status] = None) -> bool:
        self._finish(status)
        return True

    def wait(self, status: Optional[Status] = None):
        return self._finish(status)

    def Test(self, status: Optional[Status] = None) -> bool:
        if self._done:
            return True
        n = self._native
        if (_ftest(n) if type(n) is int else self._comm._hc.test(n)):
            self._finish(status)
            return True
        return False

    def test(self, status: Optional[Status] = None):
        return (True, self._result) if self.Test(status) else (False, None)

    def Free(self) -> None:
        self.Wait()

    def Cancel(self) -> None:  # cancellation of shm requests is not supported
        raise NotImplementedError("MPI.Request.Cancel")

    @staticmethod
    def Waitall(requests: Sequence["Request"], statuses: Optional[List[Status]] = None) -> bool:
        reqs = [r for r in requests if r is not None]
        groups = {}
        handles = []
        for r in reqs:
            if not r._done and r._native is not None:
                if type(r._native) is int:
                    handles.append(r._native)
                elif not isinstance(r._native, _h.Request):
                    continue  # collective / device request: finished below (collective
                    # rounds advance during the other waits)
                else:
                    groups.setdefault(id(r._comm), (r._comm, []))[1].append(r._native)
        if handles:
            _fwaitall(handles)
        for comm, natives in groups.values():
            comm._hc.waitall(natives)
        for i, r in enumerate(reqs):
            r._finish(statuses[i] if statuses is not None and i < len(statuses) else None)
        return True

    waitall = staticmethod(lambda requests, statuses=None: [r.wait() for r in requests])

    @staticmethod
    def Waitany(requests: Sequence["Request"], status: Optional[Status] = None) -> int:
        while True:
            for i, r in enumerate(requests):
                if r is not None and r.Test(status):
                    return i
            _time.sleep(0)

    @staticmethod
    def Testall(requests: Sequence["Request"], statuses=None) -> bool:
        return all(r.Test() for r in requests if r is not None)


class _CollRequest(Request):
    """Request of a non-blocking collective (``Comm.Iallreduce`` & co.,
    csrc/host/nbcoll.cpp): a schedule of P2P rounds that every progress call on
    the communicator advances; ``Wait`` finishes it."""

    __slots__ = ()

    def _finish(self, status: Optional[Status]):
        if not self._done:
            self._comm._hc.nb_wait(self._native)
            self._done = True
            self._keep = None
            if self._decode is not None:
                self._result = self._decode()
        return self._result

    def Test(self, status: Optional[Status] = None) -> bool:
        if self._done:
            return True
        if self._comm._hc.nb_test(self._native):
            self._finish(status)
            return True
        return False


# --------------------------------------------------------------------------
# communicator
# --------------------------------------------------------------------------
def _dumps(obj) -> bytes:
    return pickle.dumps(obj, protocol=pickle.HIGHEST_PROTOCOL)


def _loads(b) -> Any:
    return pickle.loads(b)


class Comm:
    """mpi4py-style intracommunicator over the native shared-memory plane."""

    def __init__(self, native) -> None:
        self._hc = native
        self._p = native.ptr  # raw pointer for the fastcall entry points (lives as long as _hc)
        self._rank = native.rank
        self._size = native.size
        self._nb_keep = []  # (started collective, its buffers) until the schedule is done
        self._devgrp = None  # device plane of this communicator (first CUDA-tensor call)

    def _dev(self):
        """CUDA-aware MPI: buffer collectives given CUDA tensors run on this
        communicator's device plane (IPC / xGMI kernels, created collectively on the
        first such call, like any collective)."""
        if self._devgrp is None:
            from .device import DeviceGroup

            self._devgrp = DeviceGroup(self)
        return self._devgrp

    # -- identity ----------------------------------------------------------
    def Get_rank(self) -> int:
        return self._rank

    def Get_size(self) -> int:
        return self._size

    rank = property(Get_rank)
    size = property(Get_size)

    def Get_name(self) -> str:
        return self._hc.name

    @property
    def world_ranks(self) -> List[int]:
        """Global (COMM_WORLD) rank of each member, in this comm's rank order."""
        return list(self._hc.world_ranks)

    def __eq__(self, other) -> bool:
        return isinstance(other, Comm) and other._hc is self._hc

    def __hash__(self) -> int:
        return id(self._hc)

    def __repr__(self) -> str:
        return f"<ccmpi Comm rank={self.rank}/{self.size}>"

    # -- sync ----------------------------------------------------------------
    def Barrier(self) -> None:
        _fbarrier(self._p)

    barrier = Barrier

    # -- buffer point to point ---------------------------------------------
    def Send(self, buf, dest: int, tag: int = 0) -> None:
        if _fsend(self._p, buf, dest, tag) is _NI:
            self._hc.send(_parse(buf, False).arr, dest, tag)

    Ssend = Rsend = Bsend = Send

    def Recv(self, buf, source: int = ANY_SOURCE, tag: int = ANY_TAG, status: Optional[Status] = None) -> None:
        st = _frecv(self._p, buf, source, tag)
        if st is _NI:
            st = self._hc.recv(_parse(buf, True).arr, source, tag)
        if status is not None:
            status._set(st)

    def Isend(self, buf, dest: int, tag: int = 0) -> Request:
        h = _fisend(self._p, buf, dest, tag)
        if h is not _NI:
            return Request(self, h, buf)
        b = _parse(buf, False)
        return Request(self, self._hc.isend(b.arr, dest, tag), b.arr)

    Issend = Irsend = Ibsend = Isend

    def Irecv(self, buf, source: int = ANY_SOURCE, tag: int = ANY_TAG) -> Request:
        h = _firecv(self._p, buf, source, tag)
        if h is not _NI:
            return Request(self, h, buf)
        b = _parse(buf, True)
        return Request(self, self._hc.irecv(b.arr, source, tag), b.arr)

    def Sendrecv(self, sendbuf, dest: int, sendtag: int = 0, recvbuf=None, source: int = ANY_SOURCE,
                 recvtag: int = ANY_TAG, status: Optional[Status] = None) -> None:
        st = _fsendrecv(self._p, sendbuf, dest, sendtag, recvbuf, source, recvtag)
        if st is _NI:
            s = _parse(sendbuf, False)
            r = _parse(recvbuf, True)
            st = self._hc.sendrecv(s.arr, dest, sendtag, r.arr, source, recvtag)
        if status is not None:
            status._set(st)

    def Sendrecv_replace(self, buf, dest: int, sendtag: int = 0, source: int = ANY_SOURCE,
                         recvtag: int = ANY_TAG, status: Optional[Status] = None) -> None:
        b = _parse(buf, True)
        tmp = b.arr.copy()
        st = self._hc.sendrecv(tmp, dest, sendtag, b.arr, source, recvtag)
        if status is not None:
            status._set(st)

    def Probe(self, source: int = ANY_SOURCE, tag: int = ANY_TAG, status: Optional[Status] = None) -> bool:
        st = self._hc.probe(source, tag)
        if status is not None:
            status._set(st)
        return True

    def Iprobe(self, source: int = ANY_SOURCE, tag: int = ANY_TAG, status: Optional[Status] = None) -> bool:
        st = self._hc.iprobe(source, tag)
        if st is None:
            return False
        if status is not None:
            status._set(st)
        return True

    probe, iprobe = Probe, Iprobe

    # -- object point to point ---------------------------------------------
    def send(self, obj, dest: int, tag: int = 0) -> None:
        self._hc.send(np.frombuffer(_dumps(obj), np.uint8), dest, tag)

    ssend = send

    def recv(self, buf=None, source: int = ANY_SOURCE, tag: int = ANY_TAG, status: Optional[Status] = None):
        src, tg, n = self._hc.probe(source, tag)
        data = bytearray(n)
        st = self._hc.recv(np.frombuffer(data, np.uint8) if n else np.empty(0, np.uint8), src, tg)
        if status is not None:
            status._set(st)
        return _loads(bytes(data))

    def isend(self, obj, dest: int, tag: int = 0) -> Request:
        arr = np.frombuffer(_dumps(obj), np.uint8)
        return Request(self, self._hc.isend(arr, dest, tag), arr)

    issend = isend

    def irecv(self, buf=None, source: int = ANY_SOURCE, tag: int = ANY_TAG) -> Request:
        comm = self

        class _Lazy(Request):
            def __init__(self) -> None:
                super().__init__(comm, None, None)
                self._done = False

            def _finish(self, status):
                if not self._done:
                    self._result = comm.recv(None, source, tag, status)
                    self._done = True
                return self._result

            def Test(self, status=None):
                if self._done:
                    return True
                if comm._hc.iprobe(source, tag) is not None:
                    self._finish(status)
                    return True
                return False

        return _Lazy()

    def sendrecv(self, sendobj, dest: int, sendtag: int = 0, recvbuf=None, source: int = ANY_SOURCE,
                 recvtag: int = ANY_TAG, status: Optional[Status] = None):
        req = self.isend(sendobj, dest, sendtag)
        out = self.recv(None, source, recvtag, status)
        req.Wait()
        return out

    # -- buffer collectives ---------------------------------------------------
    def Bcast(self, buf, root: int = 0) -> None:
        if _cuda(buf):
            self._dev().bcast(buf, root)
            return
        if _fbcast(self._p, buf, root) is _NI:
            self._hc.bcast(_parse(buf, True).arr, root)

    def Allreduce(self, sendbuf, recvbuf, op: Op = SUM) -> None:
        if _fallreduce(self._p, sendbuf, recvbuf, op.code) is not _NI:
            return
        if _cuda(sendbuf, recvbuf):
            self._dev().allreduce(recvbuf if sendbuf is IN_PLACE else sendbuf, recvbuf, op)
            return
        s, r = _parse(sendbuf, False), _parse(recvbuf, True)
        if s is not None and s.arr.dtype != r.arr.dtype:
            s = _parse(s.arr.astype(r.arr.dtype), False)
        self._hc.allreduce(_raw(s), r.arr, r.dt, op.code)

    def Reduce(self, sendbuf, recvbuf, op: Op = SUM, root: int = 0) -> None:
        s = _parse(sendbuf, False)
        r = _parse(recvbuf, True) if recvbuf is not None else None
        if s is None and r is None:
            raise ValueError("MPI.Reduce: need a send buffer (or IN_PLACE at root with recvbuf)")
        dt = (s or r).dt
        self._hc.reduce(_raw(s), _raw(r), dt, op.code, root)

    def Allgather(self, sendbuf, recvbuf) -> None:
        if _fallgather(self._p, sendbuf, recvbuf) is not _NI:
            return
        if _cuda(sendbuf, recvbuf):
            if sendbuf is IN_PLACE:
                blk = recvbuf.numel() // self.size
                sendbuf = recvbuf.view(-1)[self.rank * blk:(self.rank + 1) * blk]
            self._dev().allgather(sendbuf, recvbuf)
            return
        s, r = _parse(sendbuf, False), _parse(recvbuf, True)
        p = self.size
        if r.nbytes % p:
            raise ValueError("MPI.Allgather: receive buffer not divisible by comm size")
        blk = r.nbytes // p
        if s is not None and s.nbytes != blk:
            raise ValueError(f"MPI.Allgather: send {s.nbytes} B but receive block is {blk} B")
        self._hc.allgatherv(_raw(s), r.arr, [blk] * p, [blk * i for i in range(p)])

    def Allgatherv(self, sendbuf, recvbuf) -> None:
        s, r = _parse(sendbuf, False), _parse(recvbuf, True)
        counts, displs = self._vcounts(r)
        isz = r.itemsize
        self._hc.allgatherv(_raw(s), r.arr, [c * isz for c in counts], [d * isz for d in displs])

    def Gather(self, sendbuf, recvbuf, root: int = 0) -> None:
        s = _parse(sendbuf, False)
        r = _parse(recvbuf, True) if self.rank == root else None
        p = self.size
        blk = s.nbytes if s is not None else (r.nbytes // p)
        self._hc.gatherv(_raw(s), _raw(r), [blk] * p, [blk * i for i in range(p)], root)

    def Gatherv(self, sendbuf, recvbuf, root: int = 0) -> None:
        s = _parse(sendbuf, False)
        r = _parse(recvbuf, True) if self.rank == root else None
        if r is not None:
            counts, displs = self._vcounts(r)
            isz = r.itemsize
            cb, db = [c * isz for c in counts], [d * isz for d in displs]
        else:
            cb, db = [0] * self.size, [0] * self.size
        self._hc.gatherv(_raw(s), _raw(r), cb, db, root)

    def Scatter(self, sendbuf, recvbuf, root: int = 0) -> None:
        s = _parse(sendbuf, False) if self.rank == root else None
        r = _parse(recvbuf, True)
        p = self.size
        blk = r.nbytes if r is not None else s.nbytes // p
        self._hc.scatterv(_raw(s), [blk] * p, [blk * i for i in range(p)], _raw(r), root)

    def Scatterv(self, sendbuf, recvbuf, root: int = 0) -> None:
        s = _parse(sendbuf, False) if self.rank == root else None
        r = _parse(recvbuf, True)
        if s is not None:
            counts, displs = self._vcounts(s)
            isz = s.itemsize
            cb, db = [c * isz for c in counts], [d * isz for d in displs]
        else:
            cb, db = [0] * self.size, [0] * self.size
        self._hc.scatterv(_raw(s), cb, db, _raw(r), root)

    def Reduce_scatter_block(self, sendbuf, recvbuf, op: Op = SUM) -> None:
        if _freduce_scatter_block(self._p, sendbuf, recvbuf, op.code) is not _NI:
            return
        if _cuda(sendbuf, recvbuf):
            if sendbuf is IN_PLACE:
                raise ValueError("MPI.Reduce_scatter_block: IN_PLACE is not supported for CUDA tensors")
            self._dev().reduce_scatter(sendbuf, recvbuf.view(-1)[:sendbuf.numel() // self.size], op)
            return
        s, r = _parse(sendbuf, False), _parse(recvbuf, True)
        p = self.size
        if s is not None:
            if s.arr.size % p:
                raise ValueError("MPI.Reduce_scatter_block: send count not divisible by comm size")
            n = s.arr.size // p
            if r.arr.size < n:
                raise ValueError("MPI.Reduce_scatter_block: receive buffer too small")
        else:
            n = r.arr.size // p
        self._hc.reduce_scatter(_raw(s), r.arr, [n] * p, r.dt, op.code)

    def Reduce_scatter(self, sendbuf, recvbuf, recvcounts=None, op: Op = SUM) -> None:
        s, r = _parse(sendbuf, False), _parse(recvbuf, True)
        if recvcounts is None:
            recvcounts = r.counts
        if recvcounts is None:
            total = (s.arr.size if s is not None else r.arr.size)
            recvcounts = [total // self.size] * self.size
        self._hc.reduce_scatter(_raw(s), r.arr, [int(c) for c in recvcounts], r.dt, op.code)

    def Alltoall(self, sendbuf, recvbuf) -> None:
        if _falltoall(self._p, sendbuf, recvbuf) is not _NI:
            return
        if _cuda(sendbuf, recvbuf):
            self._dev().alltoall(recvbuf.clone() if sendbuf is IN_PLACE else sendbuf, recvbuf)
            return
        s, r = _parse(sendbuf, False), _parse(recvbuf, True)
        self._hc.alltoall(_raw(s), r.arr)

    # -- non-blocking collectives (MPI-3; csrc/host/nbcoll.cpp) ------------------
    # Buffers must stay untouched until the request completes; the request keeps
    # them referenced.  Every rank starts the same collectives in the same order.
    def _nb(self, native, keep) -> Request:
        # the communicator keeps the buffers alive until the schedule finished, even
        # if the caller drops the request unwaited (its rounds keep progressing)
        pend = [e for e in self._nb_keep if not e[0].done] if self._nb_keep else []
        pend.append((native, keep))
        self._nb_keep = pend
        return _CollRequest(self, native, keep)

    def Ibarrier(self) -> Request:
        return self._nb(self._hc.ibarrier(), None)

    def Ibcast(self, buf, root: int = 0) -> Request:
        b = _parse(buf, True)
        return self._nb(self._hc.ibcast(b.arr, root), b.arr)

    def Iallreduce(self, sendbuf, recvbuf, op: Op = SUM) -> Request:
        s, r = _parse(sendbuf, False), _parse(recvbuf, True)
        if s is not None and s.arr.dtype != r.arr.dtype:
            s = _parse(s.arr.astype(r.arr.dtype), False)
        return self._nb(self._hc.iallreduce(_raw(s), r.arr, r.dt, op.code), (_raw(s), r.arr))

    def Iallgather(self, sendbuf, recvbuf) -> Request:
        s, r = _parse(sendbuf, False), _parse(recvbuf, True)
        return self._nb(self._hc.iallgather(_raw(s), r.arr), (_raw(s), r.arr))

    def Ialltoall(self, sendbuf, recvbuf) -> Request:
        s, r = _parse(sendbuf, False), _parse(recvbuf, True)
        return self._nb(self._hc.ialltoall(_raw(s), r.arr), (_raw(s), r.arr))

    def Ireduce_scatter_block(self, sendbuf, recvbuf, op: Op = SUM) -> Request:
        s, r = _parse(sendbuf, False), _parse(recvbuf, True)
        return self._nb(self._hc.ireduce_scatter_block(_raw(s), r.arr, r.dt, op.code), (_raw(s), r.arr))

    def Alltoallv(self, sendbuf, recvbuf) -> None:
        s, r = _parse(sendbuf, False), _parse(recvbuf, True)
        sc, sd = self._vcounts(s)
        rc, rd = self._vcounts(r)
        si, ri = s.itemsize, r.itemsize
        self._hc.alltoallv(s.arr, [c * si for c in sc], [d * si for d in sd], r.arr,
                           [c * ri for c in rc], [d * ri for d in rd])

    def Scan(self, sendbuf, recvbuf, op: Op = SUM) -> None:
        s, r = _parse(sendbuf, False), _parse(recvbuf, True)
        self._hc.scan(_raw(s), r.arr, r.dt, op.code, False)

    def Exscan(self, sendbuf, recvbuf, op: Op = SUM) -> None:
        s, r = _parse(sendbuf, False), _parse(recvbuf, True)
        self._hc.scan(_raw(s), r.arr, r.dt, op.code, True)

    def _vcounts(self, b: _Buf):
        p = self.size
        counts = b.counts
        if counts is None:
            n = b.arr.size // p
            counts = [n] * p
        displs = b.displs
        if displs is None:
            displs, acc = [], 0
            for c in counts:
                displs.append(acc)
                acc += c
        return counts, displs

    # -- object collectives ---------------------------------------------------
    def bcast(self, obj=None, root: int = 0):
        data = self._hc.bcast_bytes(_dumps(obj) if self.rank == root else None, root)
        return obj if self.rank == root else _loads(data)

    def allgather(self, sendobj) -> list:
        return [_loads(b) for b in self._hc.allgather_bytes(_dumps(sendobj))]

    def gather(self, sendobj, root: int = 0):
        out = self._hc.gather_bytes(_dumps(sendobj), root)
        return None if out is None else [_loads(b) for b in out]

    def scatter(self, sendobj=None, root: int = 0):
        parts = [_dumps(o) for o in sendobj] if self.rank == root else None
        if parts is not None and len(parts) != self.size:
            raise ValueError("MPI.scatter: need exactly one object per rank")
        return _loads(self._hc.scatter_bytes(parts, root))

    def alltoall(self, sendobj) -> list:
        sendobj = list(sendobj)
        if len(sendobj) != self.size:
            raise ValueError(f"MPI.alltoall: need {self.size} objects, got {len(sendobj)}")
        return [_loads(b) for b in self._hc.alltoall_bytes([_dumps(o) for o in sendobj])]

    def allreduce(self, sendobj, op: Op = SUM):
        vals = self.allgather(sendobj)
        acc = vals[0]
        for v in vals[1:]:
            acc = op(acc, v)
        return acc

    def reduce(self, sendobj, op: Op = SUM, root: int = 0):
        vals = self.gather(sendobj, root)
        if vals is None:
            return None
        acc = vals[0]
        for v in vals[1:]:
            acc = op(acc, v)
        return acc

    def scan(self, sendobj, op: Op = SUM):
        vals = self.allgather(sendobj)
        acc = vals[0]
        for v in vals[1:self.rank + 1]:
            acc = op(acc, v)
        return acc

    def exscan(self, sendobj, op: Op = SUM):
        vals = self.allgather(sendobj)
        if self.rank == 0:
            return None
        acc = vals[0]
        for v in vals[1:self.rank]:
            acc = op(acc, v)
        return acc

    # -- communicator management ---------------------------------------------
    def Split(self, color: int = 0, key: int = 0) -> "Comm":
        native = self._hc.split(int(color) if color != UNDEFINED else -1, int(key))
        return COMM_NULL if native is None else Comm(native)

    def Dup(self) -> "Comm":
        return Comm(self._hc.split(0, self.rank))

    Clone = Dup

    def Free(self) -> None:
        self._hc = None
        self._p = None  # the fastcall entry points must not see the freed communicator

    def Abort(self, errorcode: int = 1) -> None:
        import os
        import sys

        sys.stderr.write(f"[ccmpi] rank {self.rank}: MPI_Abort({errorcode})\n")
        sys.stderr.flush()
        os._exit(errorcode)

    def Is_inter(self) -> bool:
        return False

    def Is_intra(self) -> bool:
        return True


class _NullComm:
    def __bool__(self) -> bool:
        return False

    def __repr__(self) -> str:
        return "MPI.COMM_NULL"

    def Get_size(self) -> int:
        raise MPIException("MPI: invalid communicator (COMM_NULL)")

    Get_rank = Get_size


COMM_NULL = _NullComm()
Intracomm = Comm

_lock = threading.Lock()
_world: Optional[Comm] = None
_self: Optional[Comm] = None
_t0 = _time.perf_counter()


def _get_world() -> Comm:
    global _world
    with _lock:
        if _world is None:
            _world = Comm(_h.HostComm.world())
        return _world


def _get_self() -> Comm:
    global _self
    w = _get_world()
    with _lock:
        if _self is None:
            _self = w.Split(w.rank, 0)
        return _self


def __getattr__(name: str):  # PEP 562: lazily bootstrap COMM_WORLD on first access
    if name == "COMM_WORLD":
        return _get_world()
    if name == "COMM_SELF":
        return _get_self()
    raise AttributeError(name)


def Wtime() -> float:
    return _h.wtime()


def Wtick() -> float:
    return 1e-9


def Init() -> None:
    _get_world()


def Init_thread(required: int = THREAD_MULTIPLE) -> int:
    _get_world()
    return THREAD_SERIALIZED


def Finalize() -> None:
    pass


def Is_initialized() -> bool:
    return _world is not None


def Is_finalized() -> bool:
    return False


def Get_processor_name() -> str:
    import socket

    return socket.gethostname()


def Get_version():
    return (VERSION, SUBVERSION)


def Query_thread() -> int:
    return THREAD_SERIALIZED


def Get_library_version() -> str:
    return "collective_communication_mpi_amd shared-memory host plane (C++)"


Exception = MPIException  # noqa: A001 - mpi4py exposes MPI.Exception
