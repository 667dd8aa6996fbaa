"""Device plane: GPU collectives for one host communicator.

``DeviceGroup`` owns a native ``DeviceComm`` (csrc/device/device_comm.cpp) and
bootstraps it over the host plane: signal-buffer and symmetric-segment IPC
handles are exchanged with the host all-gather, the RCCL unique id with the
host broadcast.  Collectives run on the caller's current HIP stream, so they
order with surrounding torch work and can be captured in a HIP graph.

Algorithms (``algo=``):

=================  ============================================================
``ll``             low-latency one-shot: (word, flag) 8-B units pushed to every
                   peer, no barriers (messages up to ``CCMPI_LL_MAX_BYTES``)
``oneshot``        every rank pulls all peers' buffers and reduces (latency)
``twoshot``        reduce-scatter + all-gather, all peers in flight (bandwidth)
``fanout``         one-phase two-shot: pull-reduce my shard from every rank, store it
                   into every rank's result (the all-gather as posted writes; 2pS
                   HBM bytes instead of (3p-1)S, no middle barrier; large default)
``fanout_lds``     the same with the peer vectors staged through LDS by DMA (buffer
                   loads into LDS: nothing held in VGPRs while in flight); measured
                   even with ``fanout`` on one GPU, a bench candidate for xGMI
``reduce_bcast``   the reference myAllreduce algorithm (mpi_wrapper/comm.py:63)
``push``           two-shot with peer writes (scatter into owners' inboxes, fan the
                   reduced shard out to every rank's result)
``ring``           hand-written pipelined ring RS+AG with peer writes on the flag
                   protocol; ``rings=k`` concurrent rings with coprime strides (k links)
``rhd``            hand-written recursive halving (RS) + doubling (AG), p = 2^k
``rccl``           vendor RCCL collective (the "library" baseline)
``auto``           tuned choice (size thresholds; ``tune()`` measures them)
=================  ============================================================

Tensors obtained from :meth:`DeviceGroup.empty` live in symmetric segments
(peer-mapped once), so collectives on them need no staging.  Any other CUDA
tensor of at least ``CCMPI_REGISTER_MIN_BYTES`` (1 MiB) is registered on
demand: one host all-gather per call carries every rank's (IPC handle,
allocation, allocator generation) of the caching-allocator segment holding
it, each distinct combination is mapped once into an LRU of
``CCMPI_REGISTER_SLOTS`` segment slots, and the kernels then read and write
the caller's tensors in place (no copy in, no copy out).  Smaller tensors are
staged through the scratch segment in identically sized chunks on every rank.
"""
from __future__ import annotations

import os
import struct
import threading
from collections import OrderedDict
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from . import _native
from .utils.trace import trace_call

_OPS = {"SUM": 0, "PROD": 1, "MIN": 2, "MAX": 3}
# all-reduce algorithms whose summation order is not rank order 0..p-1
_UNORDERED = ("ring", "rhd", "rccl")
# hand-written all-reduce algorithms -> native algorithm codes
_HAND_ALGOS = {"oneshot": "ALGO_ONESHOT", "twoshot": "ALGO_TWOSHOT", "reduce_bcast": "ALGO_REDUCE_BCAST",
               "push": "ALGO_TWOSHOT_PUSH", "ring": "ALGO_RING", "rhd": "ALGO_RHD", "ll": "ALGO_LL",
               "fanout": "ALGO_TWOSHOT_FANOUT", "fanout_lds": "ALGO_TWOSHOT_FANOUT_LDS"}


def op_code(op) -> int:
    """Map MPI.Op / string / int to the device op code."""
    if isinstance(op, int):
        return op
    name = getattr(op, "name", op)
    try:
        return _OPS[str(name).upper()]
    except KeyError:
        raise NotImplementedError(f"device reduction op {op!r} not supported (SUM, PROD, MIN, MAX)") from None


def dtype_code(torch_dtype) -> int:
    import torch

    table = {
        torch.int8: 0, torch.uint8: 1, torch.int16: 2, torch.int32: 4, torch.int64: 6,
        torch.float16: 8, torch.bfloat16: 9, torch.float32: 10, torch.float64: 11, torch.bool: 12,
    }
    try:
        return table[torch_dtype]
    except KeyError:
        raise TypeError(f"unsupported device dtype {torch_dtype}") from None


class Work:
    """Handle of a collective started with ``DeviceGroup.start``."""

    def __init__(self, group: "DeviceGroup", done, result, keep) -> None:
        self.group, self.done, self.result, self._keep = group, done, result, keep

    def is_completed(self) -> bool:
        return self.done.query()

    def wait(self):
        """Order the current stream after the collective (no host sync); returns
        the collective's output tensor."""
        torch = self.group.torch
        torch.cuda.current_stream(self.group.device).wait_event(self.done)
        pend = self.group._async_done
        if pend is not None and pend[1] is self.done:
            self.group._async_done = None  # the current stream is now ordered after it
        self._keep = None
        return self.result

    def synchronize(self):
        """Block the host until the collective finished; raises on a device timeout."""
        self.done.synchronize()
        self.group.check()
        self._keep = None
        return self.result


def alltoallv_plan(counts, me: int, es: int):
    """Byte offsets of rank ``me``'s ragged all-to-all from the p x p count matrix
    (``counts[i][j]`` = elements rank i sends to rank j; both sides packed in rank
    order): (send offset of each peer's segment, offset in each peer's output where
    this rank's segment lands, segment lengths, the largest total send of any rank,
    which sizes the grid identically on every rank)."""
    b = np.asarray(counts, dtype=np.int64) * int(es)
    p = b.shape[0]
    soff = [int(x) for x in np.concatenate([[0], np.cumsum(b[me])[:-1]])]
    doff = [int(b[:me, j].sum()) for j in range(p)]
    return soff, doff, [int(x) for x in b[me]], int(b.sum(axis=1).max())


def stale_keys(keys, key) -> List[tuple]:
    """On-demand registration slots that ``key`` invalidates: a slot is keyed by one
    (IPC handle, allocation base, bytes, allocator generation) per rank; it is stale
    when, on some rank, its allocation overlaps the new one's address range but is
    not the same allocation (the range was freed and reallocated).  Pure function of
    the keys, which every rank holds identically, so every rank drops the same slots."""
    out = []
    for k in keys:
        for a, b in zip(k, key):
            if a != b and a[1] < b[1] + b[2] and b[1] < a[1] + a[2]:
                out.append(k)
                break
    return out


def tuning_key(size: int, ranks_per_device: int, device_name: str) -> str:
    """Identity of a tuning table: group size, GPU sharing and device model."""
    return f"p{size}-share{ranks_per_device}-{device_name}"


def load_tuning(path: str, key: str) -> Dict[Tuple[int, int], str]:
    """{(size, log2 bytes): algo} saved by ``save_tuning`` for ``key``; {} if absent."""
    import json

    try:
        with open(path) as f:
            tables = json.load(f)
    except (OSError, ValueError):
        return {}
    out = {}
    for k, algo in tables.get(key, {}).items():
        size, lg = (int(v) for v in k.split(","))
        out[(size, lg)] = str(algo)
    return out


def save_tuning(path: str, key: str, table: Dict[Tuple[int, int], str]) -> None:
    """Merge ``table`` into the JSON file at ``path`` under ``key`` (atomic rename)."""
    import json

    try:
        with open(path) as f:
            tables = json.load(f)
    except (OSError, ValueError):
        tables = {}
    tables[key] = {f"{s},{lg}": a for (s, lg), a in sorted(table.items())}
    tmp = f"{path}.tmp{os.getpid()}"
    with open(tmp, "w") as f:
        json.dump(tables, f, indent=1, sort_keys=True)
    os.replace(tmp, path)


def row_mode_key(tune_key: str) -> str:
    """Tuning-file key of the TP row-parallel output modes measured for one group identity."""
    return f"rowmode:{tune_key}"


def load_row_modes(path: str, tune_key: str) -> Dict[Tuple[int, int], str]:
    """{(M, N): row-parallel mode} measured for groups of ``tune_key`` (``save_row_modes``)."""
    import json

    try:
        with open(path) as f:
            tables = json.load(f)
    except (OSError, ValueError):
        return {}
    out = {}
    for k, mode in tables.get(row_mode_key(tune_key), {}).items():
        m, n = (int(v) for v in k.split(","))
        out[(m, n)] = str(mode)
    return out


def save_row_modes(path: str, tune_key: str, table: Dict[Tuple[int, int], str]) -> None:
    """Merge the row-mode table into the tuning file (same file as ``save_tuning``)."""
    import json

    try:
        with open(path) as f:
            tables = json.load(f)
    except (OSError, ValueError):
        tables = {}
    tables[row_mode_key(tune_key)] = {f"{m},{n}": mode for (m, n), mode in sorted(table.items())}
    tmp = f"{path}.tmp{os.getpid()}"
    with open(tmp, "w") as f:
        json.dump(tables, f, indent=1, sort_keys=True)
    os.replace(tmp, path)


class _CountingComm:
    """Proxy of the host communicator that counts the host calls the device plane makes
    (``calls``): a steady-state device collective should make none (tests)."""

    def __init__(self, comm) -> None:
        self._comm = comm
        self.calls = 0

    def __getattr__(self, name):
        attr = getattr(self._comm, name)
        if not callable(attr):
            return attr

        def counted(*a, **k):
            self.calls += 1
            return attr(*a, **k)

        return counted


# set by any DeviceGroup of this process whose ranks share one GPU (tensor_parallel uses it
# for groups of one rank, which cannot measure sharing themselves)
SHARED_GPU_IN_PROCESS = False


def _env_int(name: str, default: int) -> int:
    v = os.environ.get(name)
    return int(v) if v else default


def device_identity(props) -> str:
    """Identity of a physical GPU across processes: its UUID plus PCI domain:bus:device.
    Not the device ordinal -- with one visible device per rank (per-rank isolation) every
    rank's GPU is ordinal 0 -- and not the bus number alone: two GPUs in different PCI
    domains can share a bus number.  Ranks whose identities are equal share one GPU."""
    uuid = str(getattr(props, "uuid", "") or "")
    if uuid.strip("0-") == "":
        uuid = ""  # an all-zero UUID identifies nothing
    return (f"{uuid}|{getattr(props, 'pci_domain_id', 0):04x}:{getattr(props, 'pci_bus_id', 0):02x}:"
            f"{getattr(props, 'pci_device_id', 0):02x}|{props.name}")


class DeviceGroup:
    """GPU side of a communicator (one per host communicator per process)."""

    def __init__(self, host_comm, device=None, scratch_bytes: Optional[int] = None) -> None:
        import torch

        self.torch = torch
        self.host = _CountingComm(host_comm)
        self.rank = host_comm.Get_rank()
        self.size = host_comm.Get_size()
        if device is None:
            n = torch.cuda.device_count()
            local = int(os.environ.get("CCMPI_LOCAL_RANK", os.environ.get("LOCAL_RANK", "0")))
            device = torch.device("cuda", local % max(n, 1))
        self.device = torch.device(device)
        torch.cuda.set_device(self.device)
        self.D = _native.device()
        self.dc = self.D.DeviceComm(self.rank, self.size, self.device.index or 0)
        self.dc.connect([bytes(h) for h in host_comm.allgather(bytes(self.dc.signal_handle()))])
        # how many ranks share each physical GPU (multi-process-per-GPU testing):
        # all their CTAs must be co-resident (CTA b of one rank spins on CTA b
        # of the others), so the total over the sharing ranks is capped at 512
        # (~117 VGPRs -> 4 CTAs of 256 threads per CU fit; 2 per CU are used).
        # Measured (profiles/r2_coll): 512 CTAs in total move 0.65-0.86 of the
        # HBM roofline on 64-256 MiB collectives, 96 in total only 0.3, 1024 less
        # than 512.  One rank per GPU gets the same 512 (2 CTAs per CU).
        props = torch.cuda.get_device_properties(self.device)
        key = device_identity(props)
        keys = host_comm.allgather(key)
        self.ranks_per_device = keys.count(key)
        self.shared_device = self.ranks_per_device > 1
        self.shared_ring = self.shared_device and os.environ.get("CCMPI_SHARED_RING") == "1"
        if self.shared_device:
            global SHARED_GPU_IN_PROCESS
            SHARED_GPU_IN_PROCESS = True
            # The LDS-ring GEMM needs a whole CU per workgroup (128 KiB LDS, 512 VGPRs a
            # wave); next to another rank's spinning collective CTAs (one per CU) none of
            # its workgroups can start, and the two ranks wait on each other (TP = 2 MLP
            # on one GPU timed out, profiles/r3_tp2).  A process whose GPU is shared uses
            # the smaller-footprint kernels instead -- unless CCMPI_SHARED_RING=1: then
            # every collective of every sharing rank stays within half the CUs in total
            # (below), so the ring GEMM always finds free CUs (the kernels an 8-GPU TP run
            # uses, exercised beside another rank's collectives on one GPU)
            if not self.shared_ring:
                self.D.gemm_set_ring_min(0)
            # the fused attention forward's fold-only workgroups help only on a GPU with CUs
            # to spare; several ranks' kernels already fill it (profiles/r6_attn)
            self.D.attn_set_qkv_fold_grid(0)
        self._async_done = None  # (stream, event) of the last start()ed collective, until ordered
        self._inflight: List = []  # (done event, tensors) of start()ed collectives not yet known complete
        default_blocks = max(1, 512 // self.ranks_per_device)
        self.max_blocks = _env_int("CCMPI_MAX_BLOCKS", default_blocks)
        if self.shared_device and self.shared_ring:
            self.max_blocks = min(self.max_blocks, self._shared_cap())
        # CTA budget of collectives that run NEXT TO compute (DP gradient buckets, TP
        # pipelines on side streams): spinning collective CTAs hold CU slots the GEMMs
        # could use, and with ranks sharing a GPU a 256-CTA bucket all-reduce beside
        # another rank's GEMMs never became co-resident (timeouts, profiles/r2_overlap);
        # 64 CTAs keep both the GEMMs and the collective moving
        self.overlap_blocks = min(self.max_blocks, _env_int("CCMPI_OVERLAP_BLOCKS", 64))
        # Upper bound of that budget.  With ranks sharing a GPU, one rank's spinning grid
        # must leave CUs free: a bucket all-reduce of 256 CTAs (one per CU) beside the
        # other rank's backward blocked every GEMM workgroup of that rank, so the peer
        # never arrived -- 60 s device timeout, then both processes' queues were torn down
        # (hipErrorIllegalAddress, profiles/r4_dp).  All sharing ranks together on half
        # the CUs at most; no bound when every rank owns its GPU (its peers progress on
        # their own devices).
        self.overlap_cap = self._shared_cap() if self.shared_device else self.max_blocks
        self.overlap_blocks = min(self.overlap_blocks, self.overlap_cap)
        if scratch_bytes is None:
            scratch_bytes = _env_int("CCMPI_SCRATCH_MB", 64 if self.shared_device else 512) << 20
        self._keep: List = []   # registered segments (scratch, heap arenas) live as long as the group
        self.heap = self.D.SymHeap()
        self.arena_bytes = _env_int("CCMPI_HEAP_ARENA_MB", 256) << 20
        self._inbox = None
        self.scratch = torch.empty(max(scratch_bytes, 1 << 16), dtype=torch.uint8, device=self.device)
        seg = self._register(self.scratch)
        assert seg == 0, "scratch must be segment 0"
        self._rccl = False
        # one-shot reads p x the message; above LL sizes the one-phase fan-out wins
        # from 2 MiB at 2 ranks and from 64 KiB beyond (profiles/r2_coll/fanout.md)
        self.oneshot_max = _env_int("CCMPI_ONESHOT_MAX_BYTES", (1 << 20) if self.size <= 2 else (64 << 10))
        self.ll_max = (_env_int("CCMPI_LL_MAX_BYTES", 512 << 10) + 15) // 16 * 16
        # LL pushes 2 x the payload to each of the p-1 peers: up to 256 KiB at 2 ranks,
        # 64 KiB beyond (profiles/r2_coll/ll_latency.md).  With > 2 ranks SHARING a GPU
        # the polling ranks compete with their peers' pushes for the same CUs and LL
        # loses to one-shot from 8 KiB (small_p4/p8.jsonl): 4 KiB there
        ll_default = (256 << 10) if self.size <= 2 else ((4 << 10) if self.shared_device else (64 << 10))
        self.ll_auto_max = min(self.ll_max, _env_int("CCMPI_LL_AUTO_MAX_BYTES", ll_default))
        # deterministic mode: only algorithms that reduce in rank order
        # 0..p-1 (bitwise identical on every rank and to a sequential fp32 sum in rank
        # order, like the reference's root loop, comm.py:85-93); ring / rhd / RCCL are
        # replaced by the fan-out two-shot kernel
        self.deterministic = os.environ.get("CCMPI_DETERMINISTIC", "0") not in ("0", "")
        # algorithms `auto` must not pick (CCMPI_DISABLE_ALGOS, or failed self_test())
        self.disabled = {a for a in os.environ.get("CCMPI_DISABLE_ALGOS", "").split(",") if a}
        # concurrent rings of algo="ring": every stride coprime to p, up to 4 (p = 8: strides
        # 1, 3, 5, 7 -> 4 links per direction); CCMPI_RINGS overrides
        coprime = [k for k in range(1, self.size) if _gcd(k, self.size) == 1] or [1]
        self.default_rings = _env_int("CCMPI_RINGS", min(4, len(coprime)))
        self.inbox_cap = _env_int("CCMPI_INBOX_MAX_MB", 1024) << 20
        self.tuned: Dict[Tuple[int, int], str] = {}
        # persisted tune() results (CCMPI_TUNE_FILE), keyed by group size, GPU sharing and model
        self.tune_key = tuning_key(self.size, self.ranks_per_device, props.name)
        self.tune_file = os.environ.get("CCMPI_TUNE_FILE")
        # TP row-parallel output mode per (M, N), measured by the bench's mlp phase
        # (tensor_parallel._row_mode reads it for mode "auto")
        self.row_modes: Dict[Tuple[int, int], str] = {}
        if self.tune_file:
            self.tuned.update(load_tuning(self.tune_file, self.tune_key))
            self.row_modes.update(load_row_modes(self.tune_file, self.tune_key))
        # on-demand registration of ordinary CUDA tensors (collectives >= reg_min bytes)
        self.reg_min = _env_int("CCMPI_REGISTER_MIN_BYTES", 1 << 20)  # 0 = off
        self.reg_slots = max(1, _env_int("CCMPI_REGISTER_SLOTS", 32))
        self._dyn: "OrderedDict[tuple, int]" = OrderedDict()  # identity of every rank's allocation -> slot
        self._exports: Dict[int, Tuple[bytes, int, int]] = {}  # allocation base -> (handle, base, bytes)
        self._free_slots: List[int] = []  # released slot indices (reused before new ones)
        self.registrations = 0  # slots (re)mapped so far (tests, traces)
        # slots a captured HIP graph resolves: never evicted or cleared (the graph baked
        # in their (segment, offset) codes); see _register_call / unpin_captured
        self._pinned: set = set()
        # persistent symmetric-heap buffers by key (persistent()): allocated once, so the
        # steady state allocates nothing and makes no host call
        self._persist: Dict[tuple, object] = {}
        # CCMPI_VERIFY_SYMMETRIC=1: every heap-only collective >= reg_min checks with one
        # host all-gather that every rank passed heap blocks (debug; off = no host call)
        self.verify_symmetric = os.environ.get("CCMPI_VERIFY_SYMMETRIC", "0") not in ("0", "")
        self._lock = threading.Lock()
        self._watchdog: Optional[threading.Thread] = None
        mode = os.environ.get("CCMPI_WATCHDOG", "warn").lower()
        if mode in ("warn", "abort"):
            self.start_watchdog(mode)

    @property
    def host_calls(self) -> int:
        """Host-plane calls this group has made (bootstrap, registration, heap growth)."""
        return self.host.calls

    # ---------------------------------------------------------------- watchdog
    def start_watchdog(self, mode: str = "warn", period_s: float = 0.2) -> None:
        """Host-side watchdog.  Device kernels never hang: every
        spin is bounded (``CCMPI_DEVICE_TIMEOUT_S``) and a timeout writes a
        rank/phase/peer code into pinned host memory.  This daemon thread polls
        that word *without* synchronising the device and reports it once per
        code (``warn``), or prints a rank-tagged message and aborts the whole
        process (``abort``) so the launcher tears the job down."""
        if self._watchdog is not None:
            return
        dc, rank = self.dc, self.rank
        stop = self._wd_stop = threading.Event()

        def run():
            import sys

            last = 0
            while not stop.wait(period_s):
                code = dc.poll_error()
                if code and code != last:
                    msg = (f"[ccmpi watchdog] rank {rank}: device collective timed out "
                           f"(code 0x{code:x}: phase {code >> 8}, waiting on peer {code & 0xff})")
                    print(msg, file=sys.stderr, flush=True)
                    if mode == "abort":
                        os._exit(70)
                last = code

        self._watchdog = threading.Thread(target=run, name=f"ccmpi-watchdog-{rank}", daemon=True)
        self._watchdog.start()

    def stop_watchdog(self) -> None:
        if self._watchdog is not None:
            self._wd_stop.set()
            self._watchdog.join()
            self._watchdog = None

    # ------------------------------------------------------------------ memory
    def _register(self, t) -> int:
        """Collectively register tensor storage as a symmetric segment."""
        h, off = self.dc.export_range(t.data_ptr())
        allh = self.host.allgather((bytes(h), int(off)))
        seg = self.dc.add_segment(t.data_ptr(), t.numel() * t.element_size(),
                                  [x[0] for x in allh], [x[1] for x in allh])
        self._keep.append(t)
        if self._rccl_registering():
            self.dc.rccl_register_segments()
        return seg

    def _rccl_registering(self) -> bool:
        return getattr(self, "_rccl", False) and os.environ.get("CCMPI_RCCL_REGISTER") == "1"

    def empty(self, shape, dtype=None):
        """Collective symmetric allocation (same call sequence on every rank).

        Blocks come from the symmetric heap (csrc/device/symheap.cpp): a
        best-fit allocator over IPC-registered arenas of ``CCMPI_HEAP_ARENA_MB``
        (default 256 MiB, or the request if larger), grown collectively when
        full.  The tensor owns its block through a DLPack deleter: the block
        returns to the heap when the last view dies.  As with torch's caching
        allocator, reuse is ordered only with work on the allocating (current)
        stream: keep a tensor used on a side stream alive until that stream has
        been joined.  Peers' writes into a block never outlive the collective
        that made them: a rank's kernel ends only after every peer write into
        its buffers has landed (end barrier, or the per-step flags it awaits).
        """
        torch = self.torch
        dtype = dtype or torch.float32
        if isinstance(shape, int):
            shape = (shape,)
        n = 1
        for s in shape:
            n *= int(s)
        nbytes = n * torch.empty((), dtype=dtype).element_size()
        need = max(nbytes, 1)
        idx = self.device.index or 0
        cap = self.heap.block(need, idx)
        # Whether the heap grows is decided collectively: blocks return to the heap
        # when their last view dies, which can happen at different times on different
        # ranks (GC, autograd, unwaited work), so a local "no block" must not start
        # the registration all-gather on one rank only.  Every rank grows when any
        # rank needs to, by the largest request.
        grow = self.host.allreduce(0 if cap is not None else need, op=_host_max())
        if grow:
            self._grow_heap(grow)
            if cap is None:
                cap = self.heap.block(need, idx)
        raw = torch.utils.dlpack.from_dlpack(cap)
        return raw[:nbytes].view(dtype).view(shape)

    def _grow_heap(self, need: int) -> None:
        """Collective: register one more arena (every rank grows at the same call,
        by the same ``need``)."""
        arena = max(self.arena_bytes, (need + (2 << 20) - 1) // (2 << 20) * (2 << 20) + 4096)
        raw = self.torch.empty(arena, dtype=self.torch.uint8, device=self.device)
        self._register(raw)
        self.heap.add_arena(raw.data_ptr(), arena)

    def persistent(self, key, shape, dtype=None):
        """A symmetric-heap buffer cached under ``(key, shape, dtype)``: the first call
        allocates it (collective, like ``empty``; every rank must ask for the same keys in
        the same order), later calls return the same tensor with no host call.  For
        scratch that never escapes its owner -- the TP layers' GEMM partial products,
        which their all-reduce clobbers (``allreduce_to_local``)."""
        torch = self.torch
        dtype = dtype or torch.float32
        shape = (shape,) if isinstance(shape, int) else tuple(int(s) for s in shape)
        k = (key, shape, dtype)
        t = self._persist.get(k)
        if t is None:
            t = self._persist[k] = self.empty(shape, dtype)
        return t

    def scratch_view(self, key, shape, dtype=None):
        """Grow-only persistent symmetric scratch under ``(key, dtype)``: one heap block per
        key, reallocated (collectively, to the new size) only when a call needs more than it
        holds; every smaller request is a view of it.  Variable token counts (eval, packing,
        a last partial batch) then reuse one block instead of leaking one per shape, and the
        steady state makes no host call.  Every rank must ask for the same keys and sizes in
        the same order (the TP layers do: same shapes on every rank of the group)."""
        torch = self.torch
        dtype = dtype or torch.float32
        shape = (shape,) if isinstance(shape, int) else tuple(int(s) for s in shape)
        n = 1
        for d in shape:
            n *= d
        k = ("grow", key, dtype)
        t = self._persist.get(k)
        if t is None or t.numel() < n:
            if t is not None:
                # the old block returns to the heap: no queued kernel of this rank may still use it
                torch.cuda.synchronize(self.device)
                del self._persist[k]
                t = None
            t = self._persist[k] = self.empty(max(n, 1), dtype)
        return t[:n].view(shape)

    def release_persistent(self, key=None) -> None:
        """Drop cached persistent buffers (all, or those of ``key``); their blocks return
        to the heap when no other reference remains."""
        for k in [k for k in self._persist if key is None or k[0] == key or (k[0] == "grow" and k[1] == key)]:
            del self._persist[k]

    def zeros(self, shape, dtype=None):
        t = self.empty(shape, dtype)
        t.zero_()
        return t

    def is_symmetric(self, t) -> bool:
        seg, _ = self.dc.find(t.data_ptr(), t.numel() * t.element_size())
        return seg > 0

    def _ensure_ll(self) -> None:
        """Collective on first use: every rank allocates its uncached LL buffer
        (2 parities x p sources x 2 x ``ll_max`` bytes; 16 MiB at p = 8) and maps
        every peer's through IPC."""
        if self.dc.ll_max_bytes:
            return
        h = bytes(self.dc.ll_alloc(self.ll_max))
        self.dc.ll_connect([bytes(x) for x in self.host.allgather(h)])

    def _ensure_inbox(self, nbytes: int) -> None:
        """Collective (all ranks call with the same size): symmetric inbox of
        p shards for the push two-shot all-reduce (p - 1 chunk slots for the
        ring / rhd schedules), grown on demand up to ``CCMPI_INBOX_MAX_MB``;
        ring / rhd process larger buffers in inbox-sized pieces."""
        shard = ((nbytes + self.size - 1) // self.size + 15) // 16 * 16
        need = min(shard * self.size, max(self.inbox_cap, 1 << 20))
        if self.dc.inbox_bytes >= need:
            return
        cap = max(need, 64 << 20)
        self.dc.set_inbox(0, 0)
        self._inbox = None  # old inbox back to the heap first (same order on every rank)
        self._inbox = self.empty(cap, self.torch.uint8)
        self.dc.set_inbox(self._inbox.data_ptr(), cap)

    # ------------------------------------------- fused row-parallel GEMM + all-reduce
    def _ensure_fused(self, tiles: int) -> None:
        """Collective on first use / growth: the peer-mapped fused-GEMM state (tickets,
        slot and done flags) and a symmetric inbox of ceil(tiles / p) * p bf16 tile slots."""
        if self.dc.fused_inbox_bytes == 0 and not getattr(self, "_fused_connected", False):
            h = bytes(self.dc.fused_alloc())
            self.dc.fused_connect([bytes(x) for x in self.host.allgather(h)])
            self._fused_connected = True
        need = (tiles + self.size - 1) // self.size * self.size * (256 * 256 * 2)
        if self.dc.fused_inbox_bytes >= need:
            return
        self.torch.cuda.synchronize(self.device)
        self._fused_inbox = None  # back to the heap first (same order on every rank)
        self._fused_inbox = self.empty(need, self.torch.uint8)
        ptr = self._fused_inbox.data_ptr()
        codes = self.host.allgather(int(self.dc.code_of(ptr, need)))
        self.dc.set_fused_inbox(ptr, need, codes)

    def gemm_allreduce(self, x, w, bias=None, out=None, alpha: float = 1.0):
        """Row-parallel layer output: ``sum over the group of x_r @ w_r^T (+ bias)`` in bf16,
        with the all-reduce fused into the GEMM (csrc/device/gemm_w4.hip): every output
        tile's partials go straight from the GEMM epilogues into the tile owner's inbox,
        and the last rank to finish the tile reduces it in rank order and writes it into
        every rank's output.  x: [M, K_r] bf16, w: [N, K_r] bf16 (K_r % 64 == 0), bias: [N]
        fp32 / bf16.  ``out`` (default: a symmetric-heap block) is registered on demand.
        Collective: every rank calls with the same M, N."""
        torch = self.torch
        if x.dtype != torch.bfloat16 or w.dtype != torch.bfloat16 or x.dim() != 2 or w.dim() != 2:
            raise TypeError("gemm_allreduce: x [M, K] and w [N, K] must be 2-D bf16")
        M, K = x.shape
        N = w.shape[0]
        if w.shape[1] != K or x.stride(1) != 1 or w.stride(1) != 1:
            raise ValueError("gemm_allreduce: shape mismatch or non K-contiguous operand")
        tiles = ((M + 255) // 256) * ((N + 255) // 256)
        self._ensure_fused(tiles)
        if out is None:
            out = self.empty((M, N), torch.bfloat16)
        elif not (self._symm(out) or self._register_call((out,))):  # heap blocks: no host call
            raise ValueError("gemm_allreduce: out could not be registered")
        bk, bp = 0, 0
        if bias is not None:
            bk = 1 if bias.dtype == torch.float32 else 2
            bp = bias.data_ptr()
        self.dc.gemm_rowpar(x.data_ptr(), w.data_ptr(), out.data_ptr(), bp, M, N, K, x.stride(0), w.stride(0),
                            out.stride(0), float(alpha), bk, self._stream())
        return out

    def gemm_push_allreduce(self, x, w, out, alpha: float = 1.0, max_blocks: Optional[int] = None):
        """Row-parallel layer output ``out = sum over the group of x_r @ w_r^T`` (bf16, no
        bias) with the reduce-scatter's traffic inside the GEMM: the GEMM epilogue stores
        row block j of this rank's partial (M / p rows) straight into rank j's inbox slot
        as posted writes (over xGMI while the other tiles still compute), then one
        inbox-to-local two-shot reduces the slots and pulls every block into ``out``
        (``DeviceComm::gemm_push_rowpar``).  No CTA spins inside the GEMM.  The inbox is a
        persistent symmetric-heap block of the output's size.  x: [M, K_r], w: [N, K_r];
        M % (256 p) == 0, K_r % 64 == 0, N % 8 == 0; ``out`` any local [M, N] bf16 tensor.
        Collective: every rank calls with the same M, N."""
        torch = self.torch
        if x.dtype != torch.bfloat16 or w.dtype != torch.bfloat16 or x.dim() != 2 or w.dim() != 2:
            raise TypeError("gemm_push_allreduce: x [M, K] and w [N, K] must be 2-D bf16")
        M, K = x.shape
        N = w.shape[0]
        if w.shape[1] != K or x.stride(1) != 1 or w.stride(1) != 1 or tuple(out.shape) != (M, N) \
                or not out.is_contiguous() or out.dtype != torch.bfloat16:
            raise ValueError("gemm_push_allreduce: shape mismatch, non K-contiguous operand or bad output")
        inbox = self.scratch_view("gemm_push_inbox", (M * N,), torch.bfloat16)
        self.dc.gemm_push_rowpar(x.data_ptr(), w.data_ptr(), out.data_ptr(), inbox.data_ptr(), M, N, K, x.stride(0),
                                 w.stride(0), float(alpha), self._stream(), self._budget(max_blocks))
        return out

    # -------------------------------------------------------------------- rccl
    def ensure_rccl(self) -> None:
        """Collective: create the RCCL communicator on first use."""
        if self._rccl:
            return
        uid = self.D.rccl_unique_id() if self.rank == 0 else None
        uid = self.host.bcast(uid, root=0)
        self.dc.rccl_init(uid)
        self._rccl = True
        if os.environ.get("CCMPI_RCCL_REGISTER") == "1":  # user-buffer registration of the symmetric heap
            self.dc.rccl_register_segments()

    def split_rccl_into(self, child: Optional["DeviceGroup"], color: int, key: int) -> None:
        """Collective over THIS group's ranks: derive the child group's RCCL
        communicator with ncclCommSplit (shares the parent's RCCL resources)
        instead of a fresh unique-id bootstrap.  ``child`` is None on ranks
        that join no child (UNDEFINED color)."""
        if not self._rccl:
            return
        if child is None:
            self.D.DeviceComm.rccl_split_nocolor(self.dc)
            return
        child.dc.rccl_split_from(self.dc, color, key)
        child._rccl = True

    # ----------------------------------------------------------------- helpers
    def _stream(self) -> int:
        cur = self.torch.cuda.current_stream(self.device)
        if self._async_done is not None and self._async_done[0] != cur.cuda_stream:
            self._order_after_async(cur)
        return cur.cuda_stream

    def _order_after_async(self, cur) -> None:
        """A collective issued on another stream than the last ``start()``ed one waits
        for it on the device: one collective of a group at a time (they share the
        per-CTA epochs, flags and the staging scratch), while compute on that stream
        still overlaps the started collective."""
        if self.torch.cuda.is_current_stream_capturing():
            raise RuntimeError("wait() on the started collective before capturing another collective of this group")
        cur.wait_event(self._async_done[1])
        self._async_done = None

    def _check(self, t, name: str):
        if not (hasattr(t, "is_cuda") and t.is_cuda):
            raise TypeError(f"{name} must be a CUDA tensor")
        if not t.is_contiguous():
            raise ValueError(f"{name} must be contiguous")
        return t

    def _budget(self, max_blocks: Optional[int]) -> int:
        """Per-rank CTA budget.  Ranks sharing a GPU spin on each other's CTAs, so
        their grids must be co-resident.  The kernels' VGPR use allows 4 CTAs per
        CU, but a grid that needs every slot of every CU (1024 in total) was seen
        to leave some CTAs undispatched behind spinning ones (timeout): the total
        is capped at 512 (2 per CU)."""
        mb = max_blocks or self.max_blocks
        if self.shared_device:
            mb = min(mb, self._shared_cap() if self.shared_ring else max(1, 512 // self.ranks_per_device))
        return mb

    def _shared_cap(self) -> int:
        """CCMPI_SHARED_RING: per-rank CTA cap keeping all sharing ranks' collectives on
        at most half the CUs."""
        cus = getattr(self, "_cus", None)
        if cus is None:
            cus = self._cus = _cu_count(self.device)  # one device query per group
        return max(1, (cus // 2) // self.ranks_per_device)

    def _symm(self, *ts) -> bool:
        return all(self.is_symmetric(t) and t.data_ptr() % 16 == 0 for t in ts)

    def _symm_call(self, nbytes: int, *ts, promise: Optional[bool] = None) -> bool:
        """The ``symmetric`` decision of one collective, identical on every rank.
        Below ``reg_min`` bytes (or with registration off): every tensor from the
        symmetric heap (the caller's promise).  From ``reg_min`` up: collective
        on-demand registration of whatever the tensors live in (one host all-gather;
        a rank-local check is not enough there: a view at a rank-dependent offset can be
        aligned on one rank and not on another).  ``promise=True``: the caller guarantees
        heap blocks of the same layout on every rank (DDP buckets, persistent TP scratch,
        the bench's buffers) -- no host call; ``CCMPI_VERIFY_SYMMETRIC=1`` checks it."""
        if promise:
            ok = self._symm(*ts)
            if self.verify_symmetric and not all(self.host.allgather(ok)):
                raise RuntimeError("collective: symmetric=True promised, but not every rank passed aligned heap blocks")
            if not ok:
                raise ValueError("collective: symmetric=True needs 16-B aligned symmetric-heap tensors")
            return True
        if self.size == 1:
            return self._symm(*ts)
        if self.reg_min <= 0 or nbytes < self.reg_min:
            ok = self._symm(*ts)
            if nbytes > self.scratch.numel() // 2:
                # rank-local so far, and beyond half the scratch the ring / RHD launch sequence
                # depends on the decision (symmetric: pieces bounded by the inbox alone; staged:
                # half-scratch pieces): agree on it, or one rank issues 1 launch and another N
                ok = all(self.host.allgather(ok))
            return ok
        return self._register_call(ts)

    def _alloc_generation(self) -> int:
        """Segments this process's caching allocator has returned to the driver (the
        fallback identity when the driver has no allocation ids)."""
        try:
            return int(self.torch._C._cuda_memoryStats(self.device.index or 0)["segment"]["all"]["freed"])
        except Exception:  # noqa: BLE001 - stats unavailable: assume nothing is ever freed
            return 0

    def _alloc_identity(self, base: int) -> int:
        """Identity of the allocation at ``base``: the driver's unique buffer id (a range
        freed and reallocated at the same address gets a new one, an unrelated free
        changes nothing), or the allocator's global free count if the driver has none."""
        aid = self.D.DeviceComm.alloc_id(base)
        return (1 << 63) | aid if aid else self._alloc_generation()

    def _export(self, ptr: int):
        """(IPC handle, allocation base, allocation bytes, identity) of the allocation
        holding ``ptr``; cached per base while the base's identity is unchanged."""
        for base, ent in list(self._exports.items()):
            if base <= ptr < base + ent[2]:
                if self._alloc_identity(base) == ent[3]:
                    return ent
                del self._exports[base]  # freed and reallocated: export the new allocation
                break
        h, base, size = self.dc.export_alloc(ptr)
        ent = (h, base, size, self._alloc_identity(base))
        self._exports[base] = ent
        return ent

    def _register_call(self, ts) -> bool:
        """Collective: map the allocations holding ``ts`` on every rank into peer-visible
        segment slots.  Returns False (staged path, on every rank) when any rank's
        tensor cannot be exported or is misaligned, or when a new mapping would be
        needed during a HIP graph capture."""
        mine = []
        for t in ts:
            if t.data_ptr() % 16:
                mine = None
                break
            if self.is_symmetric(t):
                mine.append(None)  # a heap block: already mapped everywhere
                continue
            try:
                mine.append(self._export(t.data_ptr()))
            except Exception:  # noqa: BLE001 - not an exportable device allocation
                mine = None
                break
        rows = self.host.allgather(mine)
        if any(r is None for r in rows):
            return False
        capturing = self.torch.cuda.is_current_stream_capturing()
        used = set()  # slots this call resolves: not evictable while it maps the others
        for i in range(len(ts)):
            if all(r[i] is None for r in rows):
                continue  # heap blocks on every rank
            ids = []
            for j, r in enumerate(rows):
                if r[i] is None:  # heap on rank j: its arena allocation is the mapping
                    ids.append(None)
                else:
                    ids.append(r[i])
            if any(x is None for x in ids):
                # mixed heap / non-heap: every rank maps its own allocation; heap ranks
                # export their arena (never freed while the group lives)
                mine_i = self._export(ts[i].data_ptr()) if mine[i] is None else mine[i]
                ids = self.host.allgather(mine_i)
            key = tuple(ids)
            used.add(key)
            slot = self._dyn.get(key)
            if slot is not None:
                self._dyn.move_to_end(key)
                if capturing:
                    self._pinned.add(key)  # the graph bakes in this slot's codes
                continue
            if capturing:
                return False
            self._map_slot(key, keep=used)
        return True

    def unpin_captured(self) -> None:
        """Release the slots pinned by HIP-graph captures (call after dropping every graph
        that captured collectives on registered tensors): they may be evicted again."""
        self._pinned.clear()

    def _map_slot(self, key, keep=()) -> None:
        """Collective: map the allocation set ``key`` (one (handle, base, bytes, gen) per
        rank) into a slot.  Slots holding an older allocation at an overlapping address
        on any rank are released first (every rank sees the same keys, so the slot
        table stays identical everywhere)."""
        torch = self.torch
        stale = stale_keys(self._dyn.keys(), key)
        pinned = [k for k in stale if k in self._pinned]
        if pinned:
            # a captured graph resolves that slot: remapping it would make the next replay
            # read unmapped memory or another allocation
            raise RuntimeError("collective: memory a captured HIP graph's collective uses was freed and reallocated; "
                               "drop the graph and call unpin_captured() first")
        evictable = [k for k in self._dyn if k not in self._pinned and k not in keep]
        full = not self._free_slots and len(self._dyn) >= self.reg_slots
        if stale or (full and evictable):
            torch.cuda.synchronize(self.device)  # no queued kernel of this rank still resolves a slot
        for k in stale:
            s = self._dyn.pop(k)
            self.dc.clear_segment(s)
            self._free_slots.append(s)
        if not self._free_slots and len(self._dyn) >= self.reg_slots and evictable:
            self._free_slots.append(self._dyn.pop(evictable[0]))  # least recently used unpinned slot
        # (every slot pinned by captures: a new slot beyond CCMPI_REGISTER_SLOTS)
        slot = self._free_slots.pop() if self._free_slots else -1
        me = key[self.rank]
        handles = [k[0] for k in key]
        keys = [k[0] + struct.pack("<QQQ", k[1], k[2], k[3]) for k in key]
        slot = self.dc.set_segment(slot, me[1], me[2], handles, [0] * self.size, keys)
        self._dyn[key] = slot
        self.registrations += 1

    def pick_allreduce(self, nbytes: int) -> str:
        if self.size == 1:
            return "twoshot"
        key = (self.size, max(0, nbytes.bit_length() - 1))
        if key in self.tuned:
            return self.tuned[key]
        forced = os.environ.get("CCMPI_ALLREDUCE_ALGO")
        if forced:
            return forced
        prefs = []
        if nbytes <= self.ll_auto_max and nbytes % 16 == 0:
            # in-kernel latency (rocprofv3, 2 ranks): 6.0 us vs 10.2 us one-shot at 4 KiB,
            # 7.1 vs 12.8 us at 64 KiB (profiles/r2_coll/ll_latency.md)
            prefs.append("ll")
        if nbytes <= self.oneshot_max:
            prefs.append("oneshot")
        # fanout vs twoshot, 2-8 ranks, 1-256 MiB: 0.8x the time (profiles/r2_coll/fanout.md)
        prefs += ["fanout", "twoshot", "reduce_bcast"]
        for a in prefs:
            if a not in self.disabled:
                return a
        return "rccl"

    # ------------------------------------------------------------- collectives
    @trace_call("allreduce")
    def allreduce(self, src, dst=None, op="SUM", algo: str = "auto", rings: int = 0,
                  max_blocks: Optional[int] = None, symmetric: Optional[bool] = None) -> object:
        """``symmetric=True``: src / dst are symmetric-heap blocks of the same layout on every
        rank (no host call; see ``_symm_call``); default: decided collectively."""
        dst = src if dst is None else dst
        self._check(src, "src")
        self._check(dst, "dst")
        if src.numel() != dst.numel() or src.dtype != dst.dtype:
            raise ValueError("allreduce: src/dst must match in size and dtype")
        opc, dt = op_code(op), dtype_code(src.dtype)
        nbytes = src.numel() * src.element_size()
        if algo == "auto":
            algo = self.pick_allreduce(nbytes)
        if self.deterministic and algo.split(":")[0] in _UNORDERED:
            algo = "fanout"
        if ":" in algo:  # "twoshot:512" = algorithm with an explicit CTA budget
            algo, mb = algo.split(":", 1)
            max_blocks = int(mb)
        s = self._stream()
        if algo in ("push", "ring", "rhd"):
            self._ensure_inbox(nbytes)
        if algo == "ll":
            self._ensure_ll()
        if algo == "ring":
            self.dc.set_rings(rings or self.default_rings)
        if algo in _HAND_ALGOS:
            # one decision on every rank (ring / rhd split the call into launches by it):
            # both tensors go through the collective check, which also covers the alignment
            # of every rank's input (ring / rhd read only the local input, but a rank-local
            # alignment test could make the ranks disagree)
            symm = self._symm_call(nbytes, src, dst, promise=symmetric)
            self.dc.allreduce(src.data_ptr(), dst.data_ptr(), src.numel(), dt, opc, getattr(self.D, _HAND_ALGOS[algo]),
                              s, self._budget(max_blocks), symm)
        elif algo == "rccl":
            self.ensure_rccl()
            self.dc.rccl_allreduce(src.data_ptr(), dst.data_ptr(), src.numel(), dt, opc, s)
        else:
            raise ValueError(f"unknown allreduce algorithm {algo!r}")
        return dst

    @trace_call("allreduce")
    def allreduce_to_local(self, src, dst, op="SUM", max_blocks: Optional[int] = None):
        """``dst = sum over ranks of src`` where ``src`` is a symmetric-heap block (on every
        rank) that the collective CLOBBERS and ``dst`` is any local CUDA tensor (no
        registration, no host call): two-shot whose reduce-scatter lands in the source's
        own shard and whose all-gather pulls every rank's shard into ``dst``
        (``DeviceComm::allreduce_to_local``).  The TP layers' GEMMs write their partial
        products into persistent heap scratch (``persistent``) and reduce them into
        fresh outputs this way: zero-copy, and the output is an ordinary tensor."""
        self._check(src, "src")
        self._check(dst, "dst")
        if src.numel() != dst.numel() or src.dtype != dst.dtype:
            raise ValueError("allreduce_to_local: src/dst must match in size and dtype")
        if self.size > 1 and not self._symm(src):
            raise ValueError("allreduce_to_local: src must be a 16-B aligned symmetric-heap block (comm.empty / "
                             "persistent)")
        self.dc.allreduce_to_local(src.data_ptr(), dst.data_ptr(), src.numel(), dtype_code(src.dtype), op_code(op),
                                   self._stream(), self._budget(max_blocks))
        return dst

    @trace_call("reduce_scatter")
    def reduce_scatter(self, src, dst, op="SUM", algo: str = "direct", max_blocks: Optional[int] = None):
        self._check(src, "src")
        self._check(dst, "dst")
        if src.numel() != dst.numel() * self.size:
            raise ValueError("reduce_scatter: src must hold size * dst elements")
        opc, dt = op_code(op), dtype_code(src.dtype)
        s = self._stream()
        if algo == "rccl":
            self.ensure_rccl()
            self.dc.rccl_reduce_scatter(src.data_ptr(), dst.data_ptr(), dst.numel(), dt, opc, s)
        else:
            self.dc.reduce_scatter(src.data_ptr(), dst.data_ptr(), dst.numel(), dt, opc, s,
                                   self._budget(max_blocks), self._symm_call(src.numel() * src.element_size(), src))
        return dst

    @trace_call("allgather")
    def allgather(self, src, dst, algo: str = "direct", max_blocks: Optional[int] = None):
        """``direct``: every rank pulls every peer's block (input from the
        symmetric heap: zero staging; otherwise staged in chunks); ``push``:
        every rank writes its block into every peer's output (outputs from the
        symmetric heap on every rank; otherwise the pull form); ``auto``: push
        when the output is symmetric, else direct; ``rccl``."""
        self._check(src, "src")
        self._check(dst, "dst")
        if dst.numel() != src.numel() * self.size or src.dtype != dst.dtype:
            raise ValueError("allgather: dst must hold size * src elements of the same dtype")
        s = self._stream()
        nb = src.numel() * src.element_size()
        if algo == "rccl":
            self.ensure_rccl()
            self.dc.rccl_allgather(src.data_ptr(), dst.data_ptr(), nb, 1, s)
        elif algo in ("push", "auto", "direct"):
            # one collective decision for the call (registers both tensors when large)
            symm = self._symm_call(nb * self.size, src, dst)
            if algo in ("push", "auto") and symm and nb % 16 == 0:
                # push: 0.85x the pull form's time at 64-256 MiB (profiles/r2_coll/allgather_push.md)
                self.dc.allgather(src.data_ptr(), dst.data_ptr(), nb, s, self._budget(max_blocks), True, self.D.A2A_PUSH)
            else:
                self.dc.allgather(src.data_ptr(), dst.data_ptr(), nb, s, self._budget(max_blocks),
                                  symm and dst.data_ptr() % 16 == 0, self.D.A2A_PULL)
        else:
            raise ValueError(f"unknown allgather algorithm {algo!r}")
        return dst

    @trace_call("alltoall")
    def alltoall(self, src, dst, algo: str = "direct", max_blocks: Optional[int] = None):
        """``direct``: every rank pulls its block from all peers (inputs from the
        symmetric heap: zero staging; otherwise one pack pass); ``push``: every
        rank writes its segments straight into the peers' outputs (reference
        myAlltoall, comm.py:130-155; outputs from the symmetric heap on every
        rank); ``pairwise``: the reference myAlltoall2 schedule (comm.py:162-199)
        hand-written -- round k pushes the block for rank + k into its output and
        waits for the block from rank - k, one peer in flight per round (outputs
        from the symmetric heap: zero staging; otherwise through the scratch
        segment); ``pairwise_rccl``: the same rounds as RCCL send/recv; ``rccl``."""
        self._check(src, "src")
        self._check(dst, "dst")
        if src.numel() != dst.numel() or src.numel() % self.size:
            raise ValueError("alltoall: src/dst must match and be divisible by the group size")
        s = self._stream()
        blk = src.numel() * src.element_size() // self.size
        if algo == "rccl":
            self.ensure_rccl()
            self.dc.rccl_alltoall(src.data_ptr(), dst.data_ptr(), blk, 1, s)
        elif algo == "pairwise_rccl":
            self.ensure_rccl()
            self.dc.p2p_pairwise_alltoall(src.data_ptr(), dst.data_ptr(), blk, s)
        elif algo in ("pairwise", "push", "direct", "auto"):
            symm = self._symm_call(blk * self.size, src, dst)
            if algo == "pairwise":
                # hand-written pairwise rounds on the flag protocol (myAlltoall2's schedule)
                self.dc.alltoall(src.data_ptr(), dst.data_ptr(), blk, s, self._budget(max_blocks),
                                 symm and src.data_ptr() % 16 == 0, self.D.A2A_PAIRWISE)
            elif algo == "push":
                self.dc.alltoall(src.data_ptr(), dst.data_ptr(), blk, s, self._budget(max_blocks),
                                 symm and src.data_ptr() % 16 == 0, self.D.A2A_PUSH)
            else:
                self.dc.alltoall(src.data_ptr(), dst.data_ptr(), blk, s, self._budget(max_blocks), symm,
                                 self.D.A2A_PULL)
        else:
            raise ValueError(f"unknown alltoall algorithm {algo!r}")
        return dst

    @trace_call("alltoallv")
    def alltoallv(self, src, send_counts, dst, recv_counts=None, max_blocks: Optional[int] = None):
        """Ragged all-to-all (MPI Alltoallv with packed displacements; the MoE token
        dispatch/combine shape): ``src`` holds ``send_counts[j]`` elements for rank j
        back to back in rank order; ``dst`` receives ``recv_counts[i]`` elements from
        rank i back to back in rank order.  One host all-gather of every rank's count
        row (p integers) gives each rank the whole count matrix, so every offset is
        known locally.  When every segment is a 16-B multiple and every rank's
        output lives in the symmetric heap, one push kernel writes each segment
        straight into its destination (``k_alltoallv_push``); otherwise the call
        runs as a padded all-to-all (blocks of the largest count) plus pack/unpack
        copies.  With ``send_counts`` a CUDA tensor the counts never leave the device
        (``_alltoallv_dev``; ``recv_counts`` is then an output tensor).  Returns ``dst``."""
        torch = self.torch
        self._check(src, "src")
        self._check(dst, "dst")
        if src.dtype != dst.dtype:
            raise ValueError("alltoallv: src/dst dtypes differ")
        p, me = self.size, self.rank
        if isinstance(send_counts, torch.Tensor) and send_counts.is_cuda:
            return self._alltoallv_dev(src, send_counts, dst, recv_counts, max_blocks)
        sc = [int(c) for c in send_counts]
        if len(sc) != p or min(sc) < 0:
            raise ValueError("alltoallv: need one non-negative send count per rank")
        if sum(sc) > src.numel():
            raise ValueError("alltoallv: send counts exceed src")
        es = src.element_size()
        # one host all-gather carries every rank's count row plus whether its buffers
        # allow the kernel path (16-B aligned input, output in the symmetric heap): a
        # local property every rank must agree on before choosing a path
        ok_local = src.data_ptr() % 16 == 0 and (dst.numel() == 0 or (dst.data_ptr() % 16 == 0 and self.is_symmetric(dst)))
        # row: [send counts (p) | kernel path ok | expected recv counts (p, -1 = unchecked) | dst capacity].
        # Every rank validates every rank's expectations against the gathered matrix, so a
        # bad call raises on ALL ranks before any kernel is launched (no lone waiter).
        given = [-1] * p if recv_counts is None else [int(c) for c in recv_counts]
        if len(given) != p:
            raise ValueError("alltoallv: need one recv count per rank")
        mat = np.zeros((p, 2 * p + 2), np.int64)
        self.host.Allgather(np.array(sc + [int(ok_local)] + given + [dst.numel()], np.int64), mat)
        counts = mat[:, :p]  # counts[i, j]: elements rank i sends to rank j
        for i in range(p):
            want_i = counts[:, i]
            if mat[i, p + 1] >= 0 and not np.array_equal(mat[i, p + 1:2 * p + 1], want_i):
                raise ValueError(f"alltoallv: rank {i} expects recv_counts {mat[i, p + 1:2 * p + 1].tolist()} "
                                 f"but the peers send {want_i.tolist()}")
            if int(want_i.sum()) > int(mat[i, 2 * p + 1]):
                raise ValueError(f"alltoallv: rank {i}'s dst ({int(mat[i, 2 * p + 1])} elements) is too small for "
                                 f"the {int(want_i.sum())} it receives")
        rc = counts[:, me].tolist()
        rtot_local = sum(rc)
        fast = bool(mat[:, p].all()) and not np.any((counts * es) % 16)
        s = self._stream()
        if fast:
            soff, doff, lens, grid_bytes = alltoallv_plan(counts, me, es)
            out = dst if rtot_local else self.scratch
            self.dc.alltoallv(src.data_ptr(), out.data_ptr(), max(16, rtot_local * es), soff, doff, lens, grid_bytes, s,
                              self._budget(max_blocks))
            return dst
        # padded fallback: blocks of the largest count through the regular all-to-all
        m = int(counts.max())
        if m == 0:
            return dst
        ps = torch.zeros(p * m, dtype=src.dtype, device=self.device)
        pr = torch.empty(p * m, dtype=src.dtype, device=self.device)
        o = 0
        for j in range(p):
            ps[j * m:j * m + sc[j]].copy_(src[o:o + sc[j]])
            o += sc[j]
        self.alltoall(ps, pr, "direct", max_blocks)
        o = 0
        for i in range(p):
            dst[o:o + rc[i]].copy_(pr[i * m:i * m + rc[i]])
            o += rc[i]
        return dst

    def _alltoallv_dev(self, src, send_counts, dst, recv_counts, max_blocks):
        """alltoallv with the counts in device memory (e.g. an MoE router's per-expert
        token counts): no host round trip, capturable in a HIP graph.  The kernel
        exchanges the count rows itself (``k_alltoallv_dev``); ``recv_counts`` (a
        CUDA int64 tensor of p elements, allocated if None) receives the counts that
        arrived.  ``dst`` must be in the symmetric heap on every rank and every segment
        a 16-B multiple; a violating or overflowing segment is not written and
        ``check()`` raises (fault code 0x900 + peer)."""
        torch = self.torch
        p = self.size
        if send_counts.numel() != p:
            raise ValueError("alltoallv: need one send count per rank")
        if not (self.is_symmetric(dst) and dst.data_ptr() % 16 == 0 and src.data_ptr() % 16 == 0):
            raise ValueError("alltoallv with device counts: dst must come from the symmetric heap (comm.empty), "
                             "src and dst 16-B aligned")
        counts = send_counts.to(torch.int64).contiguous()
        if recv_counts is None:
            recv_counts = torch.empty(p, dtype=torch.int64, device=self.device)
        elif not (recv_counts.is_cuda and recv_counts.dtype == torch.int64 and recv_counts.numel() == p
                  and recv_counts.is_contiguous()):
            raise ValueError("alltoallv: recv_counts must be a contiguous CUDA int64 tensor of p elements")
        s = self._stream()
        self.dc.alltoallv_dev(src.data_ptr(), counts.data_ptr(), dst.data_ptr(), dst.numel(), recv_counts.data_ptr(),
                              src.element_size(), s, self._budget(max_blocks))
        return dst

    @trace_call("bcast")
    def bcast(self, buf, root: int = 0, algo: str = "auto"):
        """``direct`` (= ``auto``): every rank pulls the root's buffer; ``push``:
        the root loads each vector once and writes it into every peer's buffer
        (symmetric buffers on every rank, else the pull form) -- only the root's
        CTAs work there, which measured slower than the pull form at 4 / 8 ranks
        (profiles/r2_coll/bcast_push.md); ``rccl``."""
        self._check(buf, "buf")
        s = self._stream()
        nb = buf.numel() * buf.element_size()
        if algo == "rccl":
            self.ensure_rccl()
            self.dc.rccl_bcast(buf.data_ptr(), nb, 1, root, s)
        elif algo in ("direct", "auto", "push"):
            symm = self._symm_call(nb, buf)
            mode = self.D.A2A_PUSH if (algo == "push" and symm) else self.D.A2A_PULL
            self.dc.bcast(buf.data_ptr(), nb, root, s, self._budget(None), symm, mode)
        else:
            raise ValueError(f"unknown bcast algorithm {algo!r}")
        return buf

    def allgather_lastaxis(self, src, dst, rows: int, row_bytes: int):
        """dst[m][j*k:(j+1)*k] = src_j[m]  (TP forward collect, fused layout)."""
        self.dc.allgather_lastaxis(src.data_ptr(), dst.data_ptr(), rows, row_bytes, self._stream(), self._budget(None),
                                   self._symm_call(rows * row_bytes, src))
        return dst

    def reduce_scatter_lastaxis(self, src, dst, rows: int, k: int, op="SUM"):
        """dst[m] = sum_j src_j[m][me*k:(me+1)*k]  (TP backward grad_x, fused layout)."""
        self.dc.reduce_scatter_lastaxis(src.data_ptr(), dst.data_ptr(), rows, k, dtype_code(src.dtype), op_code(op),
                                        self._stream(), self._budget(None),
                                        self._symm_call(rows * k * self.size * src.element_size(), src))
        return dst

    def local_reduce(self, inputs: Sequence, out, op="SUM"):
        self.dc.local_reduce([t.data_ptr() for t in inputs], out.data_ptr(), out.numel(), dtype_code(out.dtype),
                             op_code(op), self._stream())
        return out

    # ------------------------------------------------------------------- tuning
    def tune(self, max_bytes: int = 256 << 20, min_bytes: int = 4 << 10, algos: Sequence[str] = (),
             iters: int = 5, dtype=None, save: Optional[str] = None, apply: bool = True) -> Dict[Tuple[int, int], str]:
        """Collective: time every all-reduce algorithm at powers of 4 between
        ``min_bytes`` and ``max_bytes`` (after an exactness check) and make
        ``algo="auto"`` use the fastest per size class.  Algorithms that fail or
        time out on any rank are discarded everywhere.  The table is written by
        rank 0 to ``save`` (default ``CCMPI_TUNE_FILE``), from which later
        groups of the same size / sharing / GPU model load it at start-up.
        Every measured time is kept in ``tune_times[(dtype name, bytes)][algo]``
        (seconds per call, None = failed): the algbw-vs-size curve.  ``apply=False``
        only measures (e.g. a bf16 curve beside the fp32 table)."""
        import time

        torch = self.torch
        dtype = dtype or torch.float32
        if not algos:
            algos = ["ll", "oneshot", "twoshot", "fanout"] + ([] if self.shared_device else ["rccl"])
        times = self.__dict__.setdefault("tune_times", {})
        dname = str(dtype).replace("torch.", "")
        es = torch.empty((), dtype=dtype).element_size()
        x = self.empty(max_bytes // es, dtype)
        y = self.empty(max_bytes // es, dtype)
        x.fill_(float(self.rank + 1))
        expect = float(self.size * (self.size + 1) // 2)
        b = min_bytes
        while b <= max_bytes:
            n = b // es
            best, best_t = None, None
            row = times.setdefault((dname, b), {})
            for algo in algos:
                if algo == "oneshot" and b > (16 << 20):
                    continue
                if algo == "ll" and (b > self.ll_max or b % 16):
                    continue
                ok = 1
                try:
                    self.allreduce(x[:n], y[:n], "SUM", algo, symmetric=True)
                    torch.cuda.synchronize(self.device)
                    self.check()
                    ok = int(bool(torch.all(y[:n] == expect).item()))
                except Exception:  # noqa: BLE001 - disqualify the algorithm
                    ok = 0
                if not self.host.allreduce(ok, op=_host_min()):
                    row[algo] = None
                    self.reset()  # a timed-out kernel leaves the per-CTA epochs inconsistent
                    continue
                torch.cuda.synchronize(self.device)
                self.host.Barrier()
                t0 = time.perf_counter()
                for _ in range(iters):
                    self.allreduce(x[:n], y[:n], "SUM", algo, symmetric=True)
                torch.cuda.synchronize(self.device)
                t = self.host.allreduce(time.perf_counter() - t0, op=_host_max()) / iters
                row[algo] = t
                if best_t is None or t < best_t:
                    best, best_t = algo, t
            if best is not None and apply:
                self.tuned[(self.size, max(0, b.bit_length() - 1))] = best
                self.tuned[(self.size, max(0, b.bit_length() - 1) + 1)] = best
            b *= 4
        path = save or self.tune_file
        if path and self.rank == 0 and apply:
            save_tuning(path, self.tune_key, self.tuned)
        self.host.Barrier()
        return dict(self.tuned)

    def sweep_curve(self, dtype_name: str = "float32") -> List[dict]:
        """The algbw/busbw-vs-size curve of the ``tune`` runs of one dtype: per size, every
        algorithm's time, the fastest, and its algorithm / bus bandwidth (NCCL-tests
        conventions: busbw = algbw x 2(p-1)/p)."""
        out = []
        f = 2 * (self.size - 1) / self.size if self.size > 1 else 0.0
        for (dn, b), row in sorted(getattr(self, "tune_times", {}).items(), key=lambda kv: kv[0][1]):
            if dn != dtype_name:
                continue
            good = {a: t for a, t in row.items() if t}
            best = min(good, key=good.get) if good else None
            alg = b / good[best] / 1e9 if best else None
            out.append({"bytes": b, "best": best, "ms": {a: (round(t * 1e3, 4) if t else None) for a, t in row.items()},
                        "algbw_GBps": round(alg, 2) if alg else None,
                        "busbw_GBps": round(alg * f, 2) if alg else None})
        return out

    # ------------------------------------------------------------- async issue
    def start(self, op: str, *args, stream=None, **kw) -> "Work":
        """Non-blocking collective: ``op`` ("allreduce", "allgather", "alltoall",
        "reduce_scatter", "bcast") runs on ``stream`` (default: this group's
        communication stream, normal priority) after the work queued so far on
        the current stream; returns a ``Work`` whose ``wait()`` makes the current
        stream wait for it.  The tensors stay referenced by the ``Work`` until it
        is waited on, so their blocks cannot be reused under the collective (the
        device-side analogue of the reference's Isend/Irecv + Waitall,
        mpi_wrapper/comm.py:136-150).  Every rank must start the same
        collectives in the same order on the same stream kind.

        With more than 2 ranks sharing one GPU (this repo's test setup) the
        default is the current stream: one extra stream in each of 8 processes
        oversubscribes the GPU's hardware queues, the scheduler then time-slices
        them and every later cross-process barrier waits for a queue switch
        (measured: all collectives ~10x slower for the rest of the run)."""
        torch = self.torch
        fn = getattr(self, op)
        if stream is None:
            if self.shared_device and self.ranks_per_device > 2:
                stream = torch.cuda.current_stream(self.device)
            else:
                if getattr(self, "_comm_stream", None) is None:
                    self._comm_stream = torch.cuda.Stream(device=self.device)
                stream = self._comm_stream
        ready = torch.cuda.Event()
        ready.record(torch.cuda.current_stream(self.device))
        stream.wait_event(ready)
        if stream != torch.cuda.current_stream(self.device):
            # a caller that drops the Work unwaited must not see the caching allocator
            # hand these blocks out while the collective still reads/writes them
            # (no-op for symmetric-heap tensors, which are not allocator blocks)
            for t in args:
                if isinstance(t, torch.Tensor) and t.is_cuda:
                    t.record_stream(stream)
        with torch.cuda.stream(stream):
            if op in ("allreduce", "allreduce_to_local", "allgather", "alltoall", "reduce_scatter"):
                kw.setdefault("max_blocks", self.overlap_blocks)  # runs beside compute
            out = fn(*args, **kw)
            done = torch.cuda.Event()
            done.record(stream)
        self._async_done = (stream.cuda_stream, done)
        # keep the tensors (symmetric-heap blocks are not caching-allocator blocks, so
        # record_stream does not protect them) until the collective has completed, even
        # if the caller drops the Work unwaited -- the host plane does the same (Comm._nb)
        self._inflight = [(e, k) for e, k in self._inflight if not e.query()]
        self._inflight.append((done, args))
        return Work(self, done, out, args)

    # ------------------------------------------------------------------ health
    def self_test(self, sizes: Sequence[int] = (4096, 1 << 20),
                  algos: Sequence[str] = ("ll", "oneshot", "fanout", "twoshot")) -> Dict[str, bool]:
        """Collective: run each algorithm ``auto`` can pick once per size on
        rank-valued fp32 data and check the exact result.  An algorithm that
        fails or times out on any rank is reset away and added to ``disabled``
        on every rank, so ``auto`` falls through to the next one (ll -> oneshot
        -> fanout -> twoshot -> reduce_bcast -> rccl).  Run once after bring-up on
        a new fabric; returns {algo: passed}."""
        torch = self.torch
        if self.size == 1:
            return {a: True for a in algos}
        n = max(sizes) // 4
        x = self.empty(n, torch.float32)
        y = self.empty(n, torch.float32)
        x.fill_(float(self.rank + 1))
        expect = float(self.size * (self.size + 1) // 2)
        out = {}
        for algo in algos:
            ok = 1
            try:
                for b in sizes:
                    m = b // 4
                    y[:m].zero_()
                    self.allreduce(x[:m], y[:m], "SUM", algo)
                    torch.cuda.synchronize(self.device)
                    self.check()
                    ok &= int(bool(torch.all(y[:m] == expect).item()))
            except Exception:  # noqa: BLE001 - any failure disables the algorithm
                ok = 0
            passed = bool(self.host.allreduce(ok, op=_host_min()))
            if not passed:
                self.reset()
                self.disabled.add(algo)
            out[algo] = passed
        del x, y
        return out

    def check(self) -> None:
        """Synchronise and raise if any device collective timed out."""
        code = self.dc.error_code()
        if code:
            self.dc.clear_error()
            raise RuntimeError(f"device collective timeout/fault code 0x{code:x} on rank {self.rank} "
                               f"(phase {code >> 8}, peer {code & 0xff})")

    def reset(self) -> None:
        """Collective recovery after a device timeout: once no kernel is in
        flight anywhere, every rank zeroes its flags and epochs."""
        self.torch.cuda.synchronize(self.device)
        self.host.Barrier()
        self.dc.reset_state()
        self.dc.clear_error()
        self.host.Barrier()

    def barrier(self) -> None:
        self.torch.cuda.synchronize(self.device)
        self.host.Barrier()


def _cu_count(device) -> int:
    try:
        import torch

        return int(torch.cuda.get_device_properties(device).multi_processor_count) or 256
    except Exception:
        return 256


def _gcd(a: int, b: int) -> int:
    while b:
        a, b = b, a % b
    return a


def _host_min():
    from . import mpi as MPI

    return MPI.MIN


def _host_max():
    from . import mpi as MPI

    return MPI.MAX
