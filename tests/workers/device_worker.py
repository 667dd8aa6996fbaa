"""Multi-rank device-plane check (launched by scripts/mpirun; several ranks may
share one GPU).  Every device collective is compared with an fp64/int64
oracle built from all ranks' inputs: inputs come from per-(rank, case) seeded
device generators, so each rank regenerates every peer's input locally.

usage: device_worker.py [--matrix quick|full|wide] [--big] [--rccl] [--stress N] [--fault]

--matrix    quick: fp32/bf16, SUM, 4 sizes; full: 6 dtypes x SUM/PROD/MIN/MAX x
            8 sizes; wide: 6 dtypes x 4 ops x 4 sizes (for 8 ranks).  Every
            hand-written all-reduce algorithm (oneshot, twoshot, fanout, push,
            reduce_bcast, ring, rhd), symmetric and staged, out-of-place and
            in-place, plus reduce-scatter / all-gather / all-to-all (pull, push,
            staged, in-place) / bcast / last-axis TP collects.
--big       >= 96 MiB cases that cross the staging-chunk loop (64 MiB scratch ->
            32 MiB chunks) and the ring/rhd inbox pieces.
--rccl      RCCL collectives and the RCCL-P2P ring/rhd/pairwise schedules; fails
            loudly (RCCL refuses several ranks on one GPU: see
            benchmarks/rccl_shared_probe.py and profiles/r2_coll/rccl_shared_gpu.json).
--stress N  SURVEY §5.2: N back-to-back collectives (mixed algorithms, sizes up to
            16 MiB, symmetric and staged calls) with randomised per-rank host
            sleeps and device-side spin delays, so ranks arrive at each kernel
            in random order; every result is checked at the end (epoch/ABA safety).
--register  on-demand registration of ordinary (caching-allocator) tensors >= 1 MiB:
            every collective in place on them (no staging), reuse of mapped slots,
            and a freed-and-reallocated allocation picked up afresh.
--fault     SURVEY §5.3: rank p-1 skips one collective; the others must time out
            (bounded spins), the host watchdog must see the code without a device
            sync, check() must raise, and reset() must restore a working group.
"""
import argparse
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
from collective_communication_mpi_amd import MPI, Communicator  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--matrix", default="", choices=["", "quick", "full", "wide"])
ap.add_argument("--quick", action="store_true", help="alias of --matrix quick")
ap.add_argument("--big", action="store_true")
ap.add_argument("--rccl", action="store_true")
ap.add_argument("--sizes", default="")
ap.add_argument("--stress", type=int, default=0)
ap.add_argument("--fault", action="store_true")
ap.add_argument("--register", action="store_true")
args = ap.parse_args()
if args.quick:
    args.matrix = "quick"

comm = Communicator(MPI.COMM_WORLD)
rank, p = comm.Get_rank(), comm.Get_size()
dev = comm.dev
D = dev.device
torch.cuda.synchronize()
fails = []
ncheck = 0
POW2 = p & (p - 1) == 0
AR_ALGOS = ["oneshot", "twoshot", "fanout", "fanout_lds", "push", "reduce_bcast", "ring", "ll"] + (["rhd"] if POW2 else [])
WIDE = lambda dt: torch.float64 if dt.is_floating_point else torch.int64  # noqa: E731


def gen(r, n, dtype, salt, op="SUM"):
    """Rank r's input of case `salt` (identical on every rank that asks)."""
    g = torch.Generator(device=D).manual_seed(1_000_003 * salt + 7919 * r + 17)
    if dtype.is_floating_point:
        if op == "PROD":  # keep p-fold products in range
            x = torch.rand(n, generator=g, device=D, dtype=torch.float64) + 0.5
        else:
            x = torch.randn(n, generator=g, device=D, dtype=torch.float64) * 3
        return x.to(dtype)
    if op == "PROD":
        x = torch.randint(1, 3, (n,), generator=g, device=D, dtype=torch.int64)
        x = torch.where(torch.rand(n, generator=g, device=D) < 0.5, -x, x)
        return x.to(dtype)
    return torch.randint(-1000, 1000, (n,), generator=g, device=D, dtype=torch.int64).to(dtype)


def oracle(n, dtype, op, salt):
    acc = None
    for r in range(p):  # rank order, in fp64 / int64
        x = gen(r, n, dtype, salt, op).to(WIDE(dtype))
        if acc is None:
            acc = x
        elif op == "SUM":
            acc = acc + x
        elif op == "MAX":
            acc = torch.maximum(acc, x)
        elif op == "MIN":
            acc = torch.minimum(acc, x)
        else:
            acc = acc * x
    return acc


def check(name, got, want, dtype, nterms=1):
    global ncheck
    ncheck += 1
    got = got.detach().reshape(-1).to(WIDE(dtype))
    want = want.reshape(-1)
    if got.shape != want.shape:
        fails.append(f"{name}: shape {tuple(got.shape)} vs {tuple(want.shape)}")
        return False
    if dtype.is_floating_point:
        tol = {torch.float32: 1e-5, torch.float64: 1e-12, torch.bfloat16: 1e-2, torch.float16: 2e-3}[dtype] * nterms
        ok = torch.allclose(got, want, rtol=tol, atol=tol * 4)
    else:
        ok = torch.equal(got, want)
    if not ok:
        diff = (got - want).abs().max().item()
        fails.append(f"{name}: max diff {diff}")
    return ok


def stress(iters):
    """Random arrival order at every collective; results checked after the burst.
    Mixes symmetric (zero-copy) and staged calls, up to 16 MiB, all-reduces of every
    algorithm with push / pull all-gathers and all-to-alls."""
    import random

    rng = random.Random(1234 + rank)  # per-rank: delays only
    shared = random.Random(99)        # identical on every rank: sizes, algorithms, symmetric or not
    pending = []
    algos_s = AR_ALGOS
    big = 4 << 20  # elements: 16 MiB fp32
    sym_x = dev.empty(big, torch.float32)
    sym_y = dev.empty(big, torch.float32)
    for i in range(iters):
        n = shared.choice([1, 33, 4096, 1 << 16, 1 << 20, big])
        algo = shared.choice(algos_s)
        sym = shared.random() < 0.5
        d = rng.random()
        if d < 0.3:
            time.sleep(rng.random() * 0.004)
        elif d < 0.6:
            torch.cuda._sleep(rng.randint(1000, 200000))  # device-side skew
        kind = shared.random()
        if kind < 0.15:  # all-gather of n // p elements per rank, push or pull
            m = max(1, n // p)
            ag = shared.choice(["direct", "push"])
            x = gen(rank, m, torch.float32, 50000 + i)
            if sym:
                sym_x[:m].copy_(x)
                x, y = sym_x[:m], sym_y[:m * p]
            else:
                y = torch.empty(m * p, dtype=torch.float32, device=D)
            dev.allgather(x, y, ag)
            want = torch.cat([gen(r, m, torch.float32, 50000 + i) for r in range(p)]).double()
            pending.append((f"stress[{i},allgather-{ag},m={m},sym={sym}]", y.clone(), want, 1))
            continue
        if kind < 0.3:  # all-to-all of n // p elements per peer block, push or pull
            m = max(1, n // p)
            aa = shared.choice(["direct", "push", "pairwise"])
            x = gen(rank, m * p, torch.float32, 50000 + i)
            if sym:
                sym_x[:m * p].copy_(x)
                x, y = sym_x[:m * p], sym_y[:m * p]
            else:
                y = torch.empty(m * p, dtype=torch.float32, device=D)
            dev.alltoall(x, y, aa)
            want = torch.cat([gen(r, m * p, torch.float32, 50000 + i)[rank * m:(rank + 1) * m] for r in range(p)]).double()
            pending.append((f"stress[{i},alltoall-{aa},m={m},sym={sym}]", y.clone(), want, 1))
            continue
        x = gen(rank, n, torch.float32, 50000 + i)
        if sym:
            sym_x[:n].copy_(x)
            x, y = sym_x[:n], sym_y[:n]
        else:
            y = torch.empty(n, dtype=torch.float32, device=D)
        dev.allreduce(x, y, "SUM", algo)
        pending.append((f"stress[{i},{algo},n={n},sym={sym}]", y.clone(), (n, 50000 + i), p))
    torch.cuda.synchronize()
    dev.check()
    for name, y, want, nt in pending:
        if isinstance(want, tuple):
            want = oracle(want[0], torch.float32, "SUM", want[1])
        check(name, y, want, torch.float32, nt)


def fault():
    """One rank misses a collective; the rest time out, report, and recover."""
    dev.dc.set_timeout_seconds(0.5)
    x = dev.empty(4096, torch.float32)
    x.fill_(1.0)
    y = dev.empty(4096, torch.float32)
    torch.cuda.synchronize()
    comm.comm.Barrier()
    if rank != p - 1:
        dev.allreduce(x, y, "SUM", "twoshot")
        t0 = time.time()
        while not dev.dc.poll_error() and time.time() - t0 < 10:
            time.sleep(0.05)  # the watchdog word is host-mapped: no device sync here
        if not dev.dc.poll_error():
            fails.append("fault: host-mapped watchdog word never set")
        try:
            dev.check()
            fails.append("fault: check() did not raise after a timeout")
        except RuntimeError as e:
            if f"rank {rank}" not in str(e):
                fails.append(f"fault: message not rank-tagged: {e}")
    dev.reset()
    dev.dc.set_timeout_seconds(20.0)
    for algo in ("twoshot", "ring"):
        dev.allreduce(x, y, "SUM", algo)
        check(f"fault_recovery_allreduce[{algo}]", y, torch.full((4096,), float(p), dtype=torch.float64, device=D),
              torch.float32)


def finish(t0):
    comm.Barrier()
    print(f"[rank {rank}/{p}] device checks: {ncheck} checks, {len(fails)} failures, {time.time() - t0:.1f}s", flush=True)
    for f in fails[:20]:
        print(f"[rank {rank}] FAIL {f}", flush=True)
    sys.exit(1 if fails else 0)


t0 = time.time()
if args.stress or args.fault:
    if args.stress:
        stress(args.stress)
    if args.fault:
        fault()
    finish(t0)

ALL_DT = [torch.float32, torch.bfloat16, torch.float16, torch.float64, torch.int32, torch.int64]
ALL_OPS = ["SUM", "PROD", "MIN", "MAX"]
if args.matrix == "quick":
    sizes, dtypes, ops = [1, 7, 1000, 65536 + 3, 1 << 17], [torch.float32, torch.bfloat16], ["SUM"]
elif args.matrix == "wide":
    sizes, dtypes, ops = [1, 1000, 65536 + 3, (1 << 20) + 3], ALL_DT, ALL_OPS
elif args.matrix == "full":
    sizes, dtypes, ops = [1, 3, 8, 1000, 4097, 65536 + 3, 1 << 17, 1 << 20, (1 << 22) + 5], ALL_DT, ALL_OPS
else:
    sizes, dtypes, ops = [], [], []
if args.sizes:
    sizes = [int(x) for x in args.sizes.split(",") if x]
salt = 0


def sym_copy(t):
    s_ = dev.empty(t.numel(), t.dtype)
    s_.copy_(t)
    return s_


def determinism():
    """Rank-ordered algorithms (oneshot, twoshot, fanout, push, reduce_bcast, ll) give results
    that are bitwise identical to each other and to a sequential fp32 sum in rank order
    (bf16: fp32 accumulation, one rounding) -- the reference's root loop order
    (comm.py:85-93).  Checked in-place too, and through CCMPI_DETERMINISTIC's mapping."""
    ordered = ["oneshot", "twoshot", "fanout", "fanout_lds", "push", "reduce_bcast", "ll"]
    for dt in (torch.float32, torch.bfloat16):
        for n in (1000, 4096, 65536):
            xs = [gen(r, n, dt, 777000 + n) for r in range(p)]
            acc = xs[0].float().cpu()
            for x in xs[1:]:
                acc = acc + x.float().cpu()  # sequential fp32 adds, rank order
            want = acc.to(dt)
            sym_x = dev.empty(n, dt)
            for algo in ordered:
                sym_x.copy_(xs[rank])
                y = dev.empty(n, dt)
                dev.allreduce(sym_x, y, "SUM", algo)
                if not torch.equal(y.cpu(), want):
                    fails.append(f"determinism[{algo},{dt},n={n}]: not bitwise equal to the rank-order fp32 sum")
                global ncheck
                ncheck += 1
    old = dev.deterministic
    dev.deterministic = True
    try:
        x = gen(rank, 4096, torch.float32, 778001)
        y = torch.empty_like(x)
        dev.allreduce(x, y, "SUM", "ring")  # mapped to the rank-ordered fan-out two-shot
        acc = gen(0, 4096, torch.float32, 778001).cpu()
        for r in range(1, p):
            acc = acc + gen(r, 4096, torch.float32, 778001).cpu()
        if not torch.equal(y.cpu(), acc):
            fails.append("deterministic mode: ring not mapped to a rank-ordered algorithm")
    finally:
        dev.deterministic = old


def graphs():
    """Collectives captured once in a HIP graph and replayed with new data: the
    protocol state (per-CTA epochs, the LL call epoch) lives in device memory, so
    replays stay in step with the peers' replays.  Staged (unregistered) buffers
    too: their copies through the scratch segment are captured as well."""
    global ncheck
    n = 4096 + 8
    cases = [("allreduce", a) for a in ("ll", "oneshot", "twoshot", "fanout", "push", "ring")] + \
        [("allgather", "push"), ("allgather", "direct"), ("alltoall", "direct")]
    for sym in (True, False):
        for op, algo in cases:
            mk = (lambda m: dev.empty(m, torch.float32)) if sym else (lambda m: torch.empty(m, dtype=torch.float32, device=D))
            if op == "allreduce":
                x, y = mk(n), mk(n)
                run = lambda: dev.allreduce(x, y, "SUM", algo)
            elif op == "allgather":
                x, y = mk(n), mk(n * p)
                run = lambda: dev.allgather(x, y, algo)
            else:
                x, y = mk(n * p), mk(n * p)
                run = lambda: dev.alltoall(x, y, algo)
            x.fill_(1.0)
            run()  # eager first: lazy allocations (inbox, LL buffers) happen outside the capture
            torch.cuda.synchronize()
            comm.comm.Barrier()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                run()
            for it in range(3):
                if op == "allreduce":
                    x.fill_(float(rank + 1 + it))
                    want = torch.full((n,), float(p * (p + 1) // 2 + p * it), dtype=torch.float64, device=D)
                elif op == "allgather":
                    x.fill_(float(rank + 10 * it))
                    want = (torch.arange(p, device=D, dtype=torch.float64) + 10 * it).repeat_interleave(n)
                else:
                    x.view(p, n).copy_((rank * p + torch.arange(p, device=D, dtype=torch.float32) + 100 * it).view(p, 1).expand(p, n))
                    want = (torch.arange(p, device=D, dtype=torch.float64) * p + rank + 100 * it).repeat_interleave(n)
                g.replay()
                torch.cuda.synchronize()
                dev.check()
                check(f"graph_replay[{op},{algo},sym={sym},it={it}]", y, want, torch.float32)
            del g


def async_ops():
    """DeviceGroup.start(): collectives on the communication stream overlapped with
    compute on the current stream; Work.wait() orders the consumer after them."""
    global ncheck
    n = 1 << 16
    a = torch.randn(512, 512, device=D)
    works, wants = [], []
    for i, (op, algo) in enumerate([("allreduce", "fanout"), ("allreduce", "auto"), ("allgather", "push"),
                                    ("alltoall", "direct")]):
        sl = 93000 + i
        if op == "allreduce":
            x, y = gen(rank, n, torch.float32, sl), dev.empty(n, torch.float32)
            works.append(dev.start(op, x, y, "SUM", algo))
            wants.append(oracle(n, torch.float32, "SUM", sl))
        elif op == "allgather":
            x, y = gen(rank, n, torch.float32, sl), dev.empty(n * p, torch.float32)
            works.append(dev.start(op, x, y, algo))
            wants.append(torch.cat([gen(r, n, torch.float32, sl) for r in range(p)]).double())
        else:
            x, y = gen(rank, n * p, torch.float32, sl), torch.empty(n * p, dtype=torch.float32, device=D)
            works.append(dev.start(op, x, y, algo))
            wants.append(torch.cat([gen(r, n * p, torch.float32, sl)[rank * n:(rank + 1) * n] for r in range(p)]).double())
        del x  # the Work keeps the input alive
        a = a @ a * 1e-3  # compute on the current stream meanwhile
    for i, (w, want) in enumerate(zip(works, wants)):
        out = w.wait()
        check(f"async[{i}]", out, want, torch.float32, p)
    w = dev.start("allreduce", gen(rank, 1000, torch.float32, 93100), torch.empty(1000, device=D))
    check("async_sync", w.synchronize(), oracle(1000, torch.float32, "SUM", 93100), torch.float32, p)
    ncheck += 1
    if not w.is_completed():
        fails.append("async: is_completed() false after synchronize()")
    # a blocking collective issued on the current stream before the started one was
    # waited on: the group orders it after the started one (shared epochs/flags/scratch);
    # both staged (non-heap) so they would also share the scratch segment
    big = 1 << 20
    xs, ys = gen(rank, big, torch.float32, 93300), torch.empty(big, device=D)
    xb, yb = gen(rank, big, torch.float32, 93301), torch.empty(big, device=D)
    w = dev.start("allreduce", xs, ys, "SUM", "twoshot")
    dev.allreduce(xb, yb, "SUM", "twoshot")
    check("async_then_blocking[blocking]", yb, oracle(big, torch.float32, "SUM", 93301), torch.float32, p)
    check("async_then_blocking[started]", w.wait(), oracle(big, torch.float32, "SUM", 93300), torch.float32, p)
    # MPI-style façade: Communicator.I* on CUDA tensors -> DeviceRequest, completed by
    # Request.Waitall together with a host-plane non-blocking collective
    x, y = gen(rank, n, torch.float32, 93200), dev.empty(n, torch.float32)
    xa, ya = gen(rank, n * p, torch.float32, 93201), torch.empty(n * p, device=D)
    hx, hy = np.full(4, rank, np.int64), np.zeros(4, np.int64)
    reqs = [comm.Iallreduce(x, y, MPI.SUM), comm.Ialltoall(xa, ya), comm.comm.Iallreduce(hx, hy, MPI.SUM)]
    MPI.Request.Waitall(reqs)
    check("facade_Iallreduce", y, oracle(n, torch.float32, "SUM", 93200), torch.float32, p)
    check("facade_Ialltoall", ya,
          torch.cat([gen(r, n * p, torch.float32, 93201)[rank * n:(rank + 1) * n] for r in range(p)]).double(),
          torch.float32)
    ncheck += 1
    if not np.array_equal(hy, np.full(4, p * (p - 1) // 2)):
        fails.append("facade: host Iallreduce mixed with device requests")


def ragged():
    """alltoallv: random ragged count matrices (shared RNG), kernel path (16-B segments,
    heap output), padded fallback (odd counts / non-heap output), empty rows/columns,
    and the Communicator façade (accounting as Alltoallv)."""
    import random

    global ncheck
    shared = random.Random(4242)
    for it, (dtype, mult, heap) in enumerate([(torch.float32, 4, True), (torch.bfloat16, 8, True),
                                              (torch.float32, 1, True), (torch.float32, 4, False),
                                              (torch.int64, 2, True)]):
        C = [[shared.randint(0, 40) * mult * shared.choice([0, 1, 1, 3, 100]) for _ in range(p)] for _ in range(p)]
        if it == 0:
            C[0] = [0] * p  # rank 0 sends nothing
            for i in range(p):
                C[i][p - 1] = 0  # rank p-1 receives nothing
        sc = C[rank]
        rcv = [C[i][rank] for i in range(p)]
        x = torch.cat([gen(rank, sc[j], dtype, 94000 + 100 * it + j) for j in range(p)])
        want = torch.cat([gen(i, C[i][rank], dtype, 94000 + 100 * it + rank) for i in range(p)])
        n_out = max(1, sum(rcv))
        y = dev.empty(n_out, dtype) if heap else torch.empty(n_out, dtype=dtype, device=D)
        y.zero_()
        dev.alltoallv(x, sc, y, rcv)
        check(f"alltoallv[{it},{dtype},heap={heap}]", y[:sum(rcv)], want.to(WIDE(dtype)), dtype)
    # device-resident counts: no host exchange; recv counts come back in a device tensor
    for it, (dtype, mult) in enumerate([(torch.float32, 4), (torch.bfloat16, 8), (torch.int64, 2)]):
        C = [[shared.randint(0, 30) * mult for _ in range(p)] for _ in range(p)]
        sc = C[rank]
        x = torch.cat([gen(rank, sc[j], dtype, 94500 + 100 * it + j) for j in range(p)])
        xs = dev.empty(max(1, x.numel()), dtype)
        xs[:x.numel()].copy_(x)
        want = torch.cat([gen(i, C[i][rank], dtype, 94500 + 100 * it + rank) for i in range(p)])
        y = dev.zeros(max(1, want.numel()), dtype)
        rcnt = torch.full((p,), -1, dtype=torch.int64, device=D)
        dev.alltoallv(xs, torch.tensor(sc, device=D), y, rcnt)
        torch.cuda.synchronize()
        dev.check()
        check(f"alltoallv_dev[{dtype}]", y[:want.numel()], want.to(WIDE(dtype)), dtype)
        ncheck += 1
        if rcnt.tolist() != [C[i][rank] for i in range(p)]:
            fails.append(f"alltoallv_dev[{dtype}] recv counts {rcnt.tolist()}")
    # captured once in a HIP graph, replayed with new counts and data in the same buffers
    # (the capture stream is one more HW queue per process: skipped with > 2 ranks per GPU)
    if not serialized and dev.ranks_per_device <= 2:
        cnt = torch.zeros(p, dtype=torch.int64, device=D)
        xs = dev.empty(64 * p, torch.float32)
        y = dev.zeros(64 * p, torch.float32)
        rcnt = torch.zeros(p, dtype=torch.int64, device=D)
        cs = torch.cuda.Stream()
        cs.wait_stream(torch.cuda.current_stream())
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(cs):
            with torch.cuda.graph(g, stream=cs):
                dev.alltoallv(xs, cnt, y, rcnt)
        torch.cuda.current_stream().wait_stream(cs)
        for rep in range(3):
            C = [[shared.randint(0, 16) * 4 for _ in range(p)] for _ in range(p)]
            cnt.copy_(torch.tensor(C[rank], device=D))
            x = torch.cat([gen(rank, C[rank][j], torch.float32, 94800 + 10 * rep + j) for j in range(p)])
            xs[:x.numel()].copy_(x)
            torch.cuda.synchronize()
            dev.host.Barrier()
            g.replay()
            torch.cuda.synchronize()
            dev.check()
            want = torch.cat([gen(i, C[i][rank], torch.float32, 94800 + 10 * rep + rank) for i in range(p)])
            check(f"alltoallv_dev_graph[{rep}]", y[:want.numel()], want.double(), torch.float32)
            ncheck += 1
            if rcnt.tolist() != [C[i][rank] for i in range(p)]:
                fails.append(f"alltoallv_dev_graph[{rep}] recv counts {rcnt.tolist()}")
        del g
    # a segment that is not a 16-B multiple is refused on the device and reported
    y = dev.zeros(64, torch.float32)
    bad = torch.tensor([3] * p, device=D)
    xs = dev.empty(3 * p, torch.float32)
    dev.alltoallv(xs, bad, y, None)
    torch.cuda.synchronize()
    ncheck += 1
    try:
        dev.check()
        fails.append("alltoallv_dev: misaligned segment not reported")
    except RuntimeError as e:
        if "0x90" not in str(e):
            fails.append(f"alltoallv_dev: unexpected error {e}")
    dev.host.Barrier()
    # façade: Communicator.Alltoallv on CUDA tensors
    C = [[(i + 2 * j) % 5 * 4 for j in range(p)] for i in range(p)]
    x = torch.cat([gen(rank, C[rank][j], torch.float32, 94900 + j) for j in range(p)])
    y = dev.empty(max(1, sum(C[i][rank] for i in range(p))), torch.float32)
    before = comm.total_bytes_transferred
    comm.Alltoallv(x, C[rank], y, [C[i][rank] for i in range(p)])
    want = torch.cat([gen(i, C[i][rank], torch.float32, 94900 + rank) for i in range(p)])
    check("facade_Alltoallv", y[:want.numel()], want.double(), torch.float32)
    sent = sum(C[rank][j] for j in range(p) if j != rank) * 4
    got = sum(C[i][rank] for i in range(p) if i != rank) * 4
    ncheck += 1
    if comm.total_bytes_transferred - before != sent + got:
        fails.append(f"Alltoallv accounting {comm.total_bytes_transferred - before} != {sent + got}")


def cuda_aware_mpi():
    """CUDA-aware MPI: the raw MPI communicator's buffer collectives accept CUDA tensors
    (its own device plane, created on the first such call)."""
    global ncheck
    w = MPI.COMM_WORLD
    n = 4096
    x, y = gen(rank, n, torch.float32, 95000), torch.empty(n, device=D)
    w.Allreduce(x, y, op=MPI.SUM)
    check("mpi_cuda_Allreduce", y, oracle(n, torch.float32, "SUM", 95000), torch.float32, p)
    z = gen(rank, n, torch.float32, 95001)
    w.Allreduce(MPI.IN_PLACE, z, op=MPI.MAX)
    check("mpi_cuda_Allreduce_inplace", z, oracle(n, torch.float32, "MAX", 95001), torch.float32)
    g = torch.empty(n * p, device=D)
    w.Allgather(x, g)
    check("mpi_cuda_Allgather", g, torch.cat([gen(r, n, torch.float32, 95000) for r in range(p)]).double(), torch.float32)
    a = gen(rank, n * p, torch.float32, 95002)
    b = torch.empty(n * p, device=D)
    w.Alltoall(a, b)
    check("mpi_cuda_Alltoall", b, torch.cat([gen(r, n * p, torch.float32, 95002)[rank * n:(rank + 1) * n]
                                             for r in range(p)]).double(), torch.float32)
    rs = torch.empty(n, device=D)
    w.Reduce_scatter_block(a, rs, op=MPI.SUM)
    check("mpi_cuda_Reduce_scatter_block", rs, oracle(n * p, torch.float32, "SUM", 95002)[rank * n:(rank + 1) * n],
          torch.float32, p)
    bb = gen(p - 1, n, torch.float32, 95003) if rank == p - 1 else torch.zeros(n, device=D)
    w.Bcast(bb, root=p - 1)
    check("mpi_cuda_Bcast", bb, gen(p - 1, n, torch.float32, 95003).double(), torch.float32)


def tuning():
    """tune() -> per-size table used by auto, persisted through CCMPI_TUNE_FILE-style save."""
    import tempfile

    global ncheck
    path = os.path.join(tempfile.gettempdir(), f"ccmpi_tune_test_{os.getppid()}.json")
    table = dev.tune(max_bytes=1 << 20, min_bytes=4096, iters=2, save=path)
    ncheck += 1
    if not table or any(a not in ("ll", "oneshot", "twoshot", "fanout", "rccl") for a in table.values()):
        fails.append(f"tune: unexpected table {table}")
    from collective_communication_mpi_amd.device import load_tuning
    if rank == 0 and load_tuning(path, dev.tune_key) != table:
        fails.append("tune: saved table differs")
    for n in (1024, 16384, 1 << 18):  # auto now follows the table
        x = gen(rank, n, torch.float32, 91000 + n)
        y = torch.empty_like(x)
        dev.allreduce(x, y, "SUM", "auto")
        check(f"tuned_auto[n={n}]", y, oracle(n, torch.float32, "SUM", 91000 + n), torch.float32, p)
    comm.comm.Barrier()
    if rank == 0:
        os.unlink(path)
    dev.tuned.clear()


_LAP = [time.time()]


def _lap(label):
    if rank == 0 and os.environ.get("CCMPI_WORKER_VERBOSE") == "1":
        print(f"[worker] {label}: {time.time() - _LAP[0]:.2f}s", flush=True)
    _LAP[0] = time.time()


_lap("setup")
if args.matrix:
    # serialized launches (AMD_SERIALIZE_KERNEL, HIP's CUDA_LAUNCH_BLOCKING) synchronise
    # around every kernel, which stream capture forbids: graphs are skipped there
    serialized = os.environ.get("AMD_SERIALIZE_KERNEL", "0") not in ("", "0")
    for fn in (determinism, ragged, cuda_aware_mpi) + (() if serialized else (graphs,)) + ((tuning,) if args.matrix == "quick" else ()):
        t_s = time.time()
        fn()
        if rank == 0 and os.environ.get("CCMPI_WORKER_VERBOSE") == "1":
            print(f"[worker] {fn.__name__}: {time.time() - t_s:.2f}s", flush=True)
    st = dev.self_test()
    ncheck += 1
    if not all(st.values()) or dev.disabled:
        fails.append(f"self_test: {st}, disabled {dev.disabled}")

# ---------------------------------------------------------------- all-reduce
for sym in (False, True):
    for n in sizes:
        for dt in dtypes:
            for op in ops:
                for algo in AR_ALGOS:
                    salt += 1
                    x = gen(rank, n, dt, salt, op)
                    if sym:
                        x, y = sym_copy(x), dev.empty(n, dt)
                    else:
                        y = torch.empty_like(x)
                    dev.allreduce(x, y, op, algo)
                    want = oracle(n, dt, op, salt)
                    check(f"allreduce[{algo},{dt},{op},n={n},sym={sym}]", y, want, dt, p)
                    z = gen(rank, n, dt, salt, op)
                    if sym:
                        z = sym_copy(z)
                    dev.allreduce(z, z, op, algo)
                    check(f"allreduce_inplace[{algo},{dt},{op},n={n},sym={sym}]", z, want, dt, p)
if dtypes:  # misaligned (one-element offset: 4 B fp32, 2 B bf16) input and output
    for mdt in (torch.float32, torch.bfloat16):
        for algo in ("oneshot", "twoshot", "fanout", "fanout_lds", "push", "reduce_bcast", "ring", "ll"):
            salt += 1
            n = 4099
            xb = torch.empty(n + 1, dtype=mdt, device=D)
            yb = torch.empty(n + 1, dtype=mdt, device=D)
            x, y = xb[1:], yb[1:]
            x.copy_(gen(rank, n, mdt, salt))
            dev.allreduce(x, y, "SUM", algo)
            check(f"allreduce_misaligned[{algo},{mdt}]", y, oracle(n, mdt, "SUM", salt), mdt, p)
        salt += 1
        n = 1001
        xb = torch.empty(n + 1, dtype=mdt, device=D)
        yb = torch.empty(p * n + 1, dtype=mdt, device=D)
        x, y = xb[1:], yb[1:]
        x.copy_(gen(rank, n, mdt, salt))
        dev.allgather(x, y)
        check(f"allgather_misaligned[{mdt}]", y, torch.cat([gen(r, n, mdt, salt) for r in range(p)]).to(WIDE(mdt)), mdt)
if dtypes and not POW2:  # recursive halving/doubling refuses non-power-of-two groups on every rank
    try:
        x = torch.ones(64, device=D)
        dev.allreduce(x, x, "SUM", "rhd")
        fails.append("rhd accepted a non-power-of-two group")
    except ValueError:
        pass

_lap("allreduce matrix + misaligned")
# ------------------------------------------- reduce-scatter / gathers / bcast
for sym in (False, True):
    for n in sizes[:6]:
        for dt in dtypes[:3]:
            for op in (ops[:1] + ops[2:3]):  # SUM and MIN
                salt += 1
                x = gen(rank, p * n, dt, salt, op)
                if sym:
                    x = sym_copy(x)
                y = torch.empty(n, dtype=dt, device=D)
                dev.reduce_scatter(x, y, op)
                check(f"reduce_scatter[{dt},{op},n={n},sym={sym}]", y, oracle(p * n, dt, op, salt)[rank * n:(rank + 1) * n],
                      dt, p)
            salt += 1
            x = gen(rank, n, dt, salt)
            if sym:
                x = sym_copy(x)
            y = torch.empty(p * n, dtype=dt, device=D)
            dev.allgather(x, y)
            want = torch.cat([gen(r, n, dt, salt) for r in range(p)]).to(WIDE(dt))
            check(f"allgather[{dt},n={n},sym={sym}]", y, want, dt)
            # push: symmetric output (peer writes), also in place (input = own block of the output)
            y2 = dev.empty(p * n, dt) if sym else torch.empty(p * n, dtype=dt, device=D)
            dev.allgather(gen(rank, n, dt, salt), y2, "push")
            check(f"allgather[push,{dt},n={n},sym_out={sym}]", y2, want, dt)
            if sym:
                y3 = dev.empty(p * n, dt)
                mine = y3[rank * n:(rank + 1) * n]
                mine.copy_(gen(rank, n, dt, salt))
                dev.allgather(mine, y3, "push")
                check(f"allgather_inplace[push,{dt},n={n}]", y3, want, dt)
            # all-to-all: pull (symmetric input or staged), push (symmetric output), in-place (staged)
            salt += 1
            want = torch.cat([gen(r, p * n, dt, salt)[rank * n:(rank + 1) * n] for r in range(p)]).to(WIDE(dt))
            x = gen(rank, p * n, dt, salt)
            if sym:
                x = sym_copy(x)
            y = torch.empty(p * n, dtype=dt, device=D)
            dev.alltoall(x, y)
            check(f"alltoall[direct,{dt},n={n},sym={sym}]", y, want, dt)
            y2 = dev.empty(p * n, dt) if sym else torch.empty(p * n, dtype=dt, device=D)
            dev.alltoall(gen(rank, p * n, dt, salt), y2, "push")
            check(f"alltoall[push,{dt},n={n},sym_out={sym}]", y2, want, dt)
            # pairwise rounds (myAlltoall2): symmetric output (direct pushes) or staged
            y4 = dev.empty(p * n, dt) if sym else torch.empty(p * n, dtype=dt, device=D)
            dev.alltoall(gen(rank, p * n, dt, salt), y4, "pairwise")
            check(f"alltoall[pairwise,{dt},n={n},sym_out={sym}]", y4, want, dt)
            y5 = torch.empty(p * n, dtype=dt, device=D)
            comm.myAlltoall2(gen(rank, p * n, dt, salt), y5)
            check(f"myAlltoall2(device)[{dt},n={n}]", y5, want, dt)
            z2 = gen(rank, p * n, dt, salt)
            if sym:
                z2 = sym_copy(z2)
            dev.alltoall(z2, z2, "pairwise")
            check(f"alltoall_inplace[pairwise,{dt},n={n},sym={sym}]", z2, want, dt)
            z = gen(rank, p * n, dt, salt)
            if sym:
                z = sym_copy(z)
            dev.alltoall(z, z)
            check(f"alltoall_inplace[{dt},n={n},sym={sym}]", z, want, dt)
            # bcast from root p-1: pull (auto) and push (symmetric buffers; else pull)
            for balgo in ("auto", "push"):
                salt += 1
                root = p - 1
                b = gen(rank, n, dt, salt)
                if sym:
                    b = sym_copy(b)
                dev.bcast(b, root, balgo)
                check(f"bcast[{balgo},{dt},n={n},sym={sym}]", b, gen(root, n, dt, salt).to(WIDE(dt)), dt)

_lap("rs/ag/a2a/bcast matrix")
# ------------------------------------- TP layout-fused collectives (func_impl)
if dtypes:
    from collective_communication_mpi_amd.parallel.layout import (  # noqa: E402
        naive_collect_backward_x, naive_collect_forward_input)
    for dt in (torch.float32, torch.bfloat16):
        for (B, S, k) in [(2, 3, 8), (4, 16, 64), (3, 5, 3)]:
            salt += 1
            shards = [gen(r, B * S * k, dt, salt).view(B, S, k) for r in range(p)]
            got = naive_collect_forward_input(shards[rank].clone(), comm, p)
            check(f"forward_input_lastaxis[{dt},{B}x{S}x{k}]", got, torch.cat(shards, dim=-1).to(WIDE(dt)), dt)
            salt += 1
            full = [gen(r, B * S * k * p, dt, salt).view(B, S, k * p) for r in range(p)]
            got = naive_collect_backward_x(full[rank].clone(), comm, p)
            ref = sum(f.to(torch.float64) for f in full)[:, :, rank * k:(rank + 1) * k]
            check(f"backward_x_lastaxis[{dt},{B}x{S}x{k}]", got, ref, dt, p)

_lap("lastaxis")
# ------------------------------------- on-demand registration of torch tensors
if args.register:
    n = (1 << 20) + 4  # 4 MiB + 16 B of fp32 (>= CCMPI_REGISTER_MIN_BYTES)
    reg0 = dev.registrations
    for algo in ("oneshot", "twoshot", "fanout", "push", "ring") + (("rhd",) if POW2 else ()):
        for inplace in (False, True):
            salt += 1
            x = gen(rank, n, torch.float32, salt)  # ordinary torch tensor
            y = x if inplace else torch.empty_like(x)
            dev.allreduce(x, y, "SUM", algo)
            check(f"reg_allreduce[{algo},inplace={inplace}]", y, oracle(n, torch.float32, "SUM", salt),
                  torch.float32, p)
    nb = (1 << 18) + 4
    salt += 1
    x = gen(rank, p * nb, torch.float32, salt)
    want = torch.cat([gen(r, p * nb, torch.float32, salt)[rank * nb:(rank + 1) * nb] for r in range(p)]).double()
    for aa in ("direct", "push", "pairwise"):
        y = torch.empty_like(x)
        dev.alltoall(x, y, aa)
        check(f"reg_alltoall[{aa}]", y, want, torch.float32)
    salt += 1
    x = gen(rank, nb, torch.float32, salt)
    y = torch.empty(p * nb, device=D)
    for ag in ("direct", "push"):
        y.zero_()
        dev.allgather(x, y, ag)
        check(f"reg_allgather[{ag}]", y, torch.cat([gen(r, nb, torch.float32, salt) for r in range(p)]).double(),
              torch.float32)
    salt += 1
    x = gen(rank, p * nb, torch.float32, salt)
    y = torch.empty(nb, device=D)
    dev.reduce_scatter(x, y)
    check("reg_reduce_scatter", y, oracle(p * nb, torch.float32, "SUM", salt)[rank * nb:(rank + 1) * nb],
          torch.float32, p)
    if dev.registrations <= reg0:
        fails.append("registration: no segment was mapped for the large ordinary tensors")
    # the same tensors again: mapped slots are reused (no new registrations)
    reg1 = dev.registrations
    x = gen(rank, n, torch.float32, 424242)
    y = torch.empty_like(x)
    dev.allreduce(x, y, "SUM", "fanout")
    dev.allreduce(x, y, "SUM", "fanout")
    check("reg_reuse", y, oracle(n, torch.float32, "SUM", 424242), torch.float32, p)
    if dev.registrations - reg1 > 2:
        fails.append(f"registration: {dev.registrations - reg1} new slots for two identical calls")
    # free every cached segment, allocate again (likely at the same addresses): the
    # allocator generation changes, stale slots are dropped, results stay exact
    del x, y
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    for it in range(3):
        salt += 1
        x = gen(rank, n, torch.float32, salt)
        y = torch.empty_like(x)
        dev.allreduce(x, y, "SUM", "fanout")
        check(f"reg_after_free[{it}]", y, oracle(n, torch.float32, "SUM", salt), torch.float32, p)
        del x, y
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
    # mixed: heap input on every rank, ordinary output
    salt += 1
    xs = sym_copy(gen(rank, n, torch.float32, salt))
    y = torch.empty(n, device=D)
    dev.allreduce(xs, y, "SUM", "fanout")
    check("reg_mixed_heap_ordinary", y, oracle(n, torch.float32, "SUM", salt), torch.float32, p)
    torch.cuda.synchronize()
    dev.check()

_lap("register")
# ------------------------------------------------------- >= 96 MiB: chunk loops
if args.big:
    n = (24 << 20) + 5  # 96 MiB + 20 B of fp32: > 32 MiB staging chunks, odd tail
    for algo in ("twoshot", "fanout", "fanout_lds", "ring") + (("rhd",) if POW2 else ()):
        for sym in (False, True):
            salt += 1
            x = gen(rank, n, torch.float32, salt)
            if sym:
                x, y = sym_copy(x), dev.empty(n, torch.float32)
            else:
                y = torch.empty_like(x)
            dev.allreduce(x, y, "SUM", algo)
            check(f"big_allreduce[{algo},sym={sym}]", y, oracle(n, torch.float32, "SUM", salt), torch.float32, p)
            del x, y
    nb = ((24 << 20) // p) + 3
    salt += 1
    x = gen(rank, p * nb, torch.float32, salt)
    y = torch.empty_like(x)
    dev.alltoall(x, y)
    want = torch.cat([gen(r, p * nb, torch.float32, salt)[rank * nb:(rank + 1) * nb] for r in range(p)]).double()
    check("big_alltoall[staged]", y, want, torch.float32)
    y2 = torch.empty_like(x)
    dev.alltoall(x, y2, "pairwise")
    check("big_alltoall[pairwise,staged]", y2, want, torch.float32)
    del y2
    dev.alltoall(x, x)
    check("big_alltoall[inplace]", x, want, torch.float32)
    salt += 1
    x = gen(rank, p * nb, torch.float32, salt)
    y = torch.empty(nb, device=D)
    dev.reduce_scatter(x, y)
    check("big_reduce_scatter[staged]", y, oracle(p * nb, torch.float32, "SUM", salt)[rank * nb:(rank + 1) * nb],
          torch.float32, p)
    salt += 1
    x = gen(rank, nb, torch.float32, salt)
    y = torch.empty(p * nb, device=D)
    dev.allgather(x, y)
    check("big_allgather[staged]", y, torch.cat([gen(r, nb, torch.float32, salt) for r in range(p)]).double(),
          torch.float32)
    torch.cuda.empty_cache()

torch.cuda.synchronize()
dev.check()

# ---------------------------------------------------- RCCL (fails loudly)
if args.rccl:
    x = gen(rank, 4096, torch.float32, 7)
    y = torch.empty_like(x)
    dev.allreduce(x, y, "SUM", "rccl")
    check("rccl_allreduce", y, oracle(4096, torch.float32, "SUM", 7), torch.float32, p)
    x = gen(rank, p * 999, torch.float32, 13)
    y = torch.empty_like(x)
    dev.alltoall(x, y, "pairwise_rccl")
    check("p2p_pairwise_alltoall", y,
          torch.cat([gen(r, p * 999, torch.float32, 13)[rank * 999:(rank + 1) * 999] for r in range(p)]).double(),
          torch.float32)

# communicator façade + accounting on device tensors
x = gen(rank, 1024, torch.float32, 11)
y = torch.empty_like(x)
before = comm.total_bytes_transferred
comm.myAllreduce(x, y, MPI.SUM)
check("myAllreduce(device)", y, oracle(1024, torch.float32, "SUM", 11), torch.float32, p)
want_bytes = 2 * 4096 * (p - 1) if rank == 0 else 2 * 4096
if comm.total_bytes_transferred - before != want_bytes:
    fails.append(f"myAllreduce accounting {comm.total_bytes_transferred - before} != {want_bytes}")
_lap("big/rccl")
if args.matrix:
    async_ops()  # last: an extra stream per process slows 8 processes sharing a GPU (DeviceGroup.start)
    _lap("async_ops")
finish(t0)
