"""Multi-rank device-plane check (launched by scripts/mpirun; several ranks may
share one GPU).  Every device collective is compared with a torch fp64/exact
oracle built from all ranks' inputs (inputs are generated from per-rank seeds,
so each rank can rebuild every peer's input locally).

usage: device_worker.py [--quick] [--rccl] [--sizes 1,17,4096,...] [--stress N] [--fault]

--stress N  SURVEY §5.2: N back-to-back collectives (mixed algorithms and sizes,
            no host synchronisation in between) with randomised per-rank host
            sleeps and device-side spin delays, so ranks arrive at each kernel
            in random order; every result is checked at the end (epoch/ABA safety).
--fault     SURVEY §5.3: rank p-1 skips one collective; the others must time out
            (bounded spins), the host watchdog must see the code without a device
            sync, check() must raise, and reset() must restore a working group.
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
from collective_communication_mpi_amd import MPI, Communicator  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--quick", action="store_true")
ap.add_argument("--rccl", action="store_true")
ap.add_argument("--sizes", default="")
ap.add_argument("--stress", type=int, default=0)
ap.add_argument("--fault", action="store_true")
args = ap.parse_args()

comm = Communicator(MPI.COMM_WORLD)
rank, p = comm.Get_rank(), comm.Get_size()
dev = comm.dev
torch.cuda.synchronize()
fails = []


def gen(r, n, dtype, salt):
    g = torch.Generator(device="cpu").manual_seed(1000 * r + salt)
    if dtype.is_floating_point:
        return (torch.randn(n, generator=g, dtype=torch.float64) * 3).to(dtype)
    return torch.randint(-1000, 1000, (n,), generator=g, dtype=torch.int64).to(dtype)


def oracle(n, dtype, op, salt):
    xs = [gen(r, n, dtype, salt).to(torch.float64 if dtype.is_floating_point else torch.int64) for r in range(p)]
    acc = xs[0].clone()
    for x in xs[1:]:
        if op == "SUM":
            acc = acc + x
        elif op == "MAX":
            acc = torch.maximum(acc, x)
        elif op == "MIN":
            acc = torch.minimum(acc, x)
        else:
            acc = acc * x
    return acc


def check(name, got, want, dtype, nterms=1):
    got = got.detach().cpu().to(torch.float64 if dtype.is_floating_point else torch.int64)
    if dtype.is_floating_point:
        tol = {torch.float32: 1e-5, torch.float64: 1e-12, torch.bfloat16: 1e-2, torch.float16: 2e-3}[dtype] * nterms
        ok = torch.allclose(got, want, rtol=tol, atol=tol * 4)
    else:
        ok = torch.equal(got, want)
    if not ok:
        diff = (got - want).abs().max().item() if got.shape == want.shape else "shape"
        fails.append(f"{name}: max diff {diff}")
    return ok


def stress(iters):
    """Random arrival order at every collective; results checked after the burst."""
    import random

    rng = random.Random(1234 + rank)  # per-rank: delays only
    shared = random.Random(99)        # identical on every rank: sizes and algorithms
    pending = []
    algos_s = ["oneshot", "twoshot", "push", "reduce_bcast"]
    sym_x = dev.empty(1 << 16, torch.float32)
    for i in range(iters):
        n = shared.choice([1, 33, 4096, 1 << 16])
        algo = shared.choice(algos_s)
        d = rng.random()
        if d < 0.3:
            time.sleep(rng.random() * 0.004)
        elif d < 0.6:
            torch.cuda._sleep(rng.randint(1000, 200000))  # device-side skew
        x = gen(rank, n, torch.float32, 50000 + i).to(dev.device, non_blocking=True)
        if i % 3 == 0:  # symmetric, zero-copy path
            xs = sym_x[:n]
            xs.copy_(x)
            x = xs
        y = torch.empty(n, dtype=torch.float32, device=dev.device)
        dev.allreduce(x, y, "SUM", algo)
        pending.append((f"stress[{i},{algo},n={n}]", y.clone(), n, 50000 + i))
    torch.cuda.synchronize()
    dev.check()
    for name, y, n, sl in pending:
        check(name, y, oracle(n, torch.float32, "SUM", sl), torch.float32, p)


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
    dev.allreduce(x, y, "SUM", "twoshot")
    check("fault_recovery_allreduce", y, torch.full((4096,), float(p), dtype=torch.float64), torch.float32)


if args.stress or args.fault:
    t0 = time.time()
    if args.stress:
        stress(args.stress)
    if args.fault:
        fault()
    comm.Barrier()
    print(f"[rank {rank}/{p}] stress/fault checks: {len(fails)} failures, {time.time() - t0:.1f}s", flush=True)
    for f in fails[:20]:
        print(f"[rank {rank}] FAIL {f}", flush=True)
    sys.exit(1 if fails else 0)

sizes = [int(s) for s in args.sizes.split(",") if s] or ([1, 7, 1000, 65536 + 3] if args.quick else
                                                          [1, 3, 8, 1000, 4097, 65536 + 3, 1 << 20, (1 << 22) + 5])
dtypes = [torch.float32, torch.bfloat16] if args.quick else [torch.float32, torch.bfloat16, torch.float16,
                                                              torch.float64, torch.int32, torch.int64]
algos = ["oneshot", "twoshot", "reduce_bcast", "push"]
salt = 0
t0 = time.time()
for sym in (False, True):
    for n in sizes:
        for dt in dtypes:
            for op in (["SUM", "MAX"] if not args.quick else ["SUM"]):
                for algo in algos:
                    salt += 1
                    x = gen(rank, n, dt, salt).to(dev.device)
                    if sym:
                        xs = dev.empty(n, dt); xs.copy_(x); x = xs
                        y = dev.empty(n, dt)
                    else:
                        y = torch.empty_like(x)
                    dev.allreduce(x, y, op, algo)
                    check(f"allreduce[{algo},{dt},{op},n={n},sym={sym}]", y, oracle(n, dt, op, salt), dt, p)
                    # in-place
                    z = gen(rank, n, dt, salt).to(dev.device)
                    dev.allreduce(z, z, op, algo)
                    check(f"allreduce_inplace[{algo},{dt},{op},n={n}]", z, oracle(n, dt, op, salt), dt, p)
    for n in sizes[:6]:
        for dt in dtypes[:2]:
            salt += 1
            # reduce_scatter: input p*n, output n (block = rank)
            x = gen(rank, p * n, dt, salt).to(dev.device)
            if sym:
                xs = dev.empty(p * n, dt); xs.copy_(x); x = xs
            y = torch.empty(n, dtype=dt, device=dev.device)
            dev.reduce_scatter(x, y, "SUM")
            full = oracle(p * n, dt, "SUM", salt)
            check(f"reduce_scatter[{dt},n={n},sym={sym}]", y, full[rank * n:(rank + 1) * n], dt, p)
            # allgather
            salt += 1
            x = gen(rank, n, dt, salt).to(dev.device)
            if sym:
                xs = dev.empty(n, dt); xs.copy_(x); x = xs
            y = torch.empty(p * n, dtype=dt, device=dev.device)
            dev.allgather(x, y)
            want = torch.cat([gen(r, n, dt, salt) for r in range(p)]).to(torch.float64 if dt.is_floating_point else torch.int64)
            check(f"allgather[{dt},n={n},sym={sym}]", y, want, dt)
            # alltoall
            salt += 1
            x = gen(rank, p * n, dt, salt).to(dev.device)
            if sym:
                xs = dev.empty(p * n, dt); xs.copy_(x); x = xs
            y = torch.empty(p * n, dtype=dt, device=dev.device)
            dev.alltoall(x, y)
            want = torch.cat([gen(r, p * n, dt, salt)[rank * n:(rank + 1) * n] for r in range(p)]).to(
                torch.float64 if dt.is_floating_point else torch.int64)
            check(f"alltoall[{dt},n={n},sym={sym}]", y, want, dt)
            # bcast from root p-1
            salt += 1
            root = p - 1
            b = gen(rank, n, dt, salt).to(dev.device)
            if sym:
                bs = dev.empty(n, dt); bs.copy_(b); b = bs
            dev.bcast(b, root)
            check(f"bcast[{dt},n={n},sym={sym}]", b, gen(root, n, dt, salt).to(torch.float64 if dt.is_floating_point else torch.int64), dt)

# TP layout-fused collectives (reference naive collects on device tensors)
from collective_communication_mpi_amd.parallel.layout import (  # noqa: E402
    naive_collect_backward_x, naive_collect_forward_input)
for dt in (torch.float32, torch.bfloat16):
    for (B, S, k) in [(2, 3, 8), (4, 16, 64), (3, 5, 3)]:
        salt += 1
        shards = [gen(r, B * S * k, dt, salt).view(B, S, k) for r in range(p)]
        got = naive_collect_forward_input(shards[rank].to(dev.device), comm, p)
        want = torch.cat(shards, dim=-1).to(torch.float64 if dt.is_floating_point else torch.int64)
        check(f"forward_input_lastaxis[{dt},{B}x{S}x{k}]", got, want, dt)
        salt += 1
        full = [gen(r, B * S * k * p, dt, salt).view(B, S, k * p) for r in range(p)]
        got = naive_collect_backward_x(full[rank].to(dev.device), comm, p)
        ref = sum(f.to(torch.float64) for f in full)[:, :, rank * k:(rank + 1) * k]
        check(f"backward_x_lastaxis[{dt},{B}x{S}x{k}]", got, ref, dt, p)
torch.cuda.synchronize()
dev.check()
if args.rccl:
    try:
        x = gen(rank, 4096, torch.float32, 7).to(dev.device)
        y = torch.empty_like(x)
        dev.allreduce(x, y, "SUM", "rccl")
        check("rccl_allreduce", y, oracle(4096, torch.float32, "SUM", 7), torch.float32, p)
        for algo in ("ring", "rhd"):
            x = gen(rank, 10001, torch.float32, 9).to(dev.device)
            dev.allreduce(x, x, "SUM", algo)
            check(f"p2p_{algo}", x, oracle(10001, torch.float32, "SUM", 9), torch.float32, p)
    except Exception as e:  # noqa: BLE001
        print(f"[rank {rank}] RCCL path unavailable: {e}", flush=True)

# communicator façade + accounting on device tensors
x = gen(rank, 1024, torch.float32, 11).to(dev.device)
y = torch.empty_like(x)
comm.myAllreduce(x, y, MPI.SUM)
check("myAllreduce(device)", y, oracle(1024, torch.float32, "SUM", 11), torch.float32, p)
comm.Barrier()
msg = f"[rank {rank}/{p}] device checks: {len(fails)} failures, {time.time() - t0:.1f}s"
print(msg, flush=True)
for f in fails[:20]:
    print(f"[rank {rank}] FAIL {f}", flush=True)
sys.exit(1 if fails else 0)
