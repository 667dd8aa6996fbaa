"""Record what RCCL does when several ranks share ONE GPU.

    scripts/mpirun -n 2 python benchmarks/rccl_shared_probe.py [--out gpurun_out/rccl_probe.json]

Every rank tries, in order: ncclCommInitRank (via ``ensure_rccl``), an
ncclAllReduce, the RCCL-send/recv ring and recursive halving/doubling
schedules, and the pairwise all-to-all.  The outcome of each step (ok / the
exact exception text / wrong result) is gathered on rank 0 and written as
JSON, so the behaviour is on record instead of being swallowed.  Every step
runs under the device timeout and the launcher's wall clock.
"""
import argparse
import json
import os
import sys
import time
import traceback

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

import torch  # noqa: E402

from collective_communication_mpi_amd import MPI, Communicator  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--out", default="")
args = ap.parse_args()

comm = Communicator(MPI.COMM_WORLD)
rank, p = comm.Get_rank(), comm.Get_size()
dev = comm.dev
res = {}


def step(name, fn):
    t0 = time.time()
    try:
        ok = fn()
        torch.cuda.synchronize()
        res[name] = {"ok": bool(ok), "s": round(time.time() - t0, 3)}
    except Exception as e:  # noqa: BLE001 - the point of the probe is to record the error text
        res[name] = {"ok": False, "error": f"{type(e).__name__}: {e}", "trace": traceback.format_exc()[-800:],
                     "s": round(time.time() - t0, 3)}
    return res[name]["ok"]


def init():
    dev.ensure_rccl()
    return True


def ar(algo):
    def f():
        x = torch.full((10001,), float(rank + 1), device=dev.device)
        y = torch.empty_like(x)
        dev.allreduce(x, y, "SUM", algo)
        torch.cuda.synchronize()
        return bool(torch.all(y == p * (p + 1) / 2).item())
    return f


def a2a():
    x = torch.arange(p * 64, device=dev.device, dtype=torch.float32) + 1000 * rank
    y = torch.empty_like(x)
    dev.alltoall(x, y, "pairwise")
    torch.cuda.synchronize()
    want = torch.cat([torch.arange(rank * 64, rank * 64 + 64, dtype=torch.float32) + 1000 * r for r in range(p)])
    return bool(torch.equal(y.cpu(), want))


res["ranks_per_device"] = dev.ranks_per_device
if step("ncclCommInitRank", init):
    step("ncclAllReduce", ar("rccl"))
    step("pairwise_alltoall", a2a)
allres = comm.comm.gather(res, root=0)
if rank == 0:
    out = {"ranks": p, "torch": torch.__version__, "per_rank": allres}
    s = json.dumps(out, indent=1)
    print(s, flush=True)
    if args.out:
        with open(args.out, "w") as f:
            f.write(s + "\n")
