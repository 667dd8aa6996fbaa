"""A bench-written tuning table drives ``algo="auto"`` of a later device group.

    python -m collective_communication_mpi_amd.launch -n 4 python tests/workers/tune_worker.py --file T.json

1. bench.py's tuning sweep (``bench.tuning_sweep``: DeviceGroup.tune over every hand-written
   algorithm ``auto`` may pick, ring and RHD included) writes the table to CCMPI_TUNE_FILE;
2. rank 0 then forces "ring" for the 1 MiB class and "rhd" for the 4 MiB class in that file
   (so the check does not depend on which algorithm happened to win on this GPU);
3. a NEW communicator's device group loads the file at start-up, ``pick_allreduce`` returns
   the table's choice, and ``allreduce(algo="auto")`` runs it (exact rank-valued result).
Prints "tune OK"."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
import torch  # noqa: E402

import bench  # noqa: E402
from collective_communication_mpi_amd import MPI, Communicator  # noqa: E402
from collective_communication_mpi_amd.device import save_tuning  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--file", required=True)
args = ap.parse_args()
os.environ["CCMPI_TUNE_FILE"] = args.file
comm = Communicator(MPI.COMM_WORLD)
torch.cuda.set_device(int(os.environ.get("CCMPI_LOCAL_RANK", "0")) % torch.cuda.device_count())
rank, p = comm.Get_rank(), comm.Get_size()
fails = []
bargs = bench.parse(["--tune-max-mb", "4", "--size-mb", "64"])
rec = bench.tuning_sweep(comm, bargs, "fanout:512")
if not rec or not rec["table"]:
    fails.append(f"tuning sweep wrote no table: {rec}")
comm.comm.Barrier()
if rank == 0:
    tables = json.load(open(args.file))
    if comm.dev.tune_key not in tables:
        fails.append(f"{comm.dev.tune_key} missing from {list(tables)}")
    table = {tuple(int(v) for v in k.split(",")): a for k, a in tables.get(comm.dev.tune_key, {}).items()}
    table[(p, 20)] = "ring"
    table[(p, 22)] = "rhd"
    save_tuning(args.file, comm.dev.tune_key, table)
comm.comm.Barrier()
new = comm.Split(0, 0)  # reference order (key, color): every rank, same order -> same size
dev = new.dev
for nbytes, want in ((1 << 20, "ring"), (4 << 20, "rhd")):
    got = dev.pick_allreduce(nbytes)
    if got != want:
        fails.append(f"auto at {nbytes} B picked {got}, table says {want}")
    x = dev.empty(nbytes // 4, torch.float32)
    y = dev.empty(nbytes // 4, torch.float32)
    x.fill_(float(rank + 1))
    dev.allreduce(x, y, "SUM", "auto")
    torch.cuda.synchronize()
    if not torch.all(y == p * (p + 1) / 2).item():
        fails.append(f"auto ({want}) all-reduce at {nbytes} B wrong")
bad = comm.comm.allgather(fails)
if rank == 0:
    flat = [f"rank {r}: {m}" for r, ms in enumerate(bad) for m in ms]
    print("\n".join(flat) if flat else "tune OK", flush=True)
sys.exit(1 if any(bad) else 0)
