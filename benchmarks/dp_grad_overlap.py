"""DP gradient all-reduce overlapped with backward (BASELINE config 5); the
measurement lives in ``collective_communication_mpi_amd/parallel/overlap.py``.

    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 benchmarks/dp_grad_overlap.py --layers 32
    scripts/mpirun -n 2 python benchmarks/dp_grad_overlap.py --layers 4 --tokens 2048
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

from collective_communication_mpi_amd import MPI, Communicator  # noqa: E402
from collective_communication_mpi_amd.parallel.overlap import dp_grad_overlap  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--layers", type=int, default=32)
ap.add_argument("--tokens", type=int, default=4096, help="tokens per rank per step")
ap.add_argument("--iters", type=int, default=3)
ap.add_argument("--algo", default="auto")
ap.add_argument("--comm-priority", type=int, default=0, help="side-stream priority (-1 = high, 0 = normal)")
ap.add_argument("--verbose", action="store_true")
ap.add_argument("--blocks", type=int, default=0, help="CTA budget of the bucket all-reduces (0 = overlap_blocks)")
ap.add_argument("--bucket-mb", type=int, default=0, help="max bucket size in MiB (0 = one bucket per layer)")
args = ap.parse_args()
if args.verbose:  # a stuck setup shows where it is stuck (every rank, every 90 s)
    import faulthandler

    faulthandler.dump_traceback_later(90, repeat=True)
comm = Communicator(MPI.COMM_WORLD)
local = int(os.environ.get("LOCAL_RANK", os.environ.get("CCMPI_LOCAL_RANK", "0")))
torch.cuda.set_device(local % torch.cuda.device_count())
res = dp_grad_overlap(comm, layers=args.layers, tokens=args.tokens, iters=args.iters, algo=args.algo,
                      priority=args.comm_priority, verbose=args.verbose, max_blocks=args.blocks,
                      bucket_mb=args.bucket_mb)
if comm.Get_rank() == 0:
    print(json.dumps({"bench": "dp_grad_overlap", "comm_priority": args.comm_priority, **res}), flush=True)
