"""BASELINE config 5 on a real backward: DistributedDataParallel over a Llama-3-8B-shaped
model of the framework's own layers (parallel/llama_dp.py), bucket all-reduces launched
from the autograd backward.

    python -m collective_communication_mpi_amd.launch -n 2 python benchmarks/llama_ddp.py --layers 32
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 benchmarks/llama_ddp.py

Prints one JSON line (rank 0): compute-only / comm-only / overlapped step times, the
hidden fraction, and the CTA-budget sweep of the bucket all-reduces."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

from collective_communication_mpi_amd import MPI, Communicator  # noqa: E402
from collective_communication_mpi_amd.parallel.llama_dp import measure_ddp_overlap  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--layers", type=int, default=32)
ap.add_argument("--tokens", type=int, default=4096, help="tokens per rank per step")
ap.add_argument("--seq", type=int, default=2048)
ap.add_argument("--vocab", type=int, default=1, help="include the token embedding and the LM head")
ap.add_argument("--iters", type=int, default=2)
ap.add_argument("--bucket-mb", type=int, default=0, help="DDP bucket size (0 = CCMPI_DP_BUCKET_MB / 64)")
ap.add_argument("--blocks", default="32,64,128,256", help="CTA budgets of the bucket all-reduces to sweep")
ap.add_argument("--verbose", action="store_true")
args = ap.parse_args()
comm = Communicator(MPI.COMM_WORLD)
torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", os.environ.get("CCMPI_LOCAL_RANK", "0"))) %
                      torch.cuda.device_count())
res = measure_ddp_overlap(comm, layers=args.layers, tokens=args.tokens, seq=args.seq, vocab=bool(args.vocab),
                          iters=args.iters, bucket_mb=args.bucket_mb or None,
                          blocks_sweep=[int(b) for b in args.blocks.split(",")], verbose=args.verbose)
if comm.Get_rank() == 0:
    print(json.dumps({"bench": "llama_ddp", **res}), flush=True)
