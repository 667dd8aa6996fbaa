"""TP all-reduce overlap in the harness forward.

    scripts/mpirun -n 2 python benchmarks/tp_overlap.py [--batch 2048]

Per-token row-parallel fc_o (``fc_o_mode="token"``, the (B, S, out) shape of
reference model/func_impl.py:94-109): the TP all-reduce carries B*S x 16 fp32
partial outputs.  Times the HIP-graph forward with attention -> fc_o GEMM ->
all-reduce in 1 block (no overlap), and in 2 / 4 / 8 row blocks whose
all-reduces run on a side stream under the next block's attention, plus the
pooled row-parallel default for reference.  One JSON line.
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

from collective_communication_mpi_amd import MPI, Communicator  # noqa: E402
from collective_communication_mpi_amd.models.harness import bench_forward  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=2048)
ap.add_argument("--steps", type=int, default=50)
ap.add_argument("--chunks", default="1,2,4,8")
args = ap.parse_args()
comm = Communicator(MPI.COMM_WORLD)
local = int(os.environ.get("LOCAL_RANK", os.environ.get("CCMPI_LOCAL_RANK", "0")))
torch.cuda.set_device(local % torch.cuda.device_count())
tp = 2 if comm.Get_size() % 2 == 0 else 1
res = {}
for c in [int(x) for x in args.chunks.split(",")]:
    r = bench_forward(comm, tp=tp, batch=args.batch, steps=args.steps, warmup=5, train=False, fc_o_mode="token",
                      tp_chunks=c)
    res[f"token_chunks{c}_fwd_ms"] = round(r["fwd_ms"], 4)
r = bench_forward(comm, tp=tp, batch=args.batch, steps=args.steps, warmup=5, train=False)
res["row_pooled_fwd_ms"] = round(r["fwd_ms"], 4)
shared = comm.dev.shared_device  # collective on first use: every rank evaluates it
if comm.Get_rank() == 0:
    print(json.dumps({"bench": "tp_overlap", "ranks": comm.Get_size(), "tp": tp, "batch_per_replica": args.batch,
                      "tp_allreduce_bytes_token": args.batch * 16 * 16 * 4, "shared_gpu": shared,
                      **res}), flush=True)
