"""DP x TP harness forward on N ranks (the bench's shared-GPU dry run without the
collective sweeps), for repeated timings and rocprofv3 kernel traces.

    python -m collective_communication_mpi_amd.launch -n 8 python benchmarks/harness_dryrun.py --tp 2
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
ap.add_argument("--tp", type=int, default=2)
ap.add_argument("--batch", type=int, default=2048)
ap.add_argument("--steps", type=int, default=20)
ap.add_argument("--warmup", type=int, default=5)
ap.add_argument("--fc-o-mode", default="token", choices=["row", "token"])
ap.add_argument("--no-graph", action="store_true")
args = ap.parse_args()
comm = Communicator(MPI.COMM_WORLD)
torch.cuda.set_device(int(os.environ.get("CCMPI_LOCAL_RANK", "0")) % torch.cuda.device_count())
r = bench_forward(comm, tp=args.tp, batch=args.batch, steps=args.steps, warmup=args.warmup, train=False,
                  graph=not args.no_graph, fc_o_mode=args.fc_o_mode)
if comm.Get_rank() == 0:
    print(json.dumps({"ranks": comm.Get_size(), "hw_queues": os.environ.get("GPU_MAX_HW_QUEUES"), **r}), flush=True)
