"""Run the harness forward (eager, no graph) or full train step N times, for
rocprofv3 kernel statistics.

    python benchmarks/harness_steps.py --mode fwd|train --steps 20 [--tp 1 --batch 2048 --fc-o-mode token]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

from collective_communication_mpi_amd import MPI, Communicator  # noqa: E402
from collective_communication_mpi_amd.models.harness import build, train_step  # noqa: E402
from collective_communication_mpi_amd.models.mnist_tp import local_batch  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--mode", default="fwd")
ap.add_argument("--steps", type=int, default=20)
ap.add_argument("--tp", type=int, default=1)
ap.add_argument("--batch", type=int, default=2048)
ap.add_argument("--fc-o-mode", default="row", choices=["row", "token", "naive"])
args = ap.parse_args()
comm = Communicator(MPI.COMM_WORLD)
torch.cuda.set_device(int(os.environ.get("CCMPI_LOCAL_RANK", "0")) % torch.cuda.device_count())
cfg, layer, x_all, y_all = build(comm, args.tp, args.batch, fc_o_mode=args.fc_o_mode)
xb, yb = local_batch(cfg, x_all, y_all, 0, comm.Get_rank(), layer.device)
for _ in range(args.steps):
    if args.mode == "fwd":
        layer.forward_images(xb, cfg.batch, save=False)  # inference forward, as bench.py times it
    else:
        train_step(layer, cfg, xb, yb)
torch.cuda.synchronize()
print("done", args.mode)
