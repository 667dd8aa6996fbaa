"""Runs a few training steps of the DP x TP harness and writes rank 0's loss
curve (and final gathered weights) to --out (.npz).  Used by
tests/test_gpu_distributed.py to check that every (tp, dp, fc_o_mode) grid
reproduces the single-rank run."""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
from collective_communication_mpi_amd import MPI, Communicator  # noqa: E402
from collective_communication_mpi_amd.models.harness import build, train_step  # noqa: E402
from collective_communication_mpi_amd.models.mnist_tp import local_batch  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--tp", type=int, default=1)
ap.add_argument("--global-batch", type=int, default=256)
ap.add_argument("--steps", type=int, default=4)
ap.add_argument("--mode", default="row")
ap.add_argument("--out", required=True)
args = ap.parse_args()

comm = Communicator(MPI.COMM_WORLD)
world = comm.Get_size()
dp = world // args.tp
torch.cuda.set_device(0 if torch.cuda.device_count() == 1 else comm.Get_rank() % torch.cuda.device_count())
cfg, layer, x_all, y_all = build(comm, args.tp, args.global_batch // dp, fc_o_mode=args.mode, lr=2e-3)
losses = []
for step in range(args.steps):
    xb, yb = local_batch(cfg, x_all, y_all, step, comm.Get_rank(), layer.device)
    loss = train_step(layer, cfg, xb, yb)
    losses.append(comm.comm.allreduce(float(loss.item()), op=MPI.SUM) / cfg.tp)
torch.cuda.synchronize()
full = layer.gathered_full()
if comm.Get_rank() == 0:
    np.savez(args.out, losses=np.array(losses), q_w=full["q_w"].numpy(), o_w=full["o_w"].numpy(),
             emb_w=full["emb_w"].numpy())
    print("losses", losses, flush=True)
