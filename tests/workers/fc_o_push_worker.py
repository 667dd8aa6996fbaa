"""the harness's per-token fc_o in its two TP forms -- "plain" (attention
+ fc_o kernel, then an all-reduce of z) and "push" (the kernel stores every row block of its
partial z straight into the owner's inbox, then the inbox-to-local two-shot) -- must give
bitwise the same z and logits on every rank; then two training steps in the push form."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
from collective_communication_mpi_amd import MPI, Communicator  # noqa: E402
from collective_communication_mpi_amd.models.harness import build, fc_o_forms_agree, train_step  # noqa: E402
from collective_communication_mpi_amd.models.mnist_tp import local_batch  # noqa: E402

comm = Communicator(MPI.COMM_WORLD)
torch.cuda.set_device(0 if torch.cuda.device_count() == 1 else comm.Get_rank() % torch.cuda.device_count())
tp = int(os.environ.get("FC_O_TP", "2"))
r = fc_o_forms_agree(comm, tp, 128)
assert r["equal"], r
cfg, layer, x_all, y_all = build(comm, tp, 128, fc_o_mode="token", tp_fc_o_form="push", lr=2e-3)
losses = []
for step in range(2):
    xb, yb = local_batch(cfg, x_all, y_all, step, comm.Get_rank(), layer.device)
    losses.append(float(train_step(layer, cfg, xb, yb).item()))
torch.cuda.synchronize()
assert layer._zt_form == "push" and all(v == v for v in losses), (layer._zt_form, losses)
if comm.Get_rank() == 0:
    print("fc_o push OK", r, losses, flush=True)
