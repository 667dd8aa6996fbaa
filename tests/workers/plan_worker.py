"""MnistTPLayer.forward_plan: the forward's recorded native launches re-issued from a loop give
bitwise the forward_images logits, and keep doing so after new pixels are written into the
images tensor and a training step changes the weights (the plan reads live buffers).  The
pipelined-fold plan (the next call's weight fold in the fused kernel's tail) likewise, over
several calls and after a weight change."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
from collective_communication_mpi_amd import MPI, Communicator  # noqa: E402
from collective_communication_mpi_amd.models.harness import build, train_step  # noqa: E402
from collective_communication_mpi_amd.models.mnist_tp import local_batch  # noqa: E402

comm = Communicator(MPI.COMM_WORLD)
torch.cuda.set_device(0 if torch.cuda.device_count() == 1 else comm.Get_rank() % torch.cuda.device_count())
tp = int(os.environ.get("PL_TP", "1"))
kw = {"tp_fc_o_form": "push"} if tp > 1 else {}
cfg, layer, x_all, y_all = build(comm, tp, 256, fc_o_mode="token", lr=2e-3, **kw)
xb, yb = local_batch(cfg, x_all, y_all, 0, comm.Get_rank(), layer.device)
xb = xb.float().contiguous()
train_step(layer, cfg, xb, yb)
plan = layer.forward_plan(xb, cfg.batch)
assert plan is not None, "forward_plan unavailable"
names = plan.names()
assert "attn_qkv_fwd" in names and (tp == 1 or "inbox_mean" in names), names
ref = layer.forward_images(xb, cfg.batch, save=False).clone()
out = plan().clone()
torch.cuda.synchronize()
assert torch.equal(out, ref), (out - ref).abs().max().item()
xb.mul_(0.5)                          # new pixels, same storage
train_step(layer, cfg, xb, yb)        # new weights
ref2 = layer.forward_images(xb, cfg.batch, save=False).clone()
out2 = plan().clone()
torch.cuda.synchronize()
assert torch.equal(out2, ref2) and not torch.equal(out2, out), ((out2 - ref2).abs().max().item())
# the pipelined-fold plan: every call bitwise forward_images (W_eff folded by the previous
# call's kernel tail), across calls and after the weights change
pp = layer.forward_plan_pipelined(xb, cfg.batch)
assert pp is not None, "forward_plan_pipelined unavailable"
assert "fold_emb_qkv" not in pp.names(), pp.names()
ref3 = layer.forward_images(xb, cfg.batch, save=False).clone()
for i in range(5):
    o = pp().clone()
    torch.cuda.synchronize()
    assert torch.equal(o, ref3), (i, (o - ref3).abs().max().item())
train_step(layer, cfg, xb, yb)        # new weights: the next call folds its own W_eff first
ref4 = layer.forward_images(xb, cfg.batch, save=False).clone()
for i in range(3):
    o = pp().clone()
    torch.cuda.synchronize()
    assert torch.equal(o, ref4) and not torch.equal(o, ref3), (i, (o - ref4).abs().max().item())
if comm.Get_rank() == 0:
    print("plan OK", names, flush=True)
