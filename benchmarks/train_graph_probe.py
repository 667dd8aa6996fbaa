"""Harness training step: eager vs HIP-graph replay (models/harness.GraphedTrainStep), event
timed, one rank; run under rocprofv3 --kernel-trace to see a replay's kernels and gaps."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

from collective_communication_mpi_amd import MPI, Communicator  # noqa: E402
from collective_communication_mpi_amd.models.harness import GraphedTrainStep, TrainPlan, build, train_step  # noqa: E402
from collective_communication_mpi_amd.models.mnist_tp import local_batch  # noqa: E402

comm = Communicator(MPI.COMM_WORLD)
batch = int(os.environ.get("TG_BATCH", "2048"))
cfg, layer, x_all, y_all = build(comm, 1, batch, fc_o_mode="token")
xb, yb = local_batch(cfg, x_all, y_all, 0, 0, layer.device)
for _ in range(3):
    train_step(layer, cfg, xb, yb)
torch.cuda.synchronize()
n = 20
t0 = time.perf_counter()
for _ in range(n):
    train_step(layer, cfg, xb, yb)
torch.cuda.synchronize()
eager = (time.perf_counter() - t0) / n * 1e3
gts = GraphedTrainStep(layer, cfg, xb, yb)
for _ in range(4):
    gts.replay()
torch.cuda.synchronize()
torch.cuda.nvtx.range_push("graph") if hasattr(torch.cuda, "nvtx") else None
t0 = time.perf_counter()
for _ in range(n):
    gts.replay()
torch.cuda.synchronize()
graph = (time.perf_counter() - t0) / n * 1e3
t0 = time.perf_counter()
for _ in range(n):
    gts.graphs[0].replay()
torch.cuda.synchronize()
one = (time.perf_counter() - t0) / n * 1e3
gts.close()
res = {"eager_ms": round(eager, 4), "graph_alternating_ms": round(graph, 4), "graph_same_ms": round(one, 4)}
if TrainPlan.available(layer, cfg):
    tp_ = TrainPlan(layer, cfg, xb, yb)
    for _ in range(4):
        tp_.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        tp_.replay()
    torch.cuda.synchronize()
    res["plan_ms"] = round((time.perf_counter() - t0) / n * 1e3, 4)
    res["plan_launches"] = len(tp_.plans[0].calls)
    tp_.close()
print(res, flush=True)
