"""The harness forward (N = 1) from the launch plan with and without the pipelined weight fold,
event timed; run under rocprofv3 --kernel-trace --stats to see the kernels of each."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

from collective_communication_mpi_amd import MPI, Communicator  # noqa: E402
from collective_communication_mpi_amd.models.harness import build  # noqa: E402
from collective_communication_mpi_amd.models.mnist_tp import local_batch  # noqa: E402

comm = Communicator(MPI.COMM_WORLD)
cfg, layer, x_all, y_all = build(comm, 1, 2048, fc_o_mode="token")
xb, yb = local_batch(cfg, x_all, y_all, 0, 0, layer.device)
xb = xb.float().contiguous()
out = {}
for name, mk in (("plan", layer.forward_plan), ("plan_pipelined_fold", layer.forward_plan_pipelined)):
    p = mk(xb, cfg.batch)
    for _ in range(10):
        p()
    torch.cuda.synchronize()
    n = 200
    t0 = time.perf_counter()
    for _ in range(n):
        p()
    torch.cuda.synchronize()
    out[name + "_ms"] = round((time.perf_counter() - t0) / n * 1e3, 4)
    out[name + "_launches"] = p.names()
print(json.dumps(out), flush=True)
