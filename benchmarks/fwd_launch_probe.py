"""Harness forward launch modes at N = 1: HIP graph replay of one forward, a graph holding two
forwards (per-forward time: how much of a replay is launch cost), eager forward_images, and a
recorded launch plan (the forward's native kernel calls with their arguments frozen, replayed
from a Python loop).  Diagnostic; prints one JSON line."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

from collective_communication_mpi_amd import MPI, Communicator, _native  # noqa: E402
from collective_communication_mpi_amd.models.harness import build  # noqa: E402
from collective_communication_mpi_amd.models.mnist_tp import local_batch  # noqa: E402

comm = Communicator(MPI.COMM_WORLD)
cfg, layer, x_all, y_all = build(comm, 1, 2048, fc_o_mode="token")
xb, yb = local_batch(cfg, x_all, y_all, 0, 0, layer.device)


def fwd():
    return layer.forward_images(xb, cfg.batch, save=False)


def timed(fn, n=50, per=1):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    t_host = time.perf_counter() - t0
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n / per * 1e3, t_host / n / per * 1e3


out = {}
ref = fwd().clone()
out["eager_ms"], out["eager_host_ms"] = timed(fwd)
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    fwd()
torch.cuda.current_stream().wait_stream(s)
torch.cuda.synchronize()
g1 = torch.cuda.CUDAGraph()
with torch.cuda.graph(g1):
    fwd()
out["graph1_ms"], out["graph1_host_ms"] = timed(g1.replay)
g2 = torch.cuda.CUDAGraph()
with torch.cuda.graph(g2):
    fwd()
    fwd()
out["graph2_per_fwd_ms"], _ = timed(g2.replay, per=2)
# record the forward's native launches
dev = _native.device()
calls = []


class Rec:
    def __getattr__(self, name):
        f = getattr(dev, name)
        if not callable(f):
            return f

        def w(*a, **k):
            calls.append((name, f, a, k))
            return f(*a, **k)
        return w


orig = _native.device
_native.device = lambda: Rec()
try:
    got = fwd()
finally:
    _native.device = orig
torch.cuda.synchronize()
out["plan_calls"] = [c[0] for c in calls]


def plan():
    for _, f, a, k in calls:
        f(*a, **k)


plan()
torch.cuda.synchronize()
out["plan_equal"] = bool(torch.equal(got, ref))
out["plan_ms"], out["plan_host_ms"] = timed(plan)
print(json.dumps({k: (round(v, 4) if isinstance(v, float) else v) for k, v in out.items()}), flush=True)
