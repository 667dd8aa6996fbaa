"""Sweep the fused-projection attention forward's grid (workgroups) on the harness shape:
inference forward (save=False) and saving forward, eager, CUDA-event timed."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

from collective_communication_mpi_amd import MPI, Communicator, _native  # noqa: E402
from collective_communication_mpi_amd.models.harness import build  # noqa: E402
from collective_communication_mpi_amd.models.mnist_tp import local_batch  # noqa: E402


def t(fn, iters=30):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters * 1e3


comm = Communicator(MPI.COMM_WORLD)
D = _native.device()
for fuse in (False, True):
    cfg, layer, x_all, y_all = build(comm, 1, 2048, fuse_qkv_attn=fuse)
    xb, _ = local_batch(cfg, x_all, y_all, 0, 0, layer.device)
    grids = (256, 512, 1024, 2048) if fuse else (0,)
    for g in grids:
        D.attn_set_fwd_proj_grid(g)
        inf = t(lambda: layer.forward_images(xb, cfg.batch, save=False))
        sav = t(lambda: layer.forward_images(xb, cfg.batch, save=True))
        print(f"fuse_qkv_attn={fuse} grid={g}: inference fwd {inf:.1f} us, saving fwd {sav:.1f} us", flush=True)
D.attn_set_fwd_proj_grid(0)
