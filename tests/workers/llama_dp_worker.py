"""DistributedDataParallel over a (tiny) Llama-shaped model built from the framework's TP
layers (parallel/llama_dp.py), vs a single-process reference.

    scripts/mpirun -n 2 python tests/workers/llama_dp_worker.py --device cpu
    scripts/mpirun -n 2 python tests/workers/llama_dp_worker.py --device cuda [--measure]

Every rank builds the same model (seeded) and its own token batch; after DDP's backward +
finish every rank's gradients must equal the mean over ranks of the per-rank gradients
of an unwrapped replica (computed here for every rank's batch), for two steps (the
second exercises zero_grad's sink reset) and with a micro-batch accumulation step.  On
CUDA the weight gradients of the TP layers must arrive through the gradient sinks.
``--measure``: also run measure_ddp_overlap on the tiny model.  ``--sink``: gradient sinks on
the CPU too (host plane); ``--penalty``: a weight penalty on TP weights (their gradient then
arrives through the layer's sink AND through autograd) -- the sum must still be
averaged exactly once.  Prints "llama dp OK"."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
from collective_communication_mpi_amd import MPI, Communicator  # noqa: E402
from collective_communication_mpi_amd.parallel import tensor_parallel as tp  # noqa: E402
from collective_communication_mpi_amd.parallel.ddp import DistributedDataParallel  # noqa: E402
from collective_communication_mpi_amd.parallel.llama_dp import (LlamaConfig, LlamaModel, _self_comm,  # noqa: E402
                                                                measure_ddp_overlap)

ap = argparse.ArgumentParser()
ap.add_argument("--device", default="cpu")
ap.add_argument("--measure", action="store_true")
ap.add_argument("--sink", action="store_true")
ap.add_argument("--penalty", type=float, default=0.0)
args = ap.parse_args()
comm = Communicator(MPI.COMM_WORLD)
hc = comm.comm
rank, p = comm.Get_rank(), comm.Get_size()
if args.device == "cuda":
    torch.cuda.set_device(int(os.environ.get("CCMPI_LOCAL_RANK", "0")) % torch.cuda.device_count())
    device, dt, tol = torch.device("cuda", torch.cuda.current_device()), torch.bfloat16, 0.06
else:
    device, dt, tol = torch.device("cpu"), torch.float32, 1e-4
cfg = LlamaConfig(d=128, heads=4, kv_heads=2, ffn=256, vocab=512, layers=2)
B, S = 2, 64
selfc = _self_comm(comm)
model = LlamaModel(cfg, selfc, device, dtype=dt, seed=3)
ref = LlamaModel(cfg, selfc, device, dtype=dt, seed=3)
ddp = DistributedDataParallel(model, comm, bucket_bytes=64 << 10, broadcast_params=False,
                              **({"grad_sink": True} if args.sink else {}))


def penalized(m):
    """Weights with an extra loss term (reach the weight through autograd, beside the sink)."""
    return [m.blocks[0].wq.weight, m.blocks[-1].mlp.down.weight, m.head.weight]


def loss_of(m, ids):
    loss = m(ids)
    if args.penalty:
        loss = loss + args.penalty * sum((w.float() ** 2).sum() for w in penalized(m))
    return loss


def ids_of(r, step):
    g = torch.Generator().manual_seed(100 * step + r)
    return torch.randint(0, cfg.vocab, (B, S), generator=g).to(device)


def ref_grads(step, micro=1):
    """Mean over ranks of the replica's gradients (fp32), accumulated over `micro` batches."""
    acc = None
    for r in range(p):
        ref.zero_grad(set_to_none=True)
        for m in range(micro):
            loss_of(ref, ids_of(r, step * 10 + m)).backward()
        gs = [q.grad.float().clone() for q in ref.parameters()]
        acc = gs if acc is None else [a + b for a, b in zip(acc, gs)]
    return [a / p for a in acc]


fails = []


def compare(tag, want):
    for (name, q), w in zip(model.named_parameters(), want):
        err = ((q.grad.float() - w).abs().max() / (w.abs().max() + 1e-6)).item()
        if err > tol:
            fails.append(f"{tag} {name}: rel err {err:.4f}")


for step in range(2):
    sinks0 = tp.CALLS["wgrad_sink"]
    ddp.zero_grad()
    loss_of(model, ids_of(rank, step * 10)).backward()
    ddp.finish()
    if device.type == "cuda" or args.sink:
        if device.type == "cuda":
            torch.cuda.synchronize()
        n_tp = 4 * cfg.layers + 2 * cfg.layers + 1  # q k v o + gate_up down per layer + LM head
        if tp.CALLS["wgrad_sink"] - sinks0 != n_tp:
            fails.append(f"step {step}: {tp.CALLS['wgrad_sink'] - sinks0} sink dW GEMMs, expected {n_tp}")
    compare(f"step {step}", ref_grads(step))
# micro-batch accumulation: no sync on the first, sync on the second (the sinks add)
ddp.zero_grad()
ddp.require_backward_grad_sync = False
loss_of(model, ids_of(rank, 50)).backward()
ddp.finish()
ddp.require_backward_grad_sync = True
loss_of(model, ids_of(rank, 51)).backward()
ddp.finish()
compare("accumulate", ref_grads(5, micro=2))
if args.measure and device.type == "cuda":
    r = measure_ddp_overlap(comm, layers=2, tokens=512, seq=256, vocab=True, iters=1, cfg=cfg, bucket_mb=1,
                            blocks_sweep=[64, 128])
    if rank == 0:
        print("measure:", r, flush=True)
    if not (r["compute_ms"] > 0 and r["overlapped_ms"] > 0 and r["comm_hidden_fraction"] is not None
            and r["deferred_ms"] > 0 and r["step_ms"] == min(r["overlapped_ms"], r["deferred_ms"])):
        fails.append(f"measure_ddp_overlap record incomplete: {r}")
bad = hc.allgather(fails)
if rank == 0:
    flat = [f"rank {r}: {m}" for r, ms in enumerate(bad) for m in ms]
    print("\n".join(flat[:30]) if flat else "llama dp OK", flush=True)
sys.exit(1 if any(bad) else 0)
