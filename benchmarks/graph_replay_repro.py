"""Round-3 crash repro: the DP x TP harness's HIP-graph replay after the bench's
collective candidate loop, in ONE process per rank (the old bench layout).

    GPU_MAX_HW_QUEUES=1 python -m collective_communication_mpi_amd.launch -n 8 \
        python benchmarks/graph_replay_repro.py --prefix ar,bf16,a2a,free --tp 2

``--prefix`` picks what runs before the harness: ``ar`` (1 GiB all-reduce candidates),
``bf16`` (bf16 candidates), ``a2a`` (all-to-all 64 MiB/rank), ``free`` (drop the
buffers and ``torch.cuda.empty_cache()``, as the old bench did).  The native crash
reporter (csrc/host/crash.cpp) prints where in the runtime a crash happens.
Prints ``replay OK`` on rank 0 when every replay completed.
"""
import argparse
import faulthandler
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
faulthandler.enable()

import torch  # noqa: E402

import bench  # noqa: E402
from collective_communication_mpi_amd import MPI, Communicator, _native  # noqa: E402
from collective_communication_mpi_amd.models.harness import bench_forward  # noqa: E402

_native.host().install_crash_handler(2)
ap = argparse.ArgumentParser()
ap.add_argument("--prefix", default="ar,bf16,a2a,free")
ap.add_argument("--tp", type=int, default=2)
ap.add_argument("--batch", type=int, default=2048)
ap.add_argument("--size-mb", type=int, default=1024)
ap.add_argument("--steps", type=int, default=5)
ap.add_argument("--train", type=int, default=1)
ap.add_argument("--variants", default="token:1",
                help="harness forwards to run in order, fc_o_mode:tp_chunks (bench's harness phase: "
                     "token:1,row:1,token:4); the first one also trains (--train)")
args = ap.parse_args()
prefix = [p for p in args.prefix.split(",") if p]
comm = Communicator(MPI.COMM_WORLD)
torch.cuda.set_device(int(os.environ.get("CCMPI_LOCAL_RANK", "0")) % torch.cuda.device_count())
rank = comm.Get_rank()


def say(msg):
    if rank == 0:
        print(f"[repro] {msg}", file=sys.stderr, flush=True)


if "ar" in prefix:
    bargs = bench.parse(["--gpus", str(comm.Get_size()), "--steps", "3", "--warmup", "1",
                         "--size-mb", str(args.size_mb), "--a2a-mb", "64"])
    groups = ["ar"] + [g for g in ("bf16", "a2a") if g in prefix]
    r = bench.run_collectives(comm, bargs, say, groups=tuple(groups))
    say(f"collectives {groups}: best {r['best']} {r['t_step'] * 1e3:.3f} ms")
if "free" in prefix:
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    say("freed")
say(f"harness tp={args.tp}, dev registrations={comm.dev.registrations}")
results = []
for k, v in enumerate(args.variants.split(",")):
    mode, chunks = v.split(":")
    say(f"bench_forward fc_o={mode} tp_chunks={chunks}")
    res = bench_forward(comm, tp=args.tp, batch=args.batch, steps=args.steps, warmup=2,
                        train=bool(args.train) and k == 0, fc_o_mode=mode, tp_chunks=int(chunks))
    results.append({"variant": v, "fwd_ms": round(res["fwd_ms"], 4), "hip_graph": res["hip_graph"]})
torch.cuda.synchronize()
comm.comm.Barrier()
if rank == 0:
    print(json.dumps({"prefix": prefix, "hw_queues": os.environ.get("GPU_MAX_HW_QUEUES"),
                      "graph_queues": os.environ.get("DEBUG_HIP_FORCE_GRAPH_QUEUES"), "results": results}), flush=True)
    print("replay OK", flush=True)
