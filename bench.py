"""Flagship benchmark (driver contract).

    python bench.py --gpus N --steps K --warmup W
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

Metric (BASELINE.json): "all-reduce algbw (GB/s) @1GiB fp32 + DP4xTP2 fwd step time".

* A step = one out-of-place all-reduce (SUM) of a 1 GiB fp32 buffer through the
  framework's ``Communicator.Allreduce`` on the GPU.  Buffers come from the
  symmetric heap (``comm.empty``), the way framework users allocate
  communication buffers.  ``value`` = algbw = 1 GiB / (time per all-reduce), the
  NCCL-tests convention: a property of the whole collective, identical for every
  rank.  Per-GPU work is fixed as N grows (weak scaling).  At N = 1 the
  all-reduce is a local copy, so that number is a copy bandwidth.
* The algorithm is picked once per run, like RCCL's tuner does.  Every candidate
  runs once and is checked for an exact result (rank-valued inputs, so fp32 sums
  are exact) before it is timed.  Candidates: the hand-written two-shot kernel
  over IPC-mapped xGMI peer memory, the RCCL-send/recv multi-ring, and the RCCL
  all-reduce.  The chosen algorithm and every candidate's time are reported.
* Secondary: the DP x TP transformer-layer forward step time on MNIST-shaped
  synthetic data.  The grid is TP=2 x DP=N/2 for N >= 2 (DP4xTP2 at N = 8).

The timed region is W untimed steps, then a barrier + device sync, K steps,
and another device sync + barrier.  The time is the MAX over ranks.  Rank 0
prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--size-mb", type=int, default=1024)
    ap.add_argument("--algo", default="auto", help="auto | twoshot | oneshot | rccl | ring | rhd | reduce_bcast")
    ap.add_argument("--tp", type=int, default=0, help="TP degree of the harness step (default 2 if N>=2)")
    ap.add_argument("--batch", type=int, default=2048, help="images per DP replica for the harness step")
    ap.add_argument("--no-harness", action="store_true")
    ap.add_argument("--verbose", action="store_true")
    return ap.parse_args()


def relaunch(n: int) -> int:
    """--gpus N without a launcher: start N ranks with the framework launcher
    (child processes; this process never touches the GPU)."""
    from collective_communication_mpi_amd.launch import launch

    argv = [sys.executable, os.path.abspath(__file__)] + sys.argv[1:]
    return launch(n, argv, env_extra={"CCMPI_BENCH_CHILD": "1"})


def main() -> int:
    args = parse()
    launched = any(k in os.environ for k in ("RANK", "CCMPI_RANK", "PMI_RANK", "OMPI_COMM_WORLD_RANK"))
    if args.gpus > 1 and not launched:
        return relaunch(args.gpus)

    # a hand-written candidate that cannot complete gives up after 10 s (default 20 s):
    # the slowest legitimate 1 GiB all-reduce takes ~0.1 s, and every candidate starts
    # from a barrier, so rank skew does not count against it
    os.environ.setdefault("CCMPI_DEVICE_TIMEOUT_S", "10")
    import torch

    from collective_communication_mpi_amd import MPI, Communicator

    comm = Communicator(MPI.COMM_WORLD)
    rank, world = comm.Get_rank(), comm.Get_size()
    if world != args.gpus and rank == 0:
        print(f"[bench] warning: --gpus {args.gpus} but world size {world}", file=sys.stderr)
    local = int(os.environ.get("LOCAL_RANK", os.environ.get("CCMPI_LOCAL_RANK", "0")))
    torch.cuda.set_device(local % torch.cuda.device_count())
    dev = comm.dev
    hc = comm.comm

    def log(*a):
        if rank == 0 and args.verbose:
            print("[bench]", *a, file=sys.stderr, flush=True)

    # ------------------------------------------------------------- all-reduce
    nbytes = args.size_mb << 20
    n = nbytes // 4
    x = dev.empty(n, torch.float32)
    y = dev.empty(n, torch.float32)
    x.fill_(float(rank + 1))
    expect = float(world * (world + 1) // 2)
    torch.cuda.synchronize()

    def run(algo):
        if algo == "ring4":
            dev.allreduce(x, y, "SUM", "ring", rings=4)
        else:
            dev.allreduce(x, y, "SUM", algo)

    def valid(algo) -> bool:
        ok = 1
        try:
            y.zero_()
            torch.cuda.synchronize()
            hc.Barrier()
            run(algo)
            torch.cuda.synchronize()
            dev.check()
            ok = int(bool(torch.all(y == expect).item()))
        except Exception as e:  # noqa: BLE001 - any failure disqualifies the candidate
            log(f"candidate {algo} failed: {e}")
            ok = 0
        return bool(hc.allreduce(ok, op=MPI.MIN))

    def timed(algo, iters) -> float:
        torch.cuda.synchronize()
        hc.Barrier()
        t0 = time.perf_counter()
        for _ in range(iters):
            run(algo)
        torch.cuda.synchronize()
        hc.Barrier()
        return hc.allreduce(time.perf_counter() - t0, op=MPI.MAX) / iters

    if world == 1:
        candidates = ["twoshot"]  # single rank: the all-reduce is a device copy
    elif args.algo != "auto":
        candidates = [args.algo]
    elif dev.shared_device:  # several ranks on one GPU (CI): grid is capped, RCCL refuses
        candidates = ["twoshot", "push"]
    else:
        # RCCL first (baseline), then the hand-written two-shot at several CTA
        # budgets (per-link in-flight bytes differ on xGMI), then RCCL-P2P rings.
        candidates = ["rccl", "twoshot:128", "twoshot:256", "twoshot:512", "twoshot:1024", "push:256", "push:512", "ring4"]
    results = {}
    custom_failed = False
    for algo in candidates:
        custom = not algo.startswith(("rccl", "ring"))
        if custom and custom_failed:
            # the hand-written kernels share one flag protocol: after one of them failed
            # (and waited out the device timeout) the others are not tried
            results[algo] = None
            continue
        if not valid(algo):
            results[algo] = None
            if not algo.startswith(("rccl", "ring")):
                custom_failed = True
                dev.reset()  # a timed-out kernel leaves per-CTA epochs inconsistent
            continue
        run(algo)
        results[algo] = timed(algo, 3)
        log(f"candidate {algo}: {results[algo] * 1e3:.3f} ms")
    good = {a: t for a, t in results.items() if t}
    if not good:
        raise SystemExit("no all-reduce algorithm produced a correct result")
    best = min(good, key=good.get)

    for _ in range(args.warmup):
        run(best)
    t_step = timed(best, args.steps)
    torch.cuda.synchronize()
    final_ok = bool(torch.all(y == expect).item())
    final_ok = bool(hc.allreduce(int(final_ok), op=MPI.MIN))
    algbw = nbytes / t_step / 1e9
    busbw = algbw * (2 * (world - 1) / world) if world > 1 else 0.0

    # -------------------------------------------------------- harness step
    harness = None
    if custom_failed and results.get("rccl"):
        os.environ["CCMPI_ALLREDUCE_ALGO"] = "rccl"  # harness TP/DP collectives follow the valid path
    if not args.no_harness:
        try:
            from collective_communication_mpi_amd.models.harness import bench_forward

            tp = args.tp or (2 if world >= 2 and world % 2 == 0 else 1)
            harness = bench_forward(comm, tp=tp, batch=args.batch, steps=args.steps, warmup=args.warmup)
        except ImportError:
            harness = None

    if rank == 0:
        tp = harness["tp"] if harness else (2 if world >= 2 and world % 2 == 0 else 1)
        dp = world // tp
        out = {
            "metric": "all-reduce algbw (GB/s) @1GiB fp32 + DP4xTP2 fwd step time, 1/2/4/8 MI355X",
            "value": round(algbw, 3),
            "unit": "GB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(t_step * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "fp32",
            "data": "synthetic (rank-valued 1 GiB fp32 buffer; MNIST-shaped random images, random-init weights)",
            "config": {
                "model": "allreduce-1GiB-fp32 + MNIST-shaped TP transformer layer (768->256 qkv, 256->10 fc_o)",
                "global_batch": (harness or {}).get("global_batch"),
                "seq_len": (harness or {}).get("seq_len"),
                "parallelism": f"dp{dp}xtp{tp}" if harness else f"allreduce-world{world}",
                "allreduce_algo": best,
                "allreduce_bytes": nbytes,
                "busbw_GBps": round(busbw, 3),
                "candidates_ms": {a: (round(t * 1e3, 4) if t else None) for a, t in results.items()},
                "result_exact": final_ok,
            },
        }
        if harness:
            out["config"]["tp_fwd_step_ms"] = round(harness["fwd_ms"], 4)
            out["config"]["tp_train_step_ms"] = round(harness.get("train_ms", float("nan")), 4)
            out["config"]["harness"] = {k: v for k, v in harness.items() if k not in ("fwd_ms", "train_ms")}
        print(json.dumps(out), flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
