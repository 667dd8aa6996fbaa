"""Training / benchmarking harness for the DP x TP MNIST transformer layer.

    scripts/mpirun -n 2 python -m collective_communication_mpi_amd.models.harness --tp 2 --steps 20
    torchrun --nproc-per-node 8 -m collective_communication_mpi_amd.models.harness --tp 2 --steps 100

``bench_forward`` is what ``bench.py`` reports as the DP x TP forward step time:
the forward pass (patchify, embedding GEMM, QKV GEMM, attention, fc_o GEMM,
TP all-reduce, pooling) captured once into a HIP graph and replayed, timed over
K replays between barriers (max over ranks).  The full training step
(forward + backward + bucketed DP all-reduce + fused AdamW) is timed eagerly.
"""
from __future__ import annotations

import argparse
import os
import sys
import time

import numpy as np
import torch

from .. import device as _device
from ..data.preprocess import synthetic_mnist
from ..utils import checkpoint as ckpt
from .mnist_tp import LayerConfig, MnistTPLayer, local_batch


def _hc(comm):
    return comm.comm if hasattr(comm, "comm") else comm


def _sync_barrier(comm):
    torch.cuda.synchronize()
    _hc(comm).Barrier()


def build(comm, tp: int, batch: int, **kw):
    world = comm.Get_size()
    if "fwd_chunks" not in kw and os.environ.get("CCMPI_FWD_CHUNKS"):
        kw["fwd_chunks"] = int(os.environ["CCMPI_FWD_CHUNKS"])
    cfg = LayerConfig(batch=batch, tp=tp, dp=world // tp, **kw)
    layer = MnistTPLayer(comm, cfg)
    x_all, y_all = synthetic_mnist(cfg.batch * cfg.dp * 2, seed=cfg.seed)
    return cfg, layer, x_all, y_all


def train_step(layer: MnistTPLayer, cfg: LayerConfig, xb, yb):
    logits = layer.forward_images(xb, xb.shape[0])  # patchify + forward (cfg.fwd_chunks streams)
    layer.zero_grad()
    if layer._fused_fc_o() or (cfg.fc_o_mode == "row" and cfg.tp > 1) or \
            (cfg.fc_o_mode == "token" and layer._fused_fc_o_bwd()):
        loss = layer.loss_and_grad_fused(yb, cfg.batch * cfg.dp)  # one kernel: loss, dZ, d o_b
        layer.backward(None)
    else:
        loss, dlogits = layer.loss_and_grad(logits, yb, cfg.batch * cfg.dp)
        layer.backward(dlogits)
    layer.step()
    return loss


class GraphedTrainStep:
    """Whole training steps (patchify + forward, fused loss head, backward with its TP / DP
    collectives, fused AdamW) captured into HIP graphs and replayed: no per-kernel host
    launch, which the eager step pays ~10 times over at these kernel sizes.

    Two graphs, replayed alternately: the backward's split-K weight-gradient accumulator is a
    double buffer whose parity flips every step (one half is accumulated while the kernel
    zeroes the other), and a graph freezes the parity it was captured with.  The AdamW step
    count comes from the device counter (``FlatParams.device_step``), so replays apply the
    right bias corrections; ``close()`` syncs the host count back.  Capture happens after
    eager steps have allocated every buffer."""

    def __init__(self, layer: MnistTPLayer, cfg: LayerConfig, xb, yb):
        self.layer = layer
        layer.flat.device_step()
        torch.cuda.synchronize()
        layer.graph_step = True
        self.graphs = []
        try:
            for _ in range(2):
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    self.loss = train_step(layer, cfg, xb, yb)
                self.graphs.append(g)
        finally:
            layer.graph_step = False
        self.i = 0

    def replay(self):
        self.graphs[self.i].replay()
        self.i ^= 1
        return self.loss

    def close(self) -> int:
        torch.cuda.synchronize()
        return self.layer.flat.sync_step()


class TrainPlan:
    """Whole training steps as recorded launch plans (``MnistTPLayer.forward_plan``'s
    recorder over a full ``train_step``): two recordings, re-issued alternately (the split-K
    accumulator parity, as in ``GraphedTrainStep``), AdamW on the device step counter.
    Only where the step is all-native: TP = 1 and DP = 1 (the TP / DP paths run torch ops
    and other groups' collectives); ``available`` says so before anything runs."""

    @staticmethod
    def available(layer: MnistTPLayer, cfg: LayerConfig) -> bool:
        return (layer.tp_dev is None and layer.buckets.dp is None and cfg.fc_o_mode == "token"
                and layer._fuses_qkv(cfg.batch) and int(cfg.fwd_chunks) <= 1)

    def __init__(self, layer: MnistTPLayer, cfg: LayerConfig, xb, yb):
        from .mnist_tp import LaunchPlan, _LaunchRecorder

        self.layer = layer
        layer.flat.device_step()
        torch.cuda.synchronize()
        layer.graph_step = True
        self.plans = []
        try:
            for _ in range(2):
                rec = _LaunchRecorder(None)
                with rec.active(layer):
                    loss = train_step(layer, cfg, xb, yb)
                if rec.allocated:
                    raise RuntimeError("TrainPlan: the recorded step allocated device memory (a temporary "
                                       "whose pointer a recorded call may hold): not replayable")
                self.plans.append(LaunchPlan(rec.calls, loss))
        finally:
            layer.graph_step = False
        self.i = 0

    def replay(self):
        out = self.plans[self.i]()
        self.i ^= 1
        return out

    def close(self) -> int:
        torch.cuda.synchronize()
        return self.layer.flat.sync_step()


def train_graph_hazard(cfg: LayerConfig, layer: MnistTPLayer):
    """Why the training step must not be graph-captured here, or None: the forward's
    multi-stream hazard, or the DP bucket all-reduce's side stream with few hardware queues
    (the same HIP parallel-stream bug, ``multi_stream_graph_hazard``)."""
    h = multi_stream_graph_hazard(cfg, layer)
    if h:
        return h
    try:
        queues = int(os.environ.get("GPU_MAX_HW_QUEUES", "4"))
    except ValueError:
        queues = 4
    if layer.buckets.stream is not None and os.environ.get("CCMPI_FORCE_GRAPH") != "1":
        # (a multi-stream capture: with few hardware queues the HIP parallel-stream bug above;
        # with enough, still the one capture shape the N = 8 driver run would exercise first --
        # and the replay measured no faster than the GPU-bound eager step at N = 1)
        return f"DP bucket side stream (GPU_MAX_HW_QUEUES={queues}): training step timed eagerly"
    return None


def multi_stream_graph_hazard(cfg: LayerConfig, layer: MnistTPLayer):
    """Why a HIP graph of this forward must not be captured here, or None.

    HIP runtime bug (torch's ROCm 7.0 libamdhip64, root-caused in profiles/r4_bisect): a
    graph with parallel branches (a forward forked over several streams: the token fc_o's
    side-stream TP all-reduce pipeline, ``tp_chunks > 1``, or ``fwd_chunks > 1``) gets
    per-branch "parallel streams" at launch; with few hardware queues per process
    (``GPU_MAX_HW_QUEUES`` 1-2, the 8-ranks-on-one-GPU dry run) creating them fails
    ("[hipGraph] Failed to create parallel stream!"), the error is dropped, and the
    stream-assignment loop then reads past the short stream pool: host SIGSEGV inside
    hipGraphLaunch on every rank.  Single-stream graphs are not affected.  Such forwards
    are timed eagerly instead (``CCMPI_FORCE_GRAPH=1`` captures anyway)."""
    branches = 1
    if cfg.fc_o_mode == "token" and layer.tp_dev is not None and layer._token_chunks(cfg.batch) > 1:
        branches = 2
    if int(cfg.fwd_chunks) > 1:
        branches = max(branches, int(cfg.fwd_chunks))
    try:
        queues = int(os.environ.get("GPU_MAX_HW_QUEUES", "4"))
    except ValueError:
        queues = 4
    if branches > 1 and queues < 4 and os.environ.get("CCMPI_FORCE_GRAPH") != "1":
        return (f"{branches}-stream forward with GPU_MAX_HW_QUEUES={queues}: HIP graph launch would crash "
                "(short parallel-stream pool), timed eagerly")
    return None


def bench_forward(comm, tp: int = 2, batch: int = 2048, steps: int = 20, warmup: int = 5, graph: bool = True,
                  train: bool = True, **layer_kw):
    from .. import mpi as MPI

    hc = _hc(comm)
    rank = comm.Get_rank()
    cfg, layer, x_all, y_all = build(comm, tp, batch, **layer_kw)
    xb, yb = local_batch(cfg, x_all, y_all, 0, rank, layer.device)

    def fwd():  # inference forward: no activations kept for a backward
        return layer.forward_images(xb, cfg.batch, save=False)

    verbose = os.environ.get("CCMPI_HARNESS_VERBOSE") == "1"

    def say(msg):
        if verbose:
            print(f"[harness rank {rank}] {msg}", file=sys.stderr, flush=True)

    for _ in range(3):
        fwd()
    torch.cuda.synchronize()
    say("eager forward ok")
    used_graph = False
    g = None
    hazard = multi_stream_graph_hazard(cfg, layer) if graph else None
    if (graph and not hazard and _device.SHARED_GPU_IN_PROCESS
            and "1" not in (os.environ.get("CCMPI_FORCE_GRAPH"), os.environ.get("CCMPI_SHARED_GRAPH"))):
        # ranks sharing one GPU (the dry run): their graph replays serialise on the one hardware
        # queue each -- 0.8-15 ms against 0.22 ms for the launch plan (profiles/r6_bind)
        hazard = "ranks share one GPU: HIP graph replays serialise, not captured (CCMPI_SHARED_GRAPH=1 to capture)"
    if hazard:
        say(hazard)
    if graph and not hazard and os.environ.get("CCMPI_NO_GRAPH") != "1":
        try:
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                fwd()
            torch.cuda.current_stream().wait_stream(s)
            torch.cuda.synchronize()
            _sync_barrier(comm)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                fwd()
            used_graph = True
            say("graph captured")
        except Exception as e:  # noqa: BLE001 - fall back to eager, reported in the result
            if rank == 0:
                print(f"[harness] graph capture failed, timing eager: {e}", file=sys.stderr)
            g = None
    run = g.replay if g is not None else fwd
    for _ in range(warmup):
        run()
    _sync_barrier(comm)
    t0 = time.perf_counter()
    for _ in range(steps):
        run()
    torch.cuda.synchronize()
    hc.Barrier()
    fwd_s = hc.allreduce(time.perf_counter() - t0, op=MPI.MAX) / steps
    say(f"timed forward {fwd_s * 1e3:.3f} ms")
    fwd_eager_s = None
    if g is not None:
        # the same forward launched eagerly: with two or three kernels per step the host can
        # stay ahead of the GPU, and a graph replay pays its own launch cost per step -- the
        # step time is the faster way of running it on this node (both on record)
        for _ in range(warmup):
            fwd()
        _sync_barrier(comm)
        t0 = time.perf_counter()
        for _ in range(steps):
            fwd()
        torch.cuda.synchronize()
        hc.Barrier()
        fwd_eager_s = hc.allreduce(time.perf_counter() - t0, op=MPI.MAX) / steps
        say(f"timed eager forward {fwd_eager_s * 1e3:.3f} ms")
    fwd_graph_s = fwd_s if g is not None else None
    fwd_timed = "graph" if g is not None else "eager"
    if fwd_eager_s is not None and fwd_eager_s < fwd_s:
        fwd_s, fwd_timed = fwd_eager_s, "eager"
    # the launch plan: the forward's native launches recorded once, re-issued from a loop
    # (MnistTPLayer.forward_plan; None where the forward is not all-native -- the same on
    # every rank, so the collective recording forward runs everywhere or nowhere)
    fwd_plan_s = None
    plan = layer.forward_plan(xb, cfg.batch) if os.environ.get("CCMPI_NO_PLAN") != "1" else None
    if plan is not None:
        for _ in range(warmup):
            plan()
        _sync_barrier(comm)
        t0 = time.perf_counter()
        for _ in range(steps):
            plan()
        torch.cuda.synchronize()
        hc.Barrier()
        fwd_plan_s = hc.allreduce(time.perf_counter() - t0, op=MPI.MAX) / steps
        say(f"timed launch-plan forward {fwd_plan_s * 1e3:.3f} ms")
        if fwd_plan_s < fwd_s:
            fwd_s, fwd_timed = fwd_plan_s, "plan"
    # the same with the weight fold pipelined into the fused kernel's tail (each call folds the
    # next call's W_eff from the current weights; no fold launch)
    fwd_pipe_s = None
    pplan = layer.forward_plan_pipelined(xb, cfg.batch) if plan is not None else None
    if pplan is not None:
        for _ in range(warmup):
            pplan()
        _sync_barrier(comm)
        t0 = time.perf_counter()
        for _ in range(steps):
            pplan()
        torch.cuda.synchronize()
        hc.Barrier()
        fwd_pipe_s = hc.allreduce(time.perf_counter() - t0, op=MPI.MAX) / steps
        say(f"timed pipelined-fold launch-plan forward {fwd_pipe_s * 1e3:.3f} ms")
        if fwd_pipe_s < fwd_s:
            fwd_s, fwd_timed = fwd_pipe_s, "plan_pipelined_fold"
    # hip_graph: a graph was captured and replayed; fwd_timed: which launch mode fwd_ms is
    # (graph replay, eager forward_images, or the recorded launch plan)
    fwd_modes = {"fwd_timed": fwd_timed}
    if fwd_graph_s is not None:
        fwd_modes["fwd_ms_graph"] = round(fwd_graph_s * 1e3, 4)
    if fwd_eager_s is not None:
        fwd_modes["fwd_ms_eager"] = round(fwd_eager_s * 1e3, 4)
    if fwd_plan_s is not None:
        fwd_modes["fwd_ms_plan"] = round(fwd_plan_s * 1e3, 4)
    if fwd_pipe_s is not None:
        fwd_modes["fwd_ms_plan_pipelined_fold"] = round(fwd_pipe_s * 1e3, 4)
    form = getattr(layer, "_zt_form", None)  # the fused per-token fc_o's TP form, if it ran
    if not train:
        return {"tp": cfg.tp, "dp": cfg.dp, "fwd_ms": fwd_s * 1e3, "hip_graph": used_graph, **fwd_modes,
                "fc_o_mode": cfg.fc_o_mode,
                "tp_chunks": cfg.tp_chunks, "tokens_per_step": cfg.batch * cfg.dp * cfg.seq,
                **({"fc_o_tp_form": form} if form else {}), **({"graph_skipped": hazard} if hazard else {})}
    # training step: eager, then (where safe) replayed from HIP graphs of whole steps
    for _ in range(2):
        train_step(layer, cfg, xb, yb)
    _sync_barrier(comm)
    t0 = time.perf_counter()
    n_train = max(3, steps // 2)
    loss = None
    for i in range(n_train):
        loss = train_step(layer, cfg, xb, yb)
    torch.cuda.synchronize()
    hc.Barrier()
    train_eager_s = hc.allreduce(time.perf_counter() - t0, op=MPI.MAX) / n_train
    train_s, train_graph, train_graph_s = train_eager_s, False, None
    train_timed = "eager"
    t_hazard = train_graph_hazard(cfg, layer) if graph else "graph disabled"
    if t_hazard is None and os.environ.get("CCMPI_NO_GRAPH") != "1":
        gts = None
        try:
            _sync_barrier(comm)
            gts = GraphedTrainStep(layer, cfg, xb, yb)
            ok = 1
        except Exception as e:  # noqa: BLE001 - fall back to the eager number, reported
            ok = 0
            if rank == 0:
                print(f"[harness] training-step graph capture failed, eager number kept: {e}", file=sys.stderr)
        if hc.allreduce(ok, op=MPI.MIN) and gts is not None:
            for _ in range(2):
                gts.replay()
            _sync_barrier(comm)
            t0 = time.perf_counter()
            for i in range(n_train):
                loss = gts.replay()
            torch.cuda.synchronize()
            hc.Barrier()
            graph_s = hc.allreduce(time.perf_counter() - t0, op=MPI.MAX) / n_train
            gts.close()
            train_graph_s = graph_s
            # the step time is the faster way of running the same step on this node (eager is
            # GPU-bound already at the default batch: the host enqueues ahead of the kernels,
            # and a replay adds its launch cost -- measured 0.118 eager vs 0.125 ms graph)
            if graph_s < train_eager_s:
                train_s, train_graph = graph_s, True
                train_timed = "graph"
            say(f"timed graph train step {graph_s * 1e3:.3f} ms (eager {train_eager_s * 1e3:.3f})")
    train_plan_s = None
    tp_ = None
    if TrainPlan.available(layer, cfg) and os.environ.get("CCMPI_NO_PLAN") != "1":
        try:
            tp_ = TrainPlan(layer, cfg, xb, yb)
        except RuntimeError as e:
            say(str(e))
    if tp_ is not None:
        for _ in range(2):
            tp_.replay()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(n_train):
            loss = tp_.replay()
        torch.cuda.synchronize()
        train_plan_s = time.perf_counter() - t0
        train_plan_s = hc.allreduce(train_plan_s, op=MPI.MAX) / n_train
        tp_.close()
        say(f"timed launch-plan train step {train_plan_s * 1e3:.3f} ms")
        if train_plan_s < train_s:
            train_s, train_graph = train_plan_s, False
            train_timed = "plan"
    loss_v = hc.allreduce(float(loss.item()), op=MPI.SUM) / cfg.tp  # sum over DP of per-replica shares
    return {"tp": cfg.tp, "dp": cfg.dp, "fwd_ms": fwd_s * 1e3, **fwd_modes, "train_ms": train_s * 1e3,
            "train_ms_eager": train_eager_s * 1e3, "train_hip_graph": train_graph, "train_timed": train_timed,
            **({"train_ms_graph": round(train_graph_s * 1e3, 4)} if train_graph_s is not None else {}),
            **({"train_ms_plan": round(train_plan_s * 1e3, 4)} if train_plan_s is not None else {}),
            **({"train_graph_skipped": t_hazard} if (t_hazard and graph) else {}),
            "global_batch": cfg.batch * cfg.dp, "seq_len": cfg.seq, "tokens_per_step": cfg.batch * cfg.dp * cfg.seq,
            "hip_graph": used_graph, "fc_o_mode": cfg.fc_o_mode, **({"fc_o_tp_form": form} if form else {}),
            "fwd_saves_activations": False, "loss": round(loss_v, 5)}


def fc_o_forms_agree(comm, tp: int, batch: int) -> dict:
    """Collective: one forward of the per-token fc_o in both TP forms ("plain": kernel +
    all-reduce of z + ordered token mean; "push": kernel pushes row blocks into the owners'
    inboxes, the owners reduce them to the sequences' logits and fan those out) on the same
    input; the logits (and z, where both forms keep it) must be bitwise equal on every rank.
    Returns {"equal": bool, "max_abs_diff": float}."""
    from .. import mpi as MPI

    hc = _hc(comm)
    cfg, layer, x_all, y_all = build(comm, tp, batch, fc_o_mode="token", tp_fc_o_form="plain")
    xb, _ = local_batch(cfg, x_all, y_all, 0, comm.Get_rank(), layer.device)
    out = {}
    for form in ("plain", "push"):
        layer.cfg.tp_fc_o_form = form
        logits = layer.forward_images(xb, cfg.batch, save=False)
        torch.cuda.synchronize()
        z = layer._zt
        out[form] = (None if z is None else z.clone(), logits.clone(), layer._zt_form)
    zp, lp, fp = out["plain"]
    zq, lq, fq = out["push"]
    z_eq = zp is None or zq is None or torch.equal(zp, zq)
    eq = int(fp == "plain" and fq == "push" and z_eq and torch.equal(lp, lq))
    diff = float((lp - lq).abs().max().item())
    return {"equal": bool(hc.allreduce(eq, op=MPI.MIN)), "max_abs_diff": hc.allreduce(diff, op=MPI.MAX)}


def smoke_step(comm) -> None:
    """One tiny forward + backward + optimizer step (driver smoke)."""
    tp = 2 if comm.Get_size() % 2 == 0 and comm.Get_size() > 1 else 1
    cfg, layer, x_all, y_all = build(comm, tp, batch=64)
    xb, yb = local_batch(cfg, x_all, y_all, 0, comm.Get_rank(), layer.device)
    loss = train_step(layer, cfg, xb, yb)
    torch.cuda.synchronize()
    assert torch.isfinite(loss).item(), "non-finite loss"
    assert torch.isfinite(layer.flat.g).all().item(), "non-finite gradients"


def main(argv=None) -> int:
    from .. import MPI, Communicator

    ap = argparse.ArgumentParser()
    ap.add_argument("--tp", type=int, default=1)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--lr", type=float, default=2e-3)
    ap.add_argument("--fc-o-mode", default="row", choices=["row", "token", "naive"])
    ap.add_argument("--tp-chunks", type=int, default=1)
    ap.add_argument("--log", default="")
    ap.add_argument("--ckpt", default="", help="checkpoint directory (sharded, safetensors)")
    ap.add_argument("--save-every", type=int, default=0, help="save every K steps (and at the end)")
    ap.add_argument("--resume", action="store_true", help="continue from --ckpt if it holds a checkpoint")
    args = ap.parse_args(argv)
    comm = Communicator(MPI.COMM_WORLD)
    local = int(os.environ.get("LOCAL_RANK", os.environ.get("CCMPI_LOCAL_RANK", "0")))
    torch.cuda.set_device(local % torch.cuda.device_count())
    cfg, layer, x_all, y_all = build(comm, args.tp, args.batch, lr=args.lr, fc_o_mode=args.fc_o_mode,
                                     tp_chunks=args.tp_chunks)
    hc = _hc(comm)
    losses = []
    start = 0
    if args.resume and args.ckpt and ckpt.latest(args.ckpt):
        start = ckpt.load_sharded(args.ckpt, layer.flat, comm, layer.tp_idx, cfg.tp)["step"]
        if comm.Get_rank() == 0:
            print(f"resumed from {args.ckpt} at step {start}", flush=True)

    def save():
        ckpt.save_sharded(args.ckpt, layer.flat, comm, layer.tp_idx, layer.dp_idx, cfg.tp, cfg.dp,
                          meta={"batch": cfg.batch, "lr": cfg.lr, "fc_o_mode": cfg.fc_o_mode})

    for step in range(start, args.steps):
        # the data position is a function of the step, so a resumed run sees the same batches
        xb, yb = local_batch(cfg, x_all, y_all, step, comm.Get_rank(), layer.device)
        loss = train_step(layer, cfg, xb, yb)
        lv = hc.allreduce(float(loss.item()), op=MPI.SUM) / cfg.tp
        losses.append(lv)
        if comm.Get_rank() == 0:
            print(f"step {step} loss {lv:.5f}", flush=True)
        if args.ckpt and args.save_every and (step + 1) % args.save_every == 0:
            save()
    if args.ckpt and args.save_every:
        save()
    if args.log and comm.Get_rank() == 0:
        np.save(args.log, np.array(losses))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
