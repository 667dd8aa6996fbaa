"""DP gradient all-reduce overlapped with the backward (BASELINE config 5:
"DP8 gradient all-reduce, Llama-3-8B-sized grad (~16 GB bf16) overlapped with
backward on 8xMI355X").

A synthetic backward over the whole Llama-3-8B parameter set: the LM head
(128256 x 4096), ``layers`` decoder layers (d 4096, GQA kv 1024, MLP 14336;
218 M weights per layer) and the token embedding (128256 x 4096) -- 8.03 B
weights = 16.06 GB of bf16 gradients at 32 layers, the "~16 GB" of the config.
In backward order: the LM-head gradient dW = dLogits^T H first (the first
bucket ready), then per layer the seven weight gradients dW = dY^T X, then the
embedding gradient last (a row scatter-add of the first layer's input gradient
over the token ids, the last bucket ready).  Every GEMM is the MFMA kernel
(``gemm_nt`` over the token axis, fp32 accumulate, bf16 out) writing straight
into one flat bf16 gradient buffer on the symmetric heap.  As soon as a layer's GEMMs are queued, an event hands that
layer's slice (one bucket) to a side stream (normal priority: measured better
than high priority, profiles/r2_overlap), which all-reduces it with the
framework's device all-reduce (``overlap_blocks`` CTAs) while the next
layer's GEMMs run.
Activations are kept feature-major ([features, tokens]) so every wgrad GEMM
reads K-contiguous operands, as the real backward's saved activations are.

Reports compute-only, comm-only and overlapped step times (max over ranks),
and ``comm_hidden_fraction`` = (compute + comm - overlapped) / comm.
"""
from __future__ import annotations

import time
from typing import Dict, List, Tuple

import torch

from ..ops import gemm_nt

LLAMA3_8B = {"d": 4096, "kv": 1024, "ff": 14336, "vocab": 128256}


def layer_weight_shapes(d: int, kv: int, ff: int) -> List[Tuple[int, int]]:
    """(out_features, in_features) of q, k, v, o, gate, up, down."""
    return [(d, d), (kv, d), (kv, d), (d, d), (ff, d), (ff, d), (d, ff)]


def dp_grad_overlap(comm, layers: int = 32, tokens: int = 4096, iters: int = 3, algo: str = "auto",
                    priority: int = 0, dims: Dict[str, int] = LLAMA3_8B, seed: int = 0, verbose: bool = False,
                    max_blocks: int = 0, bucket_mb: int = 0, vocab: bool = True) -> Dict:
    """``max_blocks``: CTA budget of the bucket all-reduces (0 = the group's
    ``overlap_blocks``, the budget for collectives that run beside compute).
    ``bucket_mb``: split each layer's gradient range into all-reduces of at most
    this many MiB, each launched once the layer's GEMMs are queued (0 = one
    bucket per layer, 436 MB for Llama-3-8B, and one each for the LM head and
    the embedding, 1.05 GB).  ``vocab=False`` leaves the LM head and the
    embedding out (decoder layers only)."""
    from .. import mpi as MPI

    dev = comm.dev
    hc = comm.comm
    p = comm.Get_size()
    d, kv, ff, T = dims["d"], dims["kv"], dims["ff"], tokens
    V = dims.get("vocab", 0) if vocab else 0
    shapes = layer_weight_shapes(d, kv, ff)
    per_layer = sum(a * b for a, b in shapes)
    emb = V * d  # LM head and token embedding: V x d each
    # backward order: LM head, layer L-1 .. layer 0, embedding
    n_total = per_layer * layers + 2 * emb

    def say(msg: str) -> None:
        if verbose and comm.Get_rank() == 0:
            import sys

            print(f"[dp_overlap] {msg}", file=sys.stderr, flush=True)

    # gradients in symmetric-heap blocks of at most 512 MiB (zero-copy all-reduce): one per
    # decoder layer (436 MB for Llama-3-8B) and row chunks of the LM head and embedding
    # (one 3.85 GB registration hung in hipIpcOpenMemHandle with 2 ranks on one GPU,
    # profiles/r3_dp2; ~0.5 GB blocks register fine)
    say(f"allocating {n_total * 2 / 1e9:.2f} GB of bf16 gradients (symmetric heap)")
    chunk_rows = max(1, (256 << 20) // max(d, 1))  # 512 MiB of bf16 rows
    vchunks = [(r0, min(V, r0 + chunk_rows)) for r0 in range(0, V, chunk_rows)] if V else []
    lm_g = [dev.empty((r1 - r0, d), torch.bfloat16) for r0, r1 in vchunks]
    layer_g = [dev.empty(per_layer, torch.bfloat16) for _ in range(layers)]
    emb_g = [dev.empty((r1 - r0, d), torch.bfloat16) for r0, r1 in vchunks]
    say(f"gradients registered ({len(lm_g) + len(layer_g) + len(emb_g)} heap blocks)")
    g = torch.Generator(device=dev.device).manual_seed(seed + comm.Get_rank())
    x_t = {k: (torch.randn(k, T, generator=g, device=dev.device) * 0.05).bfloat16() for k in {d, ff}}
    dy_t = {k: (torch.randn(k, T, generator=g, device=dev.device) * 0.05).bfloat16() for k in {d, kv, ff}}
    if V:
        dlogits_t = (torch.randn(V, T, generator=g, device=dev.device) * 0.05).bfloat16()  # [vocab, tokens]
        ids = torch.randint(0, V, (T,), generator=g, device=dev.device)
        dx0 = (torch.randn(T, d, generator=g, device=dev.device) * 0.05).bfloat16()  # grad of the embedded tokens
        # per embedding chunk: the token positions whose id falls in it (host-side once)
        sel = [((ids >= r0) & (ids < r1)).nonzero().flatten() for r0, r1 in vchunks]
        emb_idx = [(ids[s_] - r0, dx0[s_]) for s_, (r0, _) in zip(sel, vchunks)]
    side = torch.cuda.Stream(device=dev.device, priority=priority)
    mb = min(max_blocks or dev.overlap_blocks, getattr(dev, "overlap_cap", 1 << 30))
    events = [torch.cuda.Event() for _ in range(layers + 2)]
    # bucket length in elements, a multiple of 8 (16-B aligned bf16 buckets)
    step = None if bucket_mb <= 0 else max(8, ((bucket_mb << 20) // 2) // 8 * 8)

    def reduce_tensors(ev, ts) -> None:
        ev.record()
        side.wait_event(ev)
        with torch.cuda.stream(side):
            for t in ts:
                flat = t.view(-1)
                st = step or flat.numel()
                for a in range(0, flat.numel(), st):
                    seg = flat[a:a + st]
                    dev.allreduce(seg, seg, "SUM", algo, max_blocks=mb)

    def backward(comm_on: bool, compute_on: bool = True) -> None:
        if V:  # LM head: the first gradient of the backward
            if compute_on:
                for (r0, r1), gt in zip(vchunks, lm_g):
                    gemm_nt(dlogits_t[r0:r1], x_t[d], out=gt)
            if comm_on:
                reduce_tensors(events[layers], lm_g)
        for layer in reversed(range(layers)):
            gl = layer_g[layer]
            if compute_on:
                o = 0
                for fo, fi in shapes:
                    gemm_nt(dy_t[fo], x_t[fi], out=gl[o:o + fo * fi].view(fo, fi))
                    o += fo * fi
            if comm_on:
                reduce_tensors(events[layer], [gl])
        if V:  # token embedding: the last gradient (row scatter-add over the token ids)
            if compute_on:
                for gt, (rows, src) in zip(emb_g, emb_idx):
                    gt.zero_()
                    gt.index_add_(0, rows, src)
            if comm_on:
                reduce_tensors(events[layers + 1], emb_g)
        torch.cuda.current_stream().wait_stream(side)

    def timed(**kw) -> float:
        say(f"timing {kw} ...")
        backward(**kw)
        torch.cuda.synchronize()
        dev.check()
        hc.Barrier()
        t0 = time.perf_counter()
        for _ in range(iters):
            backward(**kw)
        torch.cuda.synchronize()
        t = hc.allreduce((time.perf_counter() - t0) / iters, op=MPI.MAX)
        if verbose and comm.Get_rank() == 0:
            import sys

            print(f"[dp_overlap] {kw}: {t * 1e3:.3f} ms", file=sys.stderr, flush=True)
        return t

    t_compute = timed(comm_on=False)
    t_comm = timed(comm_on=True, compute_on=False) if p > 1 else 0.0
    t_both = timed(comm_on=True) if p > 1 else t_compute
    dev.check()
    hidden = None if p == 1 or t_comm == 0 else max(0.0, min(1.0, (t_compute + t_comm - t_both) / t_comm))
    flops = 2 * T * (per_layer * layers + emb)  # the embedding scatter-add is not a GEMM
    gbytes = n_total * 2
    out = {"ranks": p, "layers": layers, "grad_bytes_bf16": gbytes, "tokens_per_rank": T,
           "compute_ms": round(t_compute * 1e3, 3), "comm_ms": round(t_comm * 1e3, 3),
           "overlapped_ms": round(t_both * 1e3, 3), "comm_hidden_fraction": None if hidden is None else round(hidden, 3),
           "wgrad_TFLOPs": round(flops / t_compute / 1e12, 1), "shared_gpu": dev.shared_device,
           "comm_algbw_GBps": round(gbytes / t_comm / 1e9, 2) if t_comm else None, "algo": algo,
           "bucket_ctas": mb, "params": n_total, "vocab": V,
           "buckets": sum((t.numel() + (step or t.numel()) - 1) // (step or t.numel()) for t in lm_g + layer_g + emb_g),
           "bucket_MiB": round(min(step or per_layer, per_layer) * 2 / (1 << 20), 1)}
    del lm_g, layer_g, emb_g, x_t, dy_t
    return out
