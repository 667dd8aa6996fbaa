"""BASELINE config 5 on a real backward: "DP8 gradient all-reduce, Llama-3-8B-sized grad
(~16 GB bf16) overlapped with backward on 8xMI355X".

A Llama-3-8B-shaped decoder (token embedding, ``layers`` blocks of RMSNorm -> q/k/v/o
projections + causal GQA attention -> RMSNorm -> SwiGLU MLP, final norm, LM head: 8.03 B
weights = 16.06 GB of bf16 gradients at 32 layers) built from the framework's own layers
(``ColumnParallelLinear`` / ``RowParallelLinear`` / ``ParallelSwiGLUMLP`` at TP = 1: the
hand-written MFMA GEMMs forward and backward), wrapped in ``DistributedDataParallel`` over
the DP communicator.  ``loss.backward()`` runs the whole autograd backward (dX and dW
GEMMs, attention, norms, embedding scatter); each bucket's all-reduce is launched from
the backward itself -- by the dW GEMM that completes it (gradient sinks) or by the
post-accumulate hook -- on the communication stream, and ``finish()`` joins it.

The reference's DP is sharding plus ``dp_comm`` (data/data_parallel_preprocess.py:45-59,
model/func_impl.py:61-62, README.md:177); this is the gradient synchronisation the north
star adds on that communicator.  Attention is PyTorch's SDPA (the model compute around
the collective, not a framework kernel); RoPE is left out (no effect on gradient sizes
or the GEMM work).  Random-init weights, synthetic token ids.
"""
from __future__ import annotations

import time
from dataclasses import dataclass
from typing import Dict, List, Optional

import torch
import torch.nn.functional as F

from .ddp import DistributedDataParallel
from .tensor_parallel import ColumnParallelLinear, ParallelSwiGLUMLP, RowParallelLinear


@dataclass
class LlamaConfig:
    d: int = 4096
    heads: int = 32
    kv_heads: int = 8
    ffn: int = 14336
    vocab: int = 128256
    layers: int = 32
    eps: float = 1e-5

    @property
    def head_dim(self) -> int:
        return self.d // self.heads

    def params(self, vocab: bool = True) -> int:
        d, kv = self.d, self.kv_heads * self.head_dim
        per_layer = d * d * 2 + 2 * kv * d + 3 * self.ffn * d + 2 * d
        return per_layer * self.layers + d + (2 * self.vocab * d if vocab else 0)


LLAMA3_8B = LlamaConfig()


class RMSNorm(torch.nn.Module):
    def __init__(self, d: int, eps: float, device=None, dtype=torch.bfloat16):
        super().__init__()
        self.eps = eps
        self.weight = torch.nn.Parameter(torch.ones(d, device=device, dtype=dtype))

    def forward(self, x):
        return F.rms_norm(x, (x.shape[-1],), self.weight, self.eps)


class LlamaBlock(torch.nn.Module):
    def __init__(self, cfg: LlamaConfig, tp, seed: int, device, dtype=torch.bfloat16):
        super().__init__()
        d, kv = cfg.d, cfg.kv_heads * cfg.head_dim
        self.cfg = cfg
        kw = dict(bias=False, device=device, dtype=dtype, init="device")
        self.attn_norm = RMSNorm(d, cfg.eps, device, dtype)
        self.wq = ColumnParallelLinear(d, d, tp, seed=seed, **kw)
        self.wk = ColumnParallelLinear(d, kv, tp, seed=seed + 1, **kw)
        self.wv = ColumnParallelLinear(d, kv, tp, seed=seed + 2, **kw)
        self.wo = RowParallelLinear(d, d, tp, seed=seed + 3, **kw)
        self.mlp_norm = RMSNorm(d, cfg.eps, device, dtype)
        self.mlp = ParallelSwiGLUMLP(d, cfg.ffn, tp, device=device, dtype=dtype, seed=seed + 4, init="device")

    def forward(self, x, batch: int, seq: int):
        cfg = self.cfg
        hd = cfg.head_dim
        n = self.attn_norm(x)
        q = self.wq(n).view(batch, seq, cfg.heads, hd).transpose(1, 2)
        k = self.wk(n).view(batch, seq, cfg.kv_heads, hd).transpose(1, 2)
        v = self.wv(n).view(batch, seq, cfg.kv_heads, hd).transpose(1, 2)
        rep = cfg.heads // cfg.kv_heads
        if rep > 1:  # GQA: expand the kv heads (keeps SDPA on its fused path)
            k = k.repeat_interleave(rep, dim=1)
            v = v.repeat_interleave(rep, dim=1)
        o = F.scaled_dot_product_attention(q, k, v, is_causal=True)
        o = o.transpose(1, 2).reshape(batch * seq, cfg.d)
        h = x + self.wo(o)
        return h + self.mlp(self.mlp_norm(h))


class LlamaModel(torch.nn.Module):
    """Token ids [batch, seq] -> mean next-token cross-entropy (fp32)."""

    def __init__(self, cfg: LlamaConfig, tp, device, dtype=torch.bfloat16, seed: int = 0, vocab: bool = True):
        super().__init__()
        self.cfg = cfg
        self.vocab = vocab
        if vocab:
            self.embed = torch.nn.Embedding(cfg.vocab, cfg.d, device=device, dtype=dtype)
            with torch.no_grad():
                g = torch.Generator(device=device).manual_seed(seed)
                self.embed.weight.normal_(0.0, 0.02, generator=g)
        self.blocks = torch.nn.ModuleList(LlamaBlock(cfg, tp, seed + 10 * (i + 1), device, dtype)
                                          for i in range(cfg.layers))
        self.norm = RMSNorm(cfg.d, cfg.eps, device, dtype)
        if vocab:
            self.head = ColumnParallelLinear(cfg.d, cfg.vocab, tp, bias=False, device=device, dtype=dtype,
                                             seed=seed + 7, init="device")

    def forward(self, ids, x0: Optional[torch.Tensor] = None):
        b, s = ids.shape
        x = self.embed(ids).view(b * s, self.cfg.d) if self.vocab else x0
        for blk in self.blocks:
            x = blk(x, b, s)
        x = self.norm(x)
        if not self.vocab:
            return x.float().pow(2).mean()
        logits = self.head(x)
        tgt = torch.roll(ids, -1, dims=1).reshape(-1)
        return F.cross_entropy(logits.float(), tgt)


def _self_comm(comm):
    """A one-rank communicator (this rank alone): the TP group of a pure-DP run."""
    r = comm.Get_rank()
    return comm.Split(r, r)  # reference order (key, color)


def measure_ddp_overlap(comm, layers: int = 32, tokens: int = 4096, seq: int = 2048, vocab: bool = True,
                        iters: int = 2, cfg: LlamaConfig = LLAMA3_8B, bucket_mb: Optional[int] = None,
                        blocks_sweep: List[int] = (32, 64, 128, 256), verbose: bool = False) -> Dict:
    """Compute-only, comm-only, overlapped and deferred step times (forward + backward +
    finish, max over ranks) of the Llama-3-8B-shaped model under DDP over ``comm``, and the
    signed hidden fraction ``(compute + comm - overlapped) / comm``; the bucket all-reduces'
    CTA budget swept over ``blocks_sweep`` (the best overlapped one is the record), then the
    deferred schedule (all buckets after the backward at the full budget).  ``step_ms`` is
    the faster schedule (``schedule``), both on record.  Collective: every rank calls."""
    from .. import mpi as MPI

    hc = comm.comm
    p, rank = comm.Get_size(), comm.Get_rank()
    dev = comm.dev
    device = dev.device
    seq = min(seq, tokens)
    batch = max(1, tokens // seq)
    c = LlamaConfig(**{**cfg.__dict__, "layers": layers})

    def say(msg: str) -> None:
        if verbose and rank == 0:
            import sys

            print(f"[llama_dp] {msg}", file=sys.stderr, flush=True)

    t0 = time.perf_counter()
    tp = _self_comm(comm)
    model = LlamaModel(c, tp, device, vocab=vocab)
    nparams = sum(q.numel() for q in model.parameters())
    say(f"model: {nparams / 1e9:.2f} B params, {time.perf_counter() - t0:.1f}s")
    # the schedules are timed explicitly below (overlapped per budget, then deferred)
    ddp = DistributedDataParallel(model, comm, bucket_bytes=(bucket_mb << 20) if bucket_mb else None,
                                  broadcast_params=False, schedule="overlap")
    say(f"DDP: {len(ddp.buckets)} buckets, {time.perf_counter() - t0:.1f}s")
    g = torch.Generator(device=device).manual_seed(1234 + rank)  # each DP rank its own data shard
    ids = torch.randint(0, c.vocab, (batch, seq), generator=g, device=device)
    x0 = None if vocab else (torch.randn(batch * seq, c.d, generator=g, device=device) * 0.5).bfloat16().requires_grad_()

    def step():
        ddp.zero_grad()
        loss = ddp(ids, x0)
        loss.backward()
        ddp.finish()
        return loss

    def timed(fn) -> float:
        fn()
        torch.cuda.synchronize()
        dev.check()
        hc.Barrier()
        s0 = time.perf_counter()
        for _ in range(iters):
            fn()
        torch.cuda.synchronize()
        return hc.allreduce((time.perf_counter() - s0) / iters, op=MPI.MAX)

    ddp.require_backward_grad_sync = False
    t_compute = timed(step)
    say(f"compute-only {t_compute * 1e3:.1f} ms")
    ddp.require_backward_grad_sync = True

    def hidden_of(t_c: float, t_o: float):
        # signed: negative when the overlapped step is slower than compute + comm back to back
        return None if p == 1 or t_c == 0 else (t_compute + t_c - t_o) / t_c

    # comm-only at the group's full CTA budget (max_blocks): the bound the links set, with no
    # compute beside it
    t_full = 0.0
    if p > 1:
        def allreduce_full():
            for b in ddp.buckets:
                dev.allreduce(b.buf, b.buf, "SUM", ddp.algo, max_blocks=dev.max_blocks, symmetric=True)

        t_full = timed(allreduce_full)
        say(f"comm-only at the full budget ({dev.max_blocks} CTAs) {t_full * 1e3:.1f} ms")
    # every budget: comm-only and overlapped at the SAME bucket CTA budget, so each hidden
    # fraction compares like with like; budgets above the group's overlap cap would only be
    # clamped to it (on a shared GPU: half the CUs, the deadlock bound -- DeviceComm.overlap_cap)
    cap = getattr(dev, "overlap_cap", None)
    budgets = sorted({min(mb, cap) if cap else mb for mb in blocks_sweep}) if p > 1 else [0]
    sweep, per = {}, {}
    for mb in budgets:
        ddp.max_blocks = mb or None
        t_c = timed(ddp.allreduce_all) if p > 1 else 0.0
        sweep[mb] = timed(step)
        per[mb] = {"comm_ms": round(t_c * 1e3, 2), "overlapped_ms": round(sweep[mb] * 1e3, 2),
                   "hidden": None if hidden_of(t_c, sweep[mb]) is None else round(hidden_of(t_c, sweep[mb]), 3)}
        say(f"{mb} CTAs per bucket all-reduce: comm-only {t_c * 1e3:.1f} ms, overlapped {sweep[mb] * 1e3:.1f} ms")
    best_mb = min(sweep, key=sweep.get)
    ddp.max_blocks = best_mb or None
    t_over = sweep[best_mb]
    t_comm = per[best_mb]["comm_ms"] / 1e3
    # deferred: every bucket all-reduced after the backward at the full budget (nothing
    # beside the GEMMs); the step is the faster of the two schedules -- DDP's own
    # schedule="auto" makes the same choice in a training loop
    t_def = None
    if p > 1:
        ddp.schedule = "deferred"
        t_def = timed(step)
        say(f"deferred (post-backward, {dev.max_blocks} CTAs) {t_def * 1e3:.1f} ms")
    chosen = "deferred" if (t_def is not None and t_def < t_over) else "overlap"
    ddp.schedule = chosen
    t_both = t_def if chosen == "deferred" else t_over
    loss = float(step().item())
    torch.cuda.synchronize()
    dev.check()
    hidden = hidden_of(t_comm, t_over)
    gbytes = sum(b.buf.numel() * b.buf.element_size() for b in ddp.buckets)
    nonemb = nparams - (c.vocab * c.d if vocab else 0)
    flops = 6 * nonemb * batch * seq  # fwd + bwd GEMM work (attention scores not counted)
    from .tensor_parallel import CALLS

    out = {"model": f"Llama-3-8B-shaped, {layers} layers" + ("" if vocab else ", no embedding/LM head"),
           "ranks": p, "params": nparams, "grad_bytes_bf16": gbytes, "tokens_per_rank": batch * seq,
           "seq_len": seq, "backward": "autograd (real dX + dW GEMMs, attention, norms, embedding)",
           "compute_ms": round(t_compute * 1e3, 2), "comm_ms": round(t_comm * 1e3, 2),
           "step_ms": round(t_both * 1e3, 2), "schedule": chosen,
           "overlapped_ms": round(t_over * 1e3, 2), "deferred_ms": None if t_def is None else round(t_def * 1e3, 2),
           # signed: (compute + comm - overlapped) / comm of the overlapped schedule
           "comm_hidden_fraction": None if hidden is None else round(hidden, 3),
           "comm_algbw_GBps": round(gbytes / t_comm / 1e9, 2) if t_comm else None,
           "comm_full_ms": round(t_full * 1e3, 2), "comm_full_blocks": dev.max_blocks if p > 1 else None,
           "comm_full_algbw_GBps": round(gbytes / t_full / 1e9, 2) if t_full else None,
           "per_budget": {str(k): v for k, v in per.items()},
           "step_TFLOPs_per_rank": round(flops / t_both / 1e12, 1),
           "bucket_MiB": round(max(ddp.bucket_sizes) / (1 << 20), 1), "buckets": len(ddp.buckets),
           "bucket_ctas": best_mb, "bucket_ctas_sweep_ms": {str(k): round(v * 1e3, 2) for k, v in sweep.items()},
           "grad_sink_gemms": CALLS.get("wgrad_sink", 0), "shared_gpu": dev.shared_device,
           "loss": round(loss, 4), "setup_s": round(time.perf_counter() - t0, 1)}
    del ddp, model
    torch.cuda.empty_cache()
    return out
