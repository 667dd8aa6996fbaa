"""DP x TP transformer layer on MNIST-shaped data: the training harness the
reference assumes but does not ship (README.md:173-181: "transformer compute,
training loop and MNIST data were taken care of"; the layer dims come from its
tests: fc_q/k/v 768 -> 256 column-parallel, fc_o 256 -> 10, test_get_info.py:68-69,152-153).

Model (per image): 28x28 -> 16 patches of 7x7 (49 px) -> patch embedding
49 -> 768 (+ bias + learned position) -> fused QKV projection
768 -> 3x256 (4 heads x 64) -> softmax attention over the 16 patches ->
fc_o 256 -> 10 -> mean over patches -> cross-entropy.

Parallelism: mp-major 2-D grid from ``get_info`` (rank = dp_idx * tp + tp_idx).
* fc_q/k/v are column-parallel: TP rank t owns heads [t*H/tp, (t+1)*H/tp), i.e.
  rows of the fused QKV weight; attention is local to a rank's heads.
* fc_o is row-parallel (``fc_o_mode="row"``, default): each rank multiplies its
  local attention output by its input-dim shard of W_o, and ONE TP all-reduce
  (hand-written device kernel, symmetric buffers, graph-capturable) sums the
  partial outputs.  Because fc_o and the mean over patches are both linear,
  the attention kernel emits the patch-mean of its output and fc_o runs on B
  rows instead of B*S: the fc_o GEMMs and the TP all-reduce shrink 16x.  ``fc_o_mode="naive"`` runs the reference's collects instead
  (model/func_impl.py:76-187): all-gather the input, out-sharded fc_o, all-gather
  the output; backward slices the output gradient and reduce-scatters grad_x.
* the embedding input gradient is TP-partial and is all-reduced (Megatron's
  "f" operator) so replicated parameters get identical gradients on every TP rank.
* DP: gradients in a flat fp32 buffer on the DP group's symmetric heap,
  three buckets in backward order, all-reduced on a side stream while the
  remaining backward GEMMs run (parallel/dp.py).

All GEMMs are the hand-written MFMA kernels (ops.gemm_nt forward / input
gradients, ops.gemm_tn weight gradients); attention is the fused short-sequence
kernel; the optimizer is one fused AdamW pass.  Fusions that remove whole passes:

* the patchify kernel appends a constant-1 column and a one-hot position
  column block to every token row, so the embedding bias and the learned
  position embedding are columns of W_emb: the embedding is ONE GEMM (no bias
  add, no position add) and their gradients come out of the W_emb gradient GEMM;
* the attention backward kernel accumulates the QKV bias gradient (column sums
  of dQ/dK/dV) in-kernel;
* with TP > 1 the embedding needs only the TP-sum of its *weight* gradient
  (d_model x 72 fp32, 221 KB), not an all-reduce of the TP-partial activation
  gradient dH (tokens x d_model): W_emb's gradient is linear in dH and the
  embedding input needs no gradient;
* both weight gradients of the embedding -> QKV chain come from ONE token-length
  contraction A = dQKV^T . Xp (3hd x 72): dW_emb = W_qkv^T A and, because
  h = Xp W_emb^T, dW_qkv = dQKV^T h = A W_emb^T (``qkv_grad="reassoc"``).  The
  840-column dQKV^T . [h | xp] GEMM (65 us) becomes a 72-column one (~20 us) plus
  one fp32 kernel for both weight-sized products (csrc/device/wgrad.hip), which
  also zeroes the next step's A buffer (the split-K GEMM accumulates into it);
* the forward folds the same chain (``fold_emb``): h feeds nothing but the QKV
  projection, so qkv = Xp . W_eff^T + b with W_eff = W_qkv W_emb (3hd x 72, one
  fp32 kernel per forward, 42 MFLOP).  The 32768 x 768 x 768 QKV GEMM (54 us)
  and the 32768 x 768 x 72 embedding GEMM become ONE 72-deep GEMM; h (50 MB)
  is neither written nor read.
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass
from typing import Optional

import numpy as np
import torch

from .. import _native
from ..ops import gemm_nt, gemm_tn, transpose
from ..parallel.dp import FlatParams, GradBuckets
from ..parallel.layout import device_group_for, get_info, naive_collect_backward_output, naive_collect_backward_x, \
    naive_collect_forward_input, naive_collect_forward_output


@dataclass
class LayerConfig:
    d_model: int = 768
    d_attn: int = 256
    n_heads: int = 4
    n_classes: int = 10
    img: int = 28
    patch: int = 7
    out_pad: int = 16        # fc_o output rows padded to 16 (MFMA-friendly K for dX = dZ . W_o)
    batch: int = 2048        # images per DP replica
    tp: int = 1
    dp: int = 1
    # "row": Megatron row-parallel, pooled first (B rows, one B x 16 all-reduce);
    # "token": row-parallel per token, as model/func_impl.py:94-109 shapes it -- the TP
    #   all-reduce moves B*S x 16 partial outputs, cut into tp_chunks row blocks whose
    #   all-reduces run on a side stream under the next block's fc_o GEMM;
    # "naive": the reference collects (all-gather in, out-sharded fc_o, all-gather out)
    fc_o_mode: str = "row"
    # fc_o_mode="token": row blocks of the attention -> fc_o -> TP all-reduce pipeline.  1 by
    # default: measured with 2 ranks sharing one GPU, 2/4/8 blocks cost 0.47/0.83/1.98 ms
    # vs 0.22 ms unpipelined (profiles/r2_overlap) -- a 2 MB all-reduce per step is
    # latency-bound, and per-block attention is too short to hide it
    tp_chunks: int = 1
    lr: float = 1e-3
    weight_decay: float = 0.0
    seed: int = 1234
    dp_algo: str = "auto"
    overlap: bool = True
    plain_gemm: str = "own"  # backward dH = dQKV . W_qkv: "own" (MFMA kernel, W^T kept by AdamW) | "hipblaslt"
    emb_grad: str = "reassoc"  # "reassoc": dW_emb = W_qkv^T (dQKV^T Xp), no dH; "dh": materialize dH first
    # with emb_grad="reassoc": "reassoc": dW_qkv = (dQKV^T Xp) W_emb^T (h is not read in backward);
    # "direct": dW_qkv = dQKV^T h (one TN GEMM over the fused [h | xp] rows)
    qkv_grad: str = "reassoc"
    fuse_fc_o: bool = True   # pooled fc_o inside the attention kernels (fwd logits, bwd dpool) instead of GEMMs
    fwd_chunks: int = 1      # forward_images: row blocks run on that many HIP streams (1 = one stream)
    # forward: qkv = Xp . (W_qkv W_emb)^T + b -- h is never formed (needs the re-associated
    # backward, which does not read h); False: h = Xp . W_emb^T, then qkv = h . W_qkv^T + b
    fold_emb: bool = True
    # fc_o_mode="token" with tp_chunks = 1: the per-token fc_o runs inside the attention kernel
    # (csrc/device/attn_mfma.hip: z = O . W_o^T on the MFMA, heads summed in the workgroup; no
    # attention output tensor, no fc_o GEMM), and its TP sum takes one of two forms:
    # * "plain": the kernel writes this rank's partial z, then one TP all-reduce of z;
    # * "push":  the kernel stores row block j of its partial straight into TP rank j's inbox
    #   slot (posted writes over xGMI while the other sequences still compute), then the
    #   inbox-to-local two-shot (DeviceComm::inbox_to_local) -- the all-reduce's reduce-scatter
    #   traffic is overlapped with the attention.  Bitwise equal to "plain" (both sum the
    #   ranks' partials in rank order, in fp32).
    # * "auto" (default; CCMPI_TP_FC_O_FORM overrides): "push" when every TP rank owns its
    #   GPU, "plain" when the ranks share one (the pushes then only compete for the same HBM).
    tp_fc_o_form: str = ""
    # token mode: the QKV projection inside the attention kernel (k_qkv_attn16_fwd) -- the
    # B*S x 3hd qkv tensor is neither written (inference) nor read back, and the QKV GEMM goes
    fuse_qkv: bool = True
    @property
    def seq(self) -> int:
        return (self.img // self.patch) ** 2

    @property
    def head_dim(self) -> int:
        return self.d_attn // self.n_heads

    @property
    def pixels(self) -> int:
        return self.patch * self.patch

    @property
    def kp(self) -> int:
        """Embedding GEMM K: pixels + bias column + one-hot positions, rounded to 8."""
        return (self.pixels + 1 + self.seq + 7) // 8 * 8


def patchify(x: torch.Tensor, cfg: LayerConfig, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """(B, 784) fp32 -> (B*16, kp) bf16 token rows: 49 pixels | 1 | one-hot(position) | 0 pad."""
    B = x.shape[0]
    if out is None:
        out = torch.empty(B * cfg.seq, cfg.kp, dtype=torch.bfloat16, device=x.device)
    if out.shape != (B * cfg.seq, cfg.kp) or out.stride(1) != 1:
        raise ValueError("patchify: out must be [B*S, kp] with unit column stride")
    x = x.contiguous().float()
    _native.device().patchify(x.data_ptr(), out.data_ptr(), B, cfg.img, cfg.patch, cfg.kp,
                              torch.cuda.current_stream(x.device).cuda_stream, out.stride(0))
    return out


def full_init(cfg: LayerConfig):
    """Unsharded fp32 weights from a seeded CPU generator (identical on all ranks).
    W_emb columns: [pixels | bias | position one-hot | pad]."""
    g = torch.Generator().manual_seed(cfg.seed)
    d, a, pp = cfg.d_model, cfg.d_attn, cfg.pixels
    emb = torch.zeros(d, cfg.kp)
    emb[:, :pp] = torch.randn(d, pp, generator=g) / math.sqrt(pp)
    emb[:, pp] = 0.0                                                    # bias
    emb[:, pp + 1:pp + 1 + cfg.seq] = (torch.randn(cfg.seq, d, generator=g) * 0.02).T  # positions
    w = {
        "emb_w": emb,
        "q_w": torch.randn(a, d, generator=g) / math.sqrt(d),
        "k_w": torch.randn(a, d, generator=g) / math.sqrt(d),
        "v_w": torch.randn(a, d, generator=g) / math.sqrt(d),
        "q_b": torch.zeros(a), "k_b": torch.zeros(a), "v_b": torch.zeros(a),
        "o_w": torch.randn(cfg.n_classes, a, generator=g) / math.sqrt(a),
        "o_b": torch.zeros(cfg.n_classes),
    }
    return w


class LaunchPlan:
    """Recorded native launches of one step (``MnistTPLayer.forward_plan``); ``plan()``
    re-issues them on the streams they were recorded with and returns the logits view."""

    def __init__(self, calls, logits):
        self.calls = calls
        self.logits = logits

    def __call__(self):
        for fn, a, k in self.calls:
            fn(*a, **k)
        return self.logits

    def names(self):
        return [getattr(fn, "__name__", str(fn)) for fn, _, _ in self.calls]


class PipelinedFoldPlan:
    """Two launch plans of the image-mode fused forward used alternately (``MnistTPLayer.
    forward_plan_pipelined``): plan k reads W_eff buffer k and its kernel tail folds buffer
    k ^ 1 for the next call.  A call whose weights changed since the previous one (or the
    first call) folds its own buffer first with the fold kernel."""

    def __init__(self, layer, plans, w):
        self.layer, self.plans, self.w = layer, plans, w
        self.k = 0
        self.stamp = None

    def _stamp(self):
        f = self.layer.flat
        return (f.step_count, f.p32._version)

    def invalidate(self) -> None:
        self.stamp = None

    def names(self):
        return self.plans[0].names()

    def __call__(self) -> torch.Tensor:
        st = self._stamp()
        if st != self.stamp:
            self.layer._fold_into(self.w[self.k])
            self.stamp = st
        out = self.plans[self.k]()
        self.k ^= 1
        return out


class _LaunchRecorder:
    """Proxies ``_native.device()`` and a device group's ``dc`` while a forward runs,
    keeping every native call with its arguments (the call still executes).  A plan holds
    raw pointers, so a recording during which the caching allocator handed out any block
    (a temporary whose pointer a call may have taken) sets ``allocated`` and must not be
    replayed."""

    def __init__(self, dc):
        self.calls = []
        self.dc = dc
        self.allocated = False

    def _proxy(self, target):
        rec = self

        class P:
            def __getattr__(self, name):
                f = getattr(target, name)
                if not callable(f):
                    return f

                def w(*a, **k):
                    rec.calls.append((f, a, k))
                    return f(*a, **k)
                w.__name__ = name
                return w
        return P()

    class _Active:
        def __init__(self, rec, layer):
            self.rec, self.layer = rec, layer

        @staticmethod
        def _allocs(layer) -> int:
            return int(torch.cuda.memory_stats(layer.device).get("allocation.all.allocated", 0))

        def __enter__(self):
            self.n0 = self._allocs(self.layer)
            self.orig = _native.device
            dev = self.orig()
            proxy = self.rec._proxy(dev)
            _native.device = lambda: proxy
            if self.rec.dc is not None:
                self.layer.tp_dev.dc = self.rec._proxy(self.rec.dc)
            return self.rec

        def __exit__(self, *exc):
            _native.device = self.orig
            if self.rec.dc is not None:
                self.layer.tp_dev.dc = self.rec.dc
            self.rec.allocated = self._allocs(self.layer) != self.n0
            return False

    def active(self, layer):
        return _LaunchRecorder._Active(self, layer)


class MnistTPLayer:
    def __init__(self, comm, cfg: LayerConfig, device=None):
        self.cfg = cfg
        self.comm = comm
        world, rank = comm.Get_size(), comm.Get_rank()
        if cfg.tp * cfg.dp != world:
            raise ValueError(f"tp*dp = {cfg.tp * cfg.dp} != world size {world}")
        if cfg.n_heads % cfg.tp:
            raise ValueError("n_heads must be divisible by tp")
        self.tp_idx, self.dp_idx, self.mp_comm, self.dp_comm, _, _ = get_info(
            comm, rank, cfg.tp, cfg.dp, "fc_q", cfg.d_model, cfg.d_attn)
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.tp_dev = device_group_for(self.mp_comm) if cfg.tp > 1 else None
        self.dp_dev = device_group_for(self.dp_comm) if cfg.dp > 1 else None
        self.hl = cfg.n_heads // cfg.tp
        self.hd = self.hl * cfg.head_dim  # local attention width
        d = cfg.d_model
        specs = [  # backward order -> bucket layout
            ("o_w", (cfg.out_pad, self.hd)), ("o_b", (cfg.out_pad,)),
            ("qkv_w", (3 * self.hd, d)), ("qkv_b", (3 * self.hd,)),
            ("emb_w", (d, cfg.kp)),
        ]
        grad_alloc = (lambda n: self.dp_dev.zeros(n, torch.float32)) if self.dp_dev is not None else None
        # W_qkv^T and W_o^T (backward dH and dpool GEMMs) are kept as transposed bf16
        # copies refreshed by the fused AdamW kernel: no transpose launch per step.  Only
        # the paths that run those GEMMs need them (the default re-associated embedding
        # gradient and the in-kernel dpool read neither), and the transposed tiles are
        # the slow part of the AdamW kernel
        transposed = [n for n, used in (("qkv_w", cfg.emb_grad == "dh" and cfg.plain_gemm == "own"),
                                         ("o_w", not self._fused_fc_o_bwd())) if used]
        self.flat = FlatParams(specs, self.device, grad_alloc, transposed=transposed)
        self.buckets = GradBuckets(self.flat, self.dp_dev, [["o_w", "o_b"], ["qkv_w", "qkv_b"],
                                                            ["emb_w"]],
                                   algo=cfg.dp_algo, overlap=cfg.overlap)
        self._load(full_init(cfg))
        self._bufs = {}
        self._hx = None
        self._fold_next = None  # (W_qkv, W_emb, W_eff') for the fused kernel's fold tail (pipelined plan)
        # [h | xp] rows padded to a multiple of 64 elements (128 B): every row of h
        # and of xp starts on a cache-line boundary (an 840-wide row costs the
        # embedding and QKV GEMMs ~8 us in straddled lines)
        self._hx_ld = (cfg.d_model + cfg.kp + 63) // 64 * 64

    # ------------------------------------------------------------- params
    def _load(self, w):
        cfg, t = self.cfg, self.tp_idx
        sl = slice(t * self.hd, (t + 1) * self.hd)
        P = self.flat.param
        P("emb_w").copy_(w["emb_w"])
        P("qkv_w").copy_(torch.cat([w["q_w"][sl], w["k_w"][sl], w["v_w"][sl]]))
        P("qkv_b").copy_(torch.cat([w["q_b"][sl], w["k_b"][sl], w["v_b"][sl]]))
        ow = torch.zeros(cfg.out_pad, self.hd)
        ow[: cfg.n_classes] = w["o_w"][:, sl]
        P("o_w").copy_(ow)
        ob = torch.zeros(cfg.out_pad)
        ob[: cfg.n_classes] = w["o_b"]
        P("o_b").copy_(ob)
        self.flat.refresh_bf16()

    def gathered_full(self):
        """Reassemble the unsharded weights (CPU, fp32) for checks."""
        cfg = self.cfg
        hc = self.mp_comm.comm if hasattr(self.mp_comm, "comm") else self.mp_comm
        parts = hc.allgather({k: self.flat.param(k).detach().cpu() for k in ("qkv_w", "qkv_b", "o_w")})
        q = torch.cat([p["qkv_w"][: self.hd] for p in parts])
        return {"q_w": q, "o_w": torch.cat([p["o_w"][: cfg.n_classes] for p in parts], dim=1),
                "emb_w": self.flat.param("emb_w").detach().cpu()}

    # ------------------------------------------------------------ buffers
    def _buf(self, name, shape, dtype, symmetric_on=None):
        key = (name, tuple(shape), dtype)
        b = self._bufs.get(key)
        if b is None:
            b = symmetric_on.empty(shape, dtype) if symmetric_on is not None else torch.empty(
                shape, dtype=dtype, device=self.device)
            self._bufs[key] = b
        return b

    # ------------------------------------------------------------ forward
    def input_buffer(self, B: int) -> torch.Tensor:
        """Where patchify should write a batch of B images.  With ``qkv_grad="direct"``
        (or ``emb_grad="dh"``): the right-hand column block of the activation buffer
        hx = [h | xp] (M x (d_model + kp) bf16); with both the embedding output h and
        its input xp in one row, the backward reads dQKV once for dQKV^T . [h | xp].
        The default re-associated backward never reads h: then xp is its own
        contiguous buffer."""
        cfg = self.cfg
        if cfg.emb_grad == "reassoc" and cfg.qkv_grad == "reassoc":
            # the backward never reads h, so h and xp need not share rows: separate
            # contiguous buffers write/read ~2 us faster (profiles/r1_qkv_reassoc/layout_probe.txt)
            return self._buf("xp", (B * cfg.seq, cfg.kp), torch.bfloat16)
        hx = self._buf("hx", (B * cfg.seq, self._hx_ld), torch.bfloat16)
        return hx[:, cfg.d_model:cfg.d_model + cfg.kp]

    def _folds(self) -> bool:
        """The forward weight fold W_eff = W_qkv W_emb, within the fold kernel's limits
        (csrc/device/wgrad.hip: d_model <= 1024 staged in LDS, d_model % 4 == 0);
        other widths fall back to h = Xp W_emb^T, then the QKV GEMM."""
        cfg = self.cfg
        return (cfg.fold_emb and cfg.emb_grad == "reassoc" and cfg.qkv_grad == "reassoc"
                and cfg.d_model <= 1024 and cfg.d_model % 4 == 0 and cfg.kp <= 96)

    def folded_qkv_weight(self, stream=None) -> torch.Tensor:
        """W_eff = W_qkv . W_emb (3hd x kp bf16) from the fp32 master weights (fp32
        accumulation, fixed summation order), recomputed on every forward so it always
        follows the optimizer (and is captured into the step's HIP graph).  b_qkv is
        added in the QKV GEMM's fp32 epilogue."""
        cfg = self.cfg
        R = 3 * self.hd
        weff = self._buf("weff", (R, cfg.kp), torch.bfloat16)
        wq, we = self.flat.param("qkv_w"), self.flat.param("emb_w")
        st = stream if stream is not None else torch.cuda.current_stream(self.device).cuda_stream
        _native.device().fold_emb_qkv(wq.data_ptr(), wq.stride(0), we.data_ptr(), we.stride(0), weff.data_ptr(),
                                      weff.stride(0), R, cfg.d_model, cfg.kp, st)
        return weff

    def forward(self, xp: torch.Tensor, B: int, images: Optional[torch.Tensor] = None,
                weff: Optional[torch.Tensor] = None, save: bool = True) -> torch.Tensor:
        """xp: (B*S, kp) bf16 patches -> logits (B, n_classes) fp32.  Saves activations.
        xp is either ``input_buffer(B)`` (fused [h | xp] layout) or any other tensor.
        With ``images`` ((B, 784) fp32) and the fused layout, the patch rows are
        generated inside the embedding GEMM (and stored to xp for the backward):
        no separate patchify pass."""
        cfg = self.cfg
        S, d = cfg.seq, cfg.d_model
        M = B * S
        P16 = self.flat.param16
        hx = self._bufs.get(("hx", (M, self._hx_ld), torch.bfloat16))
        fused = hx is not None and xp.data_ptr() == hx.data_ptr() + 2 * d and xp.stride(0) == hx.stride(0)
        qkv = self._buf("qkv", (M, 3 * self.hd), torch.bfloat16)
        h = None
        fuse_qkv = self._fuses_qkv(B)
        img = None  # images the fused kernel patchifies itself (MNIST 28 x 28 / 7 x 7)
        if self._folds():
            if images is not None:
                if fuse_qkv and cfg.img == 28 and cfg.patch == 7 and images.dtype == torch.float32 \
                        and images.is_contiguous() and os.environ.get("CCMPI_FUSE_PATCHIFY", "1") != "0":
                    img = images
                else:
                    patchify(images, cfg, out=xp)
            weff = weff if weff is not None else self.folded_qkv_weight()
            if not fuse_qkv:
                gemm_nt(xp, weff, out=qkv, bias=self.flat.param("qkv_b"))
            images = None
        else:
            h = hx[:, :d] if fused else self._buf("h", (M, d), torch.bfloat16)
        if h is not None and images is not None and not fused:
            patchify(images, cfg, out=xp)
            images = None
        if images is not None:
            x = images.contiguous().float()
            w = P16("emb_w")
            _native.device().embed_patches(x.data_ptr(), w.data_ptr(), h.data_ptr(), B, cfg.img, cfg.patch, d, cfg.kp,
                                           w.stride(0), h.stride(0), xp.data_ptr(), xp.stride(0),
                                           torch.cuda.current_stream(self.device).cuda_stream)
        elif h is not None:
            gemm_nt(xp, P16("emb_w"), out=h)  # bias + position are columns of W_emb
        if h is not None:
            gemm_nt(h, P16("qkv_w"), out=qkv, bias=self.flat.param("qkv_b"))
        lse = self._buf("lse", (B * self.hl, S), torch.float32)
        D = _native.device()
        st = torch.cuda.current_stream(self.device).cuda_stream
        naive = cfg.fc_o_mode == "naive" and cfg.tp > 1
        token = cfg.fc_o_mode == "token"
        tok_fused = token and self._fused_fc_o_bwd()
        # the per-token attention output is only consumed by the naive fc_o and the unfused /
        # pipelined token fc_o; the pooled path, the fused token kernel (and the MFMA backward,
        # which never reads O) skip materializing it
        mfma_attn = S <= 16 and cfg.head_dim in (32, 64, 128)
        tok_kernel_pre = token and tok_fused and mfma_attn and self._token_chunks(B) == 1
        pool = None if (naive or (token and not tok_fused)) else self._buf("pool", (B, self.hd), torch.bfloat16)
        att = self._buf("att", (M, self.hd), torch.bfloat16) if (naive or (token and not tok_kernel_pre)
                                                                   or not mfma_attn) else None
        fc_fused = self._fused_fc_o()
        zp = None
        fc = {}
        if fc_fused:
            # logits straight from the attention kernel: per head the pooled features times
            # this rank's W_o columns, heads summed in the workgroup, bias by TP rank 0
            zp = self._buf("zp", (B, cfg.out_pad), torch.float32, self.tp_dev)
            wo = self.flat.param16("o_w")
            fc = dict(wo=wo.data_ptr(), ld_wo=wo.stride(0), n_out=cfg.out_pad, zp=zp.data_ptr(), ld_zp=zp.stride(0),
                      bo=self.flat.param("o_b").data_ptr() if self.tp_idx == 0 else 0)
        # token fc_o with TP: attention runs per row block inside the TP pipeline below
        pipelined = token and self._token_chunks(B) > 1
        tok_kernel = token and tok_fused and mfma_attn and not pipelined
        if tok_kernel:
            att = None  # the attention kernel forms z itself; O is never stored
            # fused QKV: the kernel also forms q | k | v from the patch rows (stored to qkv only
            # when a backward will read it)
            self._token_fc_o_kernel(qkv, lse, pool, B, st,
                                    qkv_from=(xp, weff, save, img) if fuse_qkv else None)
        elif not pipelined:
            D.attn_small_fwd(qkv.data_ptr(), 0 if att is None else att.data_ptr(), lse.data_ptr(), B, S,
                             self.hl, cfg.head_dim, qkv.stride(0), self.hd if att is None else att.stride(0),
                             1.0 / math.sqrt(cfg.head_dim),
                             0 if pool is None else pool.data_ptr(), 0 if pool is None else pool.stride(0), st, **fc)
        if naive:
            z = self._forward_naive_fc_o(att, B)
            logits = z.view(B, S, cfg.out_pad)[:, :, : cfg.n_classes].mean(dim=1)
        elif token:
            z = self._zt if tok_kernel else self._forward_token_fc_o(att, B, qkv=qkv, lse=lse, pool=pool)
            if tok_fused:
                # logits = mean over the S tokens of the all-reduced z (o_b is in z, TP rank 0),
                # kept in zp for the fused loss head
                zp = self._buf("zp", (B, cfg.out_pad), torch.float32, self.tp_dev)
                if z is not None:  # (None: the kernel / inbox_mean already wrote the mean into zp)
                    # ordered sum over the tokens: bitwise the push form's inbox_mean
                    D.rows_mean(z.data_ptr(), z.stride(0), zp.data_ptr(), zp.stride(0), B, S, cfg.out_pad, st)
                logits = zp[:, : cfg.n_classes]
            else:
                logits = z.view(B, S, cfg.out_pad)[:, :, : cfg.n_classes].mean(dim=1)
        else:
            # fc_o and the mean over patches are linear: pool first (fused in the
            # attention kernel), so fc_o and its TP all-reduce work on B rows, not B*S
            if not fc_fused:
                zp = self._buf("zp", (B, cfg.out_pad), torch.float32, self.tp_dev)
                # output bias in the GEMM epilogue, added by TP rank 0 only (the TP all-reduce sums ranks)
                gemm_nt(pool, P16("o_w"), out=zp, out_dtype=torch.float32, splitk=1,
                        bias=self.flat.param("o_b") if self.tp_idx == 0 else None)
            if self.tp_dev is not None:
                self.tp_dev.allreduce(zp, zp, "SUM")  # row-parallel: one TP all-reduce (B x 16 fp32)
            logits = zp[:, : cfg.n_classes]  # bias already included
        if naive:
            logits = logits + self.flat.param("o_b")[: cfg.n_classes]
        self._saved = (xp, h, qkv, att, lse, B, pool) if save else None
        self._hx = hx[:, : d + cfg.kp] if fused else None
        return logits

    def forward_plan(self, images: torch.Tensor, B: int) -> Optional["LaunchPlan"]:
        """The inference forward of ``images`` as a **launch plan**: its native kernel launches
        recorded once with their arguments (every pointer into this layer's persistent
        buffers, weights and ``images``' storage) and re-issued by ``plan()`` from a loop
        with no per-step Python logic.  Two or three launches per step keep the host ahead
        of the GPU, and direct launches skip the per-replay cost of a HIP graph: 25.1 µs
        per step against 30.0 µs for the graph replay and 37.7 µs for ``forward_images``
        (N = 1, ``benchmarks/fwd_launch_probe.py``).  Reads live buffers: new weights
        (an optimizer step) and new pixels written into ``images`` are picked up.

        Only for the all-native forward: the fused QKV kernel in the local (TP = 1) or push
        TP form with fp32 contiguous images (no torch kernel runs in that forward: buffers
        are persistent, the logits a view); None otherwise."""
        cfg = self.cfg
        if not (self._fuses_qkv(B) and cfg.fc_o_mode == "token" and self.tp_fc_o_form(B) in ("local", "push")
                and images.dtype == torch.float32 and images.is_contiguous() and images.is_cuda):
            return None
        self.forward_images(images, B, save=False)   # persistent buffers exist before recording
        rec = _LaunchRecorder(self.tp_dev.dc if self.tp_dev is not None else None)
        with rec.active(self):
            logits = self.forward_images(images, B, save=False)
        return LaunchPlan(rec.calls, logits) if not rec.allocated else None

    def _fold_into(self, out: torch.Tensor) -> None:
        """The standalone weight fold (``fold_emb_qkv``) into ``out``."""
        cfg = self.cfg
        wq, we = self.flat.param("qkv_w"), self.flat.param("emb_w")
        _native.device().fold_emb_qkv(wq.data_ptr(), wq.stride(0), we.data_ptr(), we.stride(0), out.data_ptr(),
                                      out.stride(0), 3 * self.hd, cfg.d_model, cfg.kp,
                                      torch.cuda.current_stream(self.device).cuda_stream)

    def forward_plan_pipelined(self, images: torch.Tensor, B: int) -> Optional["PipelinedFoldPlan"]:
        """``forward_plan`` with the weight fold software-pipelined into the fused kernel: call
        i reads W_eff from buffer i % 2 and, once its attention work is done, each workgroup
        folds a tile of the NEXT call's W_eff = bf16(W_qkv W_emb) into the other buffer
        (``attn_qkv_fwd(fold_*)``, bitwise the fold kernel's result).  Every call still does
        one full fold and one full forward, from the current weights; the fold kernel's
        launch and its ~5 us (a latency-bound 240-workgroup kernel) leave the step.  When the
        weights changed since the last call (an optimizer step, a write into the parameters:
        ``FlatParams.step_count`` / the buffer's version) the call folds its own W_eff
        first; weights changed only by replayed recordings (``TrainPlan``) are not seen --
        ``invalidate()`` then.  Image-mode fused forward only; None otherwise."""
        cfg = self.cfg
        if not (self._fuses_qkv(B) and cfg.fc_o_mode == "token" and self.tp_fc_o_form(B) in ("local", "push")
                and images.dtype == torch.float32 and images.is_contiguous() and images.is_cuda
                and cfg.img == 28 and cfg.patch == 7 and os.environ.get("CCMPI_FUSE_PATCHIFY", "1") != "0"):
            return None
        R = 3 * self.hd
        w = [self._buf("weff_pipe0", (R, cfg.kp), torch.bfloat16), self._buf("weff_pipe1", (R, cfg.kp), torch.bfloat16)]
        xp = self.input_buffer(B)
        self.forward_images(images, B, save=False)  # persistent buffers exist before recording
        wq, we = self.flat.param("qkv_w"), self.flat.param("emb_w")
        plans = []
        try:
            for k in (0, 1):
                self._fold_into(w[k])
                self._fold_next = (wq, we, w[k ^ 1])
                rec = _LaunchRecorder(self.tp_dev.dc if self.tp_dev is not None else None)
                with rec.active(self):
                    logits = self.forward(xp, B, images=images, weff=w[k], save=False)
                if rec.allocated:
                    return None
                plans.append(LaunchPlan(rec.calls, logits))
        finally:
            self._fold_next = None
        return PipelinedFoldPlan(self, plans, w)

    def forward_images(self, images: torch.Tensor, B: int, save: bool = True) -> torch.Tensor:
        """(B, 784) fp32 images -> logits: patchify into the fused [h | xp] rows, then
        ``forward``.  With ``cfg.fwd_chunks = c > 1`` the batch is cut into c row blocks
        whose patchify -> embedding GEMM -> QKV GEMM -> attention chains run on c HIP
        streams (forked from and joined back to the current stream, so a HIP graph
        captures them as parallel branches): one block's memory-bound kernels overlap
        another's GEMMs.  Same buffers, same per-row arithmetic, bitwise the same
        results as the single-stream forward.  Measured at 32768 tokens (graph
        forward / train step): 1 stream 0.107 / 0.192 ms, 2 streams 0.123 / 0.233,
        4 streams 0.159 / 0.365 -- every kernel of the chain already fills the chip,
        and concurrent halves only contend -- so the default stays 1."""
        cfg = self.cfg
        xp = self.input_buffer(B)
        c = max(1, int(cfg.fwd_chunks))
        S = cfg.seq
        if (c == 1 or B % c or not self._fused_fc_o() or not (S <= 16 and cfg.head_dim in (32, 64, 128))
                or (B // c) * S < 256):
            # (running the weight fold on a side stream concurrent with patchify measured
            # slower: train step 0.140 -> 0.159 ms, forward 0.061 -> 0.066 ms)
            if self._fuses_qkv(B):
                return self.forward(xp, B, images=images, save=save)  # the fused kernel patchifies
            patchify(images, cfg, out=xp)
            return self.forward(xp, B, save=save)
        d, hl, hd = cfg.d_model, self.hl, self.hd
        M = B * S
        P16 = self.flat.param16
        hx = self._bufs.get(("hx", (M, self._hx_ld), torch.bfloat16))
        folds = self._folds()
        h = None if folds else (hx[:, :d] if hx is not None else self._buf("h", (M, d), torch.bfloat16))
        # on the main stream, before the fork
        weff = self.folded_qkv_weight() if folds else None
        qkv = self._buf("qkv", (M, 3 * hd), torch.bfloat16)
        lse = self._buf("lse", (B * hl, S), torch.float32)
        pool = self._buf("pool", (B, hd), torch.bfloat16)
        zp = self._buf("zp", (B, cfg.out_pad), torch.float32, self.tp_dev)
        wo, bias = P16("o_w"), self.flat.param("qkv_b")
        bo = self.flat.param("o_b").data_ptr() if self.tp_idx == 0 else 0
        D = _native.device()
        images = images.contiguous().float()
        main = torch.cuda.current_stream(self.device)
        key = ("streams", c)
        if key not in self._bufs:
            self._bufs[key] = [torch.cuda.Stream(self.device) for _ in range(c)]
        Bc = B // c
        for i, s in enumerate(self._bufs[key]):
            s.wait_stream(main)
            b0, b1 = i * Bc, (i + 1) * Bc
            r0, r1 = b0 * S, b1 * S
            with torch.cuda.stream(s):
                patchify(images[b0:b1], cfg, out=xp[r0:r1])
                if folds:
                    gemm_nt(xp[r0:r1], weff, out=qkv[r0:r1], bias=bias)
                else:
                    gemm_nt(xp[r0:r1], P16("emb_w"), out=h[r0:r1])
                    gemm_nt(h[r0:r1], P16("qkv_w"), out=qkv[r0:r1], bias=bias)
                D.attn_small_fwd(qkv[r0:r1].data_ptr(), 0, lse[b0 * hl:b1 * hl].data_ptr(), Bc, S, hl,
                                 cfg.head_dim, qkv.stride(0), hd, 1.0 / math.sqrt(cfg.head_dim), pool[b0:b1].data_ptr(),
                                 pool.stride(0), s.cuda_stream, wo=wo.data_ptr(), ld_wo=wo.stride(0),
                                 n_out=cfg.out_pad, zp=zp[b0:b1].data_ptr(), ld_zp=zp.stride(0), bo=bo)
        for s in self._bufs[key]:
            main.wait_stream(s)
        if self.tp_dev is not None:
            self.tp_dev.allreduce(zp, zp, "SUM")  # row-parallel: one TP all-reduce (B x 16 fp32)
        self._saved = (xp, h, qkv, None, lse, B, pool) if save else None
        self._hx = hx[:, : d + cfg.kp] if hx is not None else None
        return zp[:, : cfg.n_classes]

    def tp_fc_o_form(self, B: int) -> str:
        """"plain" or "push": how the fused per-token fc_o's TP sum runs (``cfg.tp_fc_o_form``)."""
        if self.tp_dev is None:
            return "local"
        form = self.cfg.tp_fc_o_form or os.environ.get("CCMPI_TP_FC_O_FORM", "auto")
        if form == "auto":
            form = "plain" if self.tp_dev.shared_device else "push"
        if form == "push" and B % self.cfg.tp:
            form = "plain"  # push needs whole sequences per TP rank's row block
        return form

    def _fuses_qkv(self, B: int) -> bool:
        """The token-mode forward runs the QKV projection inside the attention kernel
        (``k_qkv_attn16_fwd``): folded weights, the fused per-token fc_o
        (CCMPI_FUSE_QKV=0: the QKV GEMM + attention kernel instead).  The kernel keeps a
        head's folded weight in registers: head_dim <= 64, kp <= 72 (two spare depth columns
        carry the bias), local heads | 4."""
        cfg = self.cfg
        return (cfg.fuse_qkv and os.environ.get("CCMPI_FUSE_QKV", "1") != "0" and self._folds()
                and cfg.fc_o_mode == "token" and self._fused_fc_o_bwd() and self._token_chunks(B) == 1
                and cfg.seq <= 16 and cfg.head_dim in (32, 64) and cfg.kp <= 72 and 4 % self.hl == 0)

    def _token_fc_o_kernel(self, qkv, lse, pool, B: int, st: int, qkv_from=None) -> None:
        """Attention + per-token row-parallel fc_o in ONE kernel (``k_attn16_fwd``), then the
        TP sum of z (B*S x 16 fp32, o_b added by TP rank 0): an all-reduce ("plain"), or the
        kernel pushes every row block into its owner's inbox and the inbox-to-local two-shot
        completes it ("push", reference model/func_impl.py:94-109's output path, with the
        communication under the attention; the owners then reduce their row block to the
        sequences' logits and fan those out -- ``DeviceComm.inbox_mean`` -- so z is never
        gathered).  Leaves the summed z in ``self._zt`` (None when the logits went straight
        into zp: the push form, and the fused kernel's in-kernel mean at TP = 1)."""
        cfg = self.cfg
        S = cfg.seq
        M = B * S
        D = _native.device()
        z = self._buf("ztok", (M, cfg.out_pad), torch.float32, self.tp_dev)
        wo = self.flat.param16("o_w")
        kw = dict(wo=wo.data_ptr(), ld_wo=wo.stride(0), n_out=cfg.out_pad, ld_zt=cfg.out_pad,
                  bo=self.flat.param("o_b").data_ptr() if self.tp_idx == 0 else 0)
        args = (qkv.data_ptr(), 0, lse.data_ptr(), B, S, self.hl, cfg.head_dim, qkv.stride(0), self.hd,
                1.0 / math.sqrt(cfg.head_dim), pool.data_ptr(), pool.stride(0))  # pool: dW_o in backward
        fwd = D.attn_small_fwd
        if qkv_from is not None:
            xp, weff, keep, img = qkv_from
            bq = self.flat.param("qkv_b")

            def fwd(*_a, zrows=0, zpush=(), ztok=0, ld_zt=16, wo=0, ld_wo=0, n_out=0, bo=0, zmean=0, ld_zmean=16):
                stream = _a[-1]
                # with img the kernel builds the patch rows itself (stored to xp for a backward)
                fkw = {}
                fold = self._fold_next
                if fold is not None and img is not None:  # the next call's W_eff in the kernel's tail
                    fwq, fwe, fout = fold
                    fkw = dict(fold_wq=fwq.data_ptr(), ld_fold_wq=fwq.stride(0), fold_we=fwe.data_ptr(),
                               ld_fold_we=fwe.stride(0), fold_out=fout.data_ptr(), ld_fold_out=fout.stride(0),
                               fold_R=fwq.shape[0], fold_d=fwq.shape[1])
                D.attn_qkv_fwd(0 if img is not None else xp.data_ptr(), xp.stride(0), cfg.kp, weff.data_ptr(),
                               weff.stride(0), bq.data_ptr(), qkv.data_ptr() if keep else 0, qkv.stride(0),
                               lse.data_ptr() if keep else 0,  # lse: only a backward reads it
                               B, S, self.hl, cfg.head_dim, 1.0 / math.sqrt(cfg.head_dim),
                               pool.data_ptr() if keep else 0, pool.stride(0),  # pool: only the backward reads it
                               wo, ld_wo, n_out, bo, ztok, ld_zt, zrows, list(zpush),
                               stream, img=0 if img is None else img.data_ptr(),
                               xq_out=xp.data_ptr() if (img is not None and keep) else 0, zmean=zmean,
                               ld_zmean=ld_zmean, **fkw)
        form = self.tp_fc_o_form(B)
        if form == "push":
            inbox = self._buf("ztok_inbox", (M, cfg.out_pad), torch.float32, self.tp_dev)
            key = ("ztok_targets", inbox.data_ptr(), M)
            if key not in self._bufs:  # peer-mapped slot addresses: resolved once, no host call after
                self._bufs[key] = self.tp_dev.dc.push_targets(inbox.data_ptr(), inbox.numel() * 4)
            s = self.tp_dev._stream()
            fwd(*args, s, zrows=M // cfg.tp, zpush=self._bufs[key], **kw)
            if self._fused_fc_o_bwd():
                # the owners sum their row block AND average each sequence's rows, then fan the
                # B / tp logit rows out to every rank (k_inbox_mean): z itself is never gathered
                zp = self._buf("zp", (B, cfg.out_pad), torch.float32, self.tp_dev)
                self.tp_dev.dc.inbox_mean(inbox.data_ptr(), zp.data_ptr(), inbox.numel() * 4, S, s,
                                          self.tp_dev._budget(None))
                z = None
            else:
                self.tp_dev.dc.inbox_to_local(inbox.data_ptr(), z.data_ptr(), inbox.numel() * 4, 10, s,
                                              self.tp_dev._budget(None))
        elif self.tp_dev is None and qkv_from is not None:
            # local form (TP = 1): nothing to sum across ranks, so the fused kernel reduces z to
            # the logits (mean over the tokens) itself and z is never stored
            zp = self._buf("zp", (B, cfg.out_pad), torch.float32, self.tp_dev)
            fwd(*args, st, zmean=zp.data_ptr(), ld_zmean=zp.stride(0), **kw)
            z = None
        else:
            fwd(*args, st, ztok=z.data_ptr(), **kw)
            if self.tp_dev is not None:
                self.tp_dev.allreduce(z, z, "SUM", symmetric=True)  # z: heap block (_buf), same on every rank
        self._zt = z
        self._zt_form = form

    def _token_chunks(self, B: int) -> int:
        c = max(1, int(self.cfg.tp_chunks)) if self.tp_dev is not None else 1
        return c if (B % c == 0 and (B // c) * self.cfg.seq >= 256) else 1

    def _forward_token_fc_o(self, att, B, qkv=None, lse=None, pool=None):
        """Row-parallel fc_o per token: z = att . W_o[:, shard]^T (+ o_b on TP rank 0),
        summed over the TP group (B*S x 16 fp32 partial outputs).

        With ``tp_chunks = c > 1`` the batch is cut into c row blocks and each
        block runs attention -> fc_o GEMM on the main stream, then hands its
        partial z to the TP all-reduce (hand-written kernel, symmetric buffer,
        ``overlap_blocks`` CTAs) on a normal-priority side stream: block i's
        all-reduce runs under block i+1's attention.  Fork/join by events, so
        the whole pipeline is captured into the step's HIP graph."""
        cfg = self.cfg
        S = cfg.seq
        M = B * S
        z = self._buf("ztok", (M, cfg.out_pad), torch.float32, self.tp_dev)
        wo = self.flat.param16("o_w")
        bias = self.flat.param("o_b") if self.tp_idx == 0 else None
        c = self._token_chunks(B)
        if c == 1:
            gemm_nt(att, wo, out=z, out_dtype=torch.float32, splitk=1, bias=bias)
            if self.tp_dev is not None:
                self.tp_dev.allreduce(z, z, "SUM", symmetric=True)  # z: heap block (_buf), same on every rank
            return z
        main = torch.cuda.current_stream(self.device)
        if "tp_side" not in self._bufs:
            # CCMPI_TP_STREAM_PRIORITY: 0 = normal (default: 3-24x faster than -1 with 2 ranks
            # sharing a GPU, profiles/r2_overlap/tp2_priority.md), -1 = high priority
            prio = int(os.environ.get("CCMPI_TP_STREAM_PRIORITY", "0"))
            self._bufs["tp_side"] = torch.cuda.Stream(self.device, priority=prio)
        side = self._bufs["tp_side"]
        D = _native.device()
        hl, Bc = self.hl, B // c
        for i in range(c):
            b0, b1 = i * Bc, (i + 1) * Bc
            r0, r1 = b0 * S, b1 * S
            D.attn_small_fwd(qkv[r0:r1].data_ptr(), att[r0:r1].data_ptr(), lse[b0 * hl:b1 * hl].data_ptr(), Bc, S, hl,
                             cfg.head_dim, qkv.stride(0), att.stride(0), 1.0 / math.sqrt(cfg.head_dim),
                             0 if pool is None else pool[b0:b1].data_ptr(), 0 if pool is None else pool.stride(0),
                             main.cuda_stream)
            gemm_nt(att[r0:r1], wo, out=z[r0:r1], out_dtype=torch.float32, splitk=1, bias=bias)
            side.wait_stream(main)
            with torch.cuda.stream(side):
                self.tp_dev.allreduce(z[r0:r1], z[r0:r1], "SUM", max_blocks=self.tp_dev.overlap_blocks, symmetric=True)
        main.wait_stream(side)
        return z

    def _fused_fc_o(self) -> bool:
        return self.cfg.fc_o_mode != "token" and self._fused_fc_o_bwd()

    def _fused_fc_o_bwd(self) -> bool:
        """The fc_o input gradient formed inside the attention backward, from the
        (B x out) head gradient and W_o.  Also legal for the per-token fc_o: its loss
        reads the mean over the S tokens of z, so dZ[b, s] = dlogits[b] / S for every
        s and dW_o = sum_s dZ^T att = dlogits^T pool / S -- the same products as the
        pooled form, without the B*S x out dZ, the dW_o GEMM over B*S rows and the
        B*S x hd dAtt.  The forward still produces and all-reduces every token's z."""
        cfg = self.cfg
        return (cfg.fuse_fc_o and not (cfg.fc_o_mode == "naive" and cfg.tp > 1)
                and cfg.seq <= 16
                and cfg.head_dim in (32, 64, 128) and 4 % self.hl == 0 and cfg.out_pad <= 16)

    def _forward_naive_fc_o(self, att, B):
        """Reference collects: gather fc_o's input, out-sharded fc_o, gather its output."""
        cfg = self.cfg
        S = cfg.seq
        att_full = naive_collect_forward_input(att.view(B, S, self.hd), self.mp_comm, cfg.tp)
        att_full = att_full.reshape(B * S, cfg.d_attn)
        w_full = self._naive_o_w_full()
        k = cfg.out_pad // cfg.tp
        w_sh = w_full[self.tp_idx * k:(self.tp_idx + 1) * k].contiguous()
        out_local = gemm_nt(att_full, w_sh, out_dtype=torch.float32)
        z = naive_collect_forward_output(out_local.view(B, S, k), self.mp_comm, cfg.tp).reshape(B * S, cfg.out_pad)
        self._naive = (att_full, w_sh)
        return z

    def _naive_o_w_full(self):
        """[out_pad][d_attn] bf16: all TP ranks' input-dim shards side by side."""
        cfg = self.cfg
        w = self.flat.param16("o_w")
        parts = torch.empty(cfg.tp, cfg.out_pad, self.hd, dtype=torch.bfloat16, device=self.device)
        self.tp_dev.allgather(w.contiguous().view(-1), parts.view(-1))
        return torch.cat(list(parts), dim=1).contiguous()

    # ------------------------------------------------------------ backward
    def loss_and_grad_fused(self, y: torch.Tensor, global_batch: int) -> torch.Tensor:
        """Row (pooled) fc_o mode: softmax cross-entropy on the saved pooled logits in ONE
        HIP kernel (csrc/device/head.hip).  Writes the bf16 head gradient dZ (read by
        backward) and adds dL/d o_b to the flat gradient; returns the local loss sum /
        global batch as a 1-element tensor."""
        cfg = self.cfg
        B = y.numel()
        zp = self._buf("zp", (B, cfg.out_pad), torch.float32, self.tp_dev)
        dzp = self._buf("dzp", (B, cfg.out_pad), torch.bfloat16)
        loss = self._buf("loss", (1,), torch.float32)
        if "xent_ws" not in self._bufs:  # ticket + per-workgroup partials; the kernel re-arms the ticket
            self._bufs["xent_ws"] = torch.zeros(1 + (B + 15) // 16 + 64, dtype=torch.float32, device=self.device)
        ws = self._bufs["xent_ws"]
        if ws.numel() < 1 + (B + 15) // 16:
            ws = self._bufs["xent_ws"] = torch.zeros(1 + (B + 15) // 16 + 64, dtype=torch.float32, device=self.device)
        if y.dtype not in (torch.int32, torch.int64) or not y.is_contiguous():
            y = y.to(torch.int32).contiguous()
        st = torch.cuda.current_stream(self.device).cuda_stream
        pool = self._head_wo_pool(B)
        if pool is not None:
            # + dW_o = dZ^T pool in the same launch (the backward then skips its TN GEMM)
            gw = self.flat.grad("o_w")
            _native.device().xent_head_wo(zp.data_ptr(), zp.stride(0), y.data_ptr(), y.dtype == torch.int64, B,
                                          cfg.n_classes, cfg.out_pad, 1.0 / global_batch, loss.data_ptr(),
                                          dzp.data_ptr(), dzp.stride(0), self.flat.grad("o_b").data_ptr(),
                                          pool.data_ptr(), pool.stride(0), pool.shape[1], gw.data_ptr(), gw.stride(0),
                                          st, ws.data_ptr())
            self._dwo_done = True
        else:
            self._dwo_done = False  # a stale flag from an earlier fused head must not skip dW_o
            _native.device().xent_head(zp.data_ptr(), zp.stride(0), 0, y.data_ptr(),  # zp already holds + o_b
                                       y.dtype == torch.int64, B,
                                       cfg.n_classes, cfg.out_pad, 1.0 / global_batch, loss.data_ptr(), dzp.data_ptr(),
                                       dzp.stride(0), self.flat.grad("o_b").data_ptr(), st, ws.data_ptr())
        self._dz_ready = True
        return loss[0]

    def _head_wo_pool(self, B: int):
        """The saved pooled activations when the backward's output-head branch would form
        dW_o = dZ^T pool with its TN GEMM (pooled row-parallel / fused per-token fc_o), so the
        loss head can fold it in (``xent_head_wo``); None otherwise (or CCMPI_HEAD_WO=0)."""
        cfg = self.cfg
        if os.environ.get("CCMPI_HEAD_WO", "1") == "0" or self._saved is None or cfg.out_pad > 16:
            return None
        if (cfg.fc_o_mode == "naive" and cfg.tp > 1) or (cfg.fc_o_mode == "token" and not self._fused_fc_o_bwd()):
            return None
        pool = self._saved[6]
        if pool is None or self._saved[5] != B or pool.dtype != torch.bfloat16 or pool.stride(1) != 1:
            return None
        gw = self.flat.grad("o_w")
        if gw.dim() != 2 or gw.shape[1] != pool.shape[1] or gw.stride(1) != 1:
            return None
        return pool

    def loss_and_grad(self, logits: torch.Tensor, y: torch.Tensor, global_batch: int):
        """Cross-entropy (mean over the global batch); returns (local loss sum / global batch, dlogits)."""
        lp = torch.log_softmax(logits, dim=1)
        loss = -lp.gather(1, y.long().view(-1, 1)).sum() / global_batch
        dlogits = lp.exp()
        dlogits[torch.arange(y.numel(), device=y.device), y.long()] -= 1.0
        return loss, dlogits / global_batch

    def backward(self, dlogits: Optional[torch.Tensor]) -> None:
        """dlogits=None: the fused head (loss_and_grad_fused) already wrote dZ and dL/d o_b."""
        cfg = self.cfg
        self.flat.grad_dirty = True
        if self._saved is None:
            raise RuntimeError("backward: the last forward ran with save=False (no activations kept)")
        xp, h, qkv, att, lse, B, pool = self._saved
        S, d = cfg.seq, cfg.d_model
        M = B * S
        G = self.flat.grad
        P16 = self.flat.param16
        D = _native.device()
        st = torch.cuda.current_stream(self.device).cuda_stream
        # ---- output head: logits[b,c] = mean_s z[b,s,c] + o_b  (z = att . W_o^T)
        fused = dlogits is None
        if not fused:
            G("o_b")[: cfg.n_classes].add_(dlogits.sum(0))
        if (cfg.fc_o_mode == "naive" and cfg.tp > 1) or (cfg.fc_o_mode == "token" and not self._fused_fc_o_bwd()):
            dz = self._buf("dz", (M, cfg.out_pad), torch.bfloat16)
            dz.zero_()
            dz.view(B, S, cfg.out_pad)[:, :, : cfg.n_classes] = (dlogits / S).unsqueeze(1).to(torch.bfloat16)
            datt = self._buf("datt", (M, self.hd), torch.bfloat16)
            if cfg.fc_o_mode == "token":
                # row-parallel: dZ is replicated (identity backward of the all-reduce), the
                # input gradient is local to this rank's heads -- no TP communication
                gemm_tn(dz, att, out=G("o_w"), accumulate=True)          # dW_o[:, shard] = dZ^T att
                gemm_nt(dz, self.flat.param16_t("o_w"), out=datt)         # dAtt = dZ . W_o[:, shard]
            else:
                self._backward_naive_fc_o(dz, datt, B)
            dout, dout_b, dout_r = datt, S * datt.stride(0), datt.stride(0)
        else:
            # pooled row-parallel fc_o: dZ is replicated on every TP rank (identity backward
            # of the reduce); d(att[b,s]) = dpool[b] / S for every s, broadcast in the kernel
            dzp = self._buf("dzp", (B, cfg.out_pad), torch.bfloat16)
            if not fused:
                dzp.zero_()
                dzp[:, : cfg.n_classes] = dlogits.to(torch.bfloat16)
            # dW_o = dZ^T . pooled: 16 x hd over B rows, latency-bound; 32 K-splits measured fastest
            # (benchmarks/tn_small.py: 9.6 us at 8 splits, 7.2 us at 32) -- unless the fused loss
            # head already added it (xent_head_wo)
            if not (fused and getattr(self, "_dwo_done", False)):
                gemm_tn(dzp, pool, out=G("o_w"), accumulate=True, splitk=max(1, min(32, B // 64)))
            self._dwo_done = False
            if self._fused_fc_o_bwd():
                dout, dout_b, dout_r = None, 0, 0                   # dpool formed inside the attention bwd
            else:
                dpool = self._buf("dpool", (B, self.hd), torch.bfloat16)
                gemm_nt(dzp, self.flat.param16_t("o_w"), out=dpool, alpha=1.0 / S)
                dout, dout_b, dout_r = dpool, dpool.stride(0), 0
        self.buckets.ready(0)
        # ---- attention
        dqkv = self._buf("dqkv", (M, 3 * self.hd), torch.bfloat16)
        fc = {}
        if dout is None:
            dzp = self._buf("dzp", (B, cfg.out_pad), torch.bfloat16)
            wo = P16("o_w")
            fc = dict(dz=dzp.data_ptr(), ld_dz=dzp.stride(0), wo=wo.data_ptr(), ld_wo=wo.stride(0), n_out=cfg.out_pad,
                      dz_scale=1.0 / S)
        D.attn_small_bwd(qkv.data_ptr(), 0 if att is None else att.data_ptr(), lse.data_ptr(),
                         0 if dout is None else dout.data_ptr(),
                         dqkv.data_ptr(), G("qkv_b").data_ptr(), B, S, self.hl, cfg.head_dim, qkv.stride(0),
                         self.hd if att is None else att.stride(0),
                         1.0 / math.sqrt(cfg.head_dim), dout_b, dout_r, st, **fc)  # + QKV bias grad in-kernel
        # ---- fused QKV projection (column-parallel)
        if cfg.emb_grad == "reassoc" and cfg.qkv_grad == "reassoc":
            # h = Xp . W_emb^T, so dW_qkv = dQKV^T . h = (dQKV^T . Xp) . W_emb^T: the one
            # token-length contraction is A = dQKV^T . Xp (3hd x kp, 72 columns instead of
            # the 840 of dQKV^T . [h | xp]); A then yields both weight gradients through
            # two 72-deep fp32 GEMMs on [3hd x d] / [d x kp] matrices
            # A lives in a zeroed double buffer: the split-K GEMM accumulates into it with
            # atomics (no memset launch) and the weight-gradient kernel zeroes the other half
            key = ("a_emb2", 3 * self.hd, cfg.kp)
            if key not in self._bufs:
                self._bufs[key] = torch.zeros(2, 3 * self.hd, cfg.kp, dtype=torch.float32, device=self.device)
                self._a_idx = 0
            a, a_next = self._bufs[key][self._a_idx], self._bufs[key][self._a_idx ^ 1]
            self._a_idx ^= 1
            gemm_tn(dqkv, xp, out=a, accumulate=True, workspace=False)  # A = dQKV^T . Xp (MFMA, fp32)
            tp = self.tp_dev is not None
            ge = self._buf("gemb", (d, cfg.kp), torch.float32, self.tp_dev) if tp else G("emb_w")
            we, wq, gq = self.flat.param("emb_w"), self.flat.param("qkv_w"), G("qkv_w")
            if tp:
                ge.zero_()  # this rank's partial, accumulated by atomics, then TP-summed
            # dW_qkv += A . W_emb^T and dW_emb += W_qkv^T . A (TP: the partial) in one launch
            D.emb_qkv_wgrad(a.data_ptr(), a.stride(0), we.data_ptr(), we.stride(0), wq.data_ptr(), wq.stride(0),
                            gq.data_ptr(), gq.stride(0), ge.data_ptr(), ge.stride(0), a_next.data_ptr(),
                            a_next.stride(0), 3 * self.hd, d, cfg.kp, st)
            self.buckets.ready(1)
            if tp:
                self.tp_dev.allreduce(ge, ge, "SUM")              # 221 KB instead of tokens x d_model
                G("emb_w").add_(ge)
            self.buckets.ready(2)
            return
        if cfg.emb_grad == "reassoc" and self._hx is not None:
            # one GEMM over the fused activation rows: dQKV^T . [h | xp]; the split-K
            # reduction adds the h columns into dW_qkv and writes the xp columns to A
            a = self._buf("a_emb", (3 * self.hd, cfg.kp), torch.float32)
            gemm_tn(dqkv, self._hx, out=G("qkv_w"), accumulate=True, tail=a)
            self.buckets.ready(1)
            self._emb_grad_reassoc(dqkv, xp, a=a)
            self.buckets.ready(2)
            return
        gemm_tn(dqkv, h, out=G("qkv_w"), accumulate=True)      # dW_qkv = dQKV^T . h
        self.buckets.ready(1)
        if cfg.emb_grad == "reassoc":
            self._emb_grad_reassoc(dqkv, xp)
            self.buckets.ready(2)
            return
        dh = self._buf("dh", (M, d), torch.bfloat16)            # TP-partial input gradient
        if cfg.plain_gemm == "hipblaslt":
            torch.matmul(dqkv, P16("qkv_w"), out=dh)            # library GEMM, weight in its stored layout
        else:
            gemm_nt(dqkv, self.flat.param16_t("qkv_w"), out=dh)  # W_qkv^T kept by the optimizer
        # ---- embedding (replicated across TP): only its weight gradient needs the TP sum
        if self.tp_dev is not None:
            gpart = self._buf("gemb", (d, cfg.kp), torch.float32, self.tp_dev)
            gemm_tn(dh, xp, out=gpart)                           # partial dW_emb on this TP rank
            self.tp_dev.allreduce(gpart, gpart, "SUM")           # 221 KB instead of tokens x d_model
            G("emb_w").add_(gpart)
        else:
            gemm_tn(dh, xp, out=G("emb_w"), accumulate=True)     # dW_emb = dH^T . [patches | 1 | onehot]
        self.buckets.ready(2)

    def _emb_grad_reassoc(self, dqkv, xp, a=None) -> None:
        """dW_emb = dH^T . Xp with dH = dQKV . W_qkv.  The embedding input takes no
        gradient, so dH (tokens x d_model) is only ever contracted with Xp: compute
        A = dQKV^T . Xp (3*hd x kp, reduction over the tokens, fp32) and then
        dW_emb = W_qkv^T . A (d_model x kp).  Same gradient, contracted in the cheap
        order: the dH GEMM (tokens x d x 3hd) and its 50 MB round trip disappear.
        With TP > 1 each rank's product is its heads' partial sum, TP-all-reduced
        exactly like the dH path's partial weight gradient."""
        cfg = self.cfg
        d = cfg.d_model
        if a is None:
            a = self._buf("a_emb", (3 * self.hd, cfg.kp), torch.float32)
            gemm_tn(dqkv, xp, out=a)                             # A = dQKV^T . Xp (MFMA, fp32 accumulate)
        w = self.flat.param("qkv_w")                              # fp32 [3hd, d]
        G = self.flat.grad
        if self.tp_dev is not None:
            gpart = self._buf("gemb", (d, cfg.kp), torch.float32, self.tp_dev)
            torch.mm(w.t(), a, out=gpart)                         # plain 768x768x72 library GEMM
            self.tp_dev.allreduce(gpart, gpart, "SUM")
            G("emb_w").add_(gpart)
        else:
            G("emb_w").addmm_(w.t(), a)

    def _backward_naive_fc_o(self, dz, datt, B):
        """Reference backward collects: slice the output grad, local dX, reduce-scatter dX."""
        cfg = self.cfg
        S = cfg.seq
        att_full, w_sh = self._naive
        k = cfg.out_pad // cfg.tp
        dz_local = naive_collect_backward_output(dz.view(B, S, cfg.out_pad), self.tp_idx, cfg.tp)
        dz_local = dz_local.reshape(B * S, k).contiguous()
        # weight grad of this rank's OUT-sharded rows [k, d_attn]; the stored parameter is the
        # row-parallel INPUT shard [out_pad, hd], so assemble all ranks' rows (tiny) and slice columns
        gw_sh = gemm_tn(dz_local, att_full)                                                # [k, d_attn]
        gw_full = torch.zeros(cfg.out_pad, cfg.d_attn, dtype=torch.float32, device=self.device)
        gw_full[self.tp_idx * k:(self.tp_idx + 1) * k] = gw_sh
        self.tp_dev.allreduce(gw_full, gw_full, "SUM")
        self.flat.grad("o_w").add_(gw_full[:, self.tp_idx * self.hd:(self.tp_idx + 1) * self.hd])
        dx_full = gemm_nt(dz_local, transpose(w_sh), out_dtype=torch.bfloat16)     # [M, d_attn] partial
        dx = naive_collect_backward_x(dx_full.view(B, S, cfg.d_attn), self.mp_comm, cfg.tp)
        datt.copy_(dx.reshape(B * S, self.hd))

    def zero_grad(self) -> None:
        """The fused AdamW clears the gradient it consumes, so this only zeroes a
        gradient buffer that has not been through a step (first step, or after a
        backward without step)."""
        if self.flat.grad_dirty:
            self.flat.g.zero_()
            self.flat.grad_dirty = False

    def step(self) -> None:
        self.buckets.wait()
        # (graph_step: inside a captured training step the AdamW reads t from the device counter)
        self.flat.adamw(self.cfg.lr, weight_decay=self.cfg.weight_decay, grad_scale=1.0 / self.cfg.dp,
                        device_step=getattr(self, "graph_step", False))


def local_batch(cfg: LayerConfig, x_all: np.ndarray, y_all: np.ndarray, step: int, rank: int, device):
    """This rank's share of global batch ``step``: the global batch is
    ``batch * dp`` consecutive samples; ``split_data`` (reference
    data_parallel_preprocess.py:45-59 semantics) gives DP group ``rank // tp`` its
    contiguous block, identical on every TP rank of the group."""
    from ..data.preprocess import split_data

    G = cfg.batch * cfg.dp
    nb = max(1, x_all.shape[0] // G)
    i = step % nb
    xs, ys = split_data(x_all[i * G:(i + 1) * G], y_all[i * G:(i + 1) * G], cfg.tp, cfg.dp, rank)
    xb = torch.from_numpy(np.ascontiguousarray(xs)).to(device)
    yb = torch.from_numpy(np.ascontiguousarray(ys)).to(device)
    return xb, yb
