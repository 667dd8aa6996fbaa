"""The DP x TP harness layer (single rank) against a plain PyTorch fp32 autograd
reference of the same model: loss and every parameter gradient, for both ways
of forming the embedding weight gradient (re-associated / through dH)."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu


def _reference(cfg, xp, y, P):
    """fp32 autograd: patch embedding -> QKV -> softmax attention over the 16
    patches -> mean over patches -> fc_o -> cross-entropy (mean over batch)."""
    B = y.numel()
    S, H, hd = cfg.seq, cfg.n_heads, cfg.head_dim
    w = {k: v.detach().clone().requires_grad_(True) for k, v in P.items()}
    h = xp @ w["emb_w"].t()
    qkv = h @ w["qkv_w"].t() + w["qkv_b"]
    q, k, v = qkv.split(H * hd, dim=1)
    q, k, v = (t.reshape(B, S, H, hd).transpose(1, 2) for t in (q, k, v))
    att = torch.softmax(q @ k.transpose(-1, -2) / math.sqrt(hd), dim=-1) @ v   # (B, H, S, hd)
    pooled = att.transpose(1, 2).reshape(B, S, H * hd).mean(dim=1)
    z = pooled @ w["o_w"].t() + w["o_b"]
    loss = torch.nn.functional.cross_entropy(z[:, : cfg.n_classes], y.long())
    loss.backward()
    return loss.detach(), {k: t.grad for k, t in w.items()}


@pytest.mark.parametrize("emb_grad,qkv_grad,fused,fuse_fc_o,fold_emb,d_model", [
    ("reassoc", "reassoc", True, True, True, 768), ("reassoc", "reassoc", True, False, True, 768),
    ("reassoc", "reassoc", False, True, True, 768), ("reassoc", "reassoc", False, True, False, 768),
    ("reassoc", "direct", True, True, True, 768), ("reassoc", "direct", False, True, True, 768),
    ("dh", "direct", True, True, True, 768), ("dh", "direct", False, False, True, 768),
    # d_model > 1024: beyond the fold kernel's LDS staging -> unfolded embedding + QKV GEMMs
    ("reassoc", "reassoc", True, True, True, 1280)])
def test_harness_grads_match_torch_fp32(emb_grad, qkv_grad, fused, fuse_fc_o, fold_emb, d_model):
    from collective_communication_mpi_amd import MPI, Communicator
    from collective_communication_mpi_amd.models.harness import build
    from collective_communication_mpi_amd.models.mnist_tp import local_batch, patchify

    comm = Communicator(MPI.COMM_WORLD)
    cfg, layer, x_all, y_all = build(comm, 1, 128, emb_grad=emb_grad, qkv_grad=qkv_grad, fuse_fc_o=fuse_fc_o,
                                     fold_emb=fold_emb, d_model=d_model)
    assert layer._folds() == (fold_emb and emb_grad == qkv_grad == "reassoc" and d_model <= 1024)
    # non-trivial biases so their gradients and the bias epilogues are exercised
    g = torch.Generator().manual_seed(7)
    layer.flat.param("qkv_b").copy_(torch.randn(layer.flat.param("qkv_b").shape, generator=g) * 0.1)
    ob = torch.zeros(cfg.out_pad)
    ob[: cfg.n_classes] = torch.randn(cfg.n_classes, generator=g) * 0.1
    layer.flat.param("o_b").copy_(ob)
    layer.flat.refresh_bf16()
    xb, yb = local_batch(cfg, x_all, y_all, 0, 0, layer.device)
    xp = patchify(xb, cfg, out=layer.input_buffer(cfg.batch) if fused else None)
    layer.forward(xp, cfg.batch)
    layer.zero_grad()
    loss = layer.loss_and_grad_fused(yb, cfg.batch)
    layer.backward(None)
    torch.cuda.synchronize()
    names = ["emb_w", "qkv_w", "qkv_b", "o_w", "o_b"]
    # the reference sees the same bf16-rounded weights the kernels multiply with
    P = {k: layer.flat.param(k).detach().clone() for k in names}
    for k in ("emb_w", "qkv_w", "o_w"):
        P[k] = P[k].bfloat16().float()
    ref_loss, ref = _reference(cfg, xp.float(), yb, P)
    assert abs(loss.item() - ref_loss.item()) < 2e-2 * max(1.0, abs(ref_loss.item())), (loss.item(), ref_loss.item())
    for k in names:
        got = layer.flat.grad(k).detach().float()
        err = (got - ref[k]).norm() / ref[k].norm().clamp_min(1e-12)
        assert err < 4e-2, f"{emb_grad}: grad {k} rel err {err:.3e}"


@pytest.mark.parametrize("fuse_fc_o,fused_head", [(True, True), (True, False), (False, False)])
def test_token_fc_o_grads_match_torch_fp32(fuse_fc_o, fused_head):
    """Per-token fc_o (the reference's (B, S, out) layer shape): fused loss head + in-kernel
    fc_o backward (fuse_fc_o) and the dZ / dW_o / dAtt GEMM backward both match fp32
    autograd (the mean over tokens of z equals fc_o of the pooled features); the eager loss
    head (dlogits given to backward) also takes the in-kernel backward when it is legal."""
    from collective_communication_mpi_amd import MPI, Communicator
    from collective_communication_mpi_amd.models.harness import build
    from collective_communication_mpi_amd.models.mnist_tp import local_batch, patchify

    comm = Communicator(MPI.COMM_WORLD)
    cfg, layer, x_all, y_all = build(comm, 1, 128, fc_o_mode="token", fuse_fc_o=fuse_fc_o)
    assert layer._fused_fc_o_bwd() == fuse_fc_o
    g = torch.Generator().manual_seed(11)
    layer.flat.param("qkv_b").copy_(torch.randn(layer.flat.param("qkv_b").shape, generator=g) * 0.1)
    ob = torch.zeros(cfg.out_pad)
    ob[: cfg.n_classes] = torch.randn(cfg.n_classes, generator=g) * 0.1
    layer.flat.param("o_b").copy_(ob)
    layer.flat.refresh_bf16()
    xb, yb = local_batch(cfg, x_all, y_all, 0, 0, layer.device)
    xp = patchify(xb, cfg, out=layer.input_buffer(cfg.batch))
    logits = layer.forward(xp, cfg.batch)
    layer.zero_grad()
    if fused_head:
        loss = layer.loss_and_grad_fused(yb, cfg.batch)
        layer.backward(None)
    else:
        loss, dlogits = layer.loss_and_grad(logits, yb, cfg.batch)
        layer.backward(dlogits)
    torch.cuda.synchronize()
    names = ["emb_w", "qkv_w", "qkv_b", "o_w", "o_b"]
    P = {k: layer.flat.param(k).detach().clone() for k in names}
    for k in ("emb_w", "qkv_w", "o_w"):
        P[k] = P[k].bfloat16().float()
    ref_loss, ref = _reference(cfg, xp.float(), yb, P)
    assert abs(loss.item() - ref_loss.item()) < 2e-2 * max(1.0, abs(ref_loss.item())), (loss.item(), ref_loss.item())
    for k in names:
        got = layer.flat.grad(k).detach().float()
        err = (got - ref[k]).norm() / ref[k].norm().clamp_min(1e-12)
        assert err < 4e-2, f"token fuse_fc_o={fuse_fc_o} fused_head={fused_head}: grad {k} rel err {err:.3e}"


@pytest.mark.parametrize("chunks", [2, 4])
def test_chunked_multistream_forward_is_bitwise_identical(chunks):
    """forward_images on c HIP streams == the single-stream forward: logits and the saved
    activations bitwise, and the gradients of a following backward."""
    from collective_communication_mpi_amd import MPI, Communicator
    from collective_communication_mpi_amd.models.harness import build
    from collective_communication_mpi_amd.models.mnist_tp import local_batch

    comm = Communicator(MPI.COMM_WORLD)
    out = {}
    for c in (1, chunks):
        cfg, layer, x_all, y_all = build(comm, 1, 256, fwd_chunks=c)
        xb, yb = local_batch(cfg, x_all, y_all, 0, 0, layer.device)
        logits = layer.forward_images(xb, cfg.batch).clone()
        xp, h, qkv, _, lse, _, pool = layer._saved
        layer.zero_grad()
        layer.loss_and_grad_fused(yb, cfg.batch)
        layer.backward(None)
        torch.cuda.synchronize()
        assert (h is None) == layer._folds()  # the folded forward never forms h
        out[c] = (logits, qkv.clone(), lse.clone(), pool.clone(), layer.flat.g.clone())
    for a, b in zip(out[1][:-1], out[chunks][:-1]):
        assert torch.equal(a, b)
    # the weight gradients go through split-K fp32 atomics: equal up to summation order
    torch.testing.assert_close(out[chunks][-1], out[1][-1], rtol=1e-4, atol=1e-6)


def test_inference_forward_matches_training_forward():
    """forward_images(save=False) (nothing kept for a backward) gives the same logits as
    the saving forward, and a backward after it fails loudly."""
    from collective_communication_mpi_amd import MPI, Communicator
    from collective_communication_mpi_amd.models.harness import build
    from collective_communication_mpi_amd.models.mnist_tp import local_batch

    comm = Communicator(MPI.COMM_WORLD)
    cfg, layer, x_all, y_all = build(comm, 1, 256)
    xb, _ = local_batch(cfg, x_all, y_all, 0, 0, layer.device)
    a = layer.forward_images(xb, cfg.batch).clone()
    b = layer.forward_images(xb, cfg.batch, save=False).clone()
    torch.cuda.synchronize()
    assert torch.equal(a, b)
    with pytest.raises(RuntimeError):
        layer.backward(None)
