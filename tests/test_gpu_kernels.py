"""Single-rank numerics of the HIP kernels vs plain PyTorch fp32 references."""
import os

import pytest
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _ref(a, b, bias=None, act=None, alpha=1.0):
    y = alpha * (a.float() @ b.float().T)
    if bias is not None:
        y = y + bias.float()
    if act == "relu":
        y = torch.relu(y)
    elif act == "gelu":
        y = torch.nn.functional.gelu(y, approximate="tanh")
    return y


@pytest.mark.parametrize("M,N,K", [(1, 1, 8), (16, 16, 32), (128, 128, 64), (130, 70, 72), (2048, 768, 64),
                                   (32768, 768, 72), (1000, 300, 40), (513, 1000, 128), (300, 7, 8),
                                   (4096, 768, 768), (32768, 384, 768), (777, 1000, 520)])
def test_gemm_nt_shapes(M, N, K):
    from collective_communication_mpi_amd.ops import gemm_nt

    g = torch.Generator(device="cuda").manual_seed(M * 7 + N * 3 + K)
    a = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    b = torch.randn(N, K, device="cuda", generator=g).bfloat16()
    y = gemm_nt(a, b, out_dtype=torch.float32)
    ref = _ref(a, b)
    torch.testing.assert_close(y, ref, rtol=2e-3, atol=2e-3 * K ** 0.5)


@pytest.fixture(params=[2, 3, 4], ids=["256x256", "256x128", "256x192"])
def gemm256(request):
    """Force a large-tile ping-pong kernel whenever legal (K % 128 == 0)."""
    from collective_communication_mpi_amd import _native

    D = _native.device()
    D.gemm_set_kernel(request.param)
    yield
    D.gemm_set_kernel(0)


@pytest.mark.parametrize("M,N,K", [(256, 256, 128), (1, 8, 128), (300, 520, 256), (777, 1000, 512),
                                   (4096, 768, 768), (2048, 2048, 4096), (32768, 768, 768), (32768, 384, 768),
                                   (512, 200, 384)])
def test_gemm256_shapes(gemm256, M, N, K):
    from collective_communication_mpi_amd.ops import gemm_nt

    g = torch.Generator(device="cuda").manual_seed(M * 5 + N * 11 + K)
    a = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    b = torch.randn(N, K, device="cuda", generator=g).bfloat16()
    for splitk in (1, 3):
        y = gemm_nt(a, b, out_dtype=torch.float32, splitk=splitk)
        torch.testing.assert_close(y, _ref(a, b), rtol=2e-3, atol=2e-3 * K ** 0.5)
    # repeated launches: an intermittent race shows up as a mismatch between runs
    y0 = gemm_nt(a, b, out_dtype=torch.float32, splitk=1)
    for _ in range(3):
        torch.testing.assert_close(gemm_nt(a, b, out_dtype=torch.float32, splitk=1), y0, rtol=0, atol=0)


@pytest.mark.parametrize("act", [None, "gelu"])
def test_gemm256_epilogue(gemm256, act):
    from collective_communication_mpi_amd.ops import gemm_nt

    a = torch.randn(600, 384, device="cuda").bfloat16()
    b = torch.randn(520, 384, device="cuda").bfloat16()
    bias = torch.randn(520, device="cuda").bfloat16()
    y = gemm_nt(a, b, bias=bias, act=act, alpha=0.5)
    torch.testing.assert_close(y.float(), _ref(a, b, bias, act, 0.5), rtol=2e-2, atol=8e-2)
    c = torch.randn(600, 520, device="cuda")
    c0 = c.clone()
    gemm_nt(a, b, out=c, accumulate=True, splitk=1)
    torch.testing.assert_close(c, c0 + _ref(a, b), rtol=2e-3, atol=5e-2)


@pytest.mark.parametrize("sched", [0, 1, 3, 4, 5, 8, 9, 8 | 16384, 9 | 16384],
                         ids=["w4", "w4p", "w4po", "w4f", "w4pf", "ring", "ringp", "ringpair", "ringpairp"])
@pytest.mark.parametrize("M,N,K", [(256, 256, 64), (256, 256, 128), (300, 520, 256), (777, 1000, 512),
                                   (2048, 2048, 4096), (1, 8, 192), (4096, 768, 768)])
def test_gemm_w4_shapes(sched, M, N, K):
    """Four-wave 256x256 kernels (gemm_w4.hip), every schedule variant incl. the LDS ring,
    against an fp32 reference; bias + bf16 out and accumulate on one shape."""
    from collective_communication_mpi_amd import _native
    from collective_communication_mpi_amd.ops import gemm_nt

    D = _native.device()
    D.gemm_set_kernel(5)
    D.gemm_set_w4_sched(sched)
    try:
        g = torch.Generator(device="cuda").manual_seed(M * 3 + N * 7 + K + sched)
        a = torch.randn(M, K, device="cuda", generator=g).bfloat16()
        b = torch.randn(N, K, device="cuda", generator=g).bfloat16()
        y = gemm_nt(a, b, out_dtype=torch.float32)
        torch.testing.assert_close(y, _ref(a, b), rtol=2e-3, atol=2e-3 * K ** 0.5)
        for _ in range(2):
            torch.testing.assert_close(gemm_nt(a, b, out_dtype=torch.float32), y, rtol=0, atol=0)
        # bf16 out, no bias: the ring kernel's fast epilogue (bf16 = RNE of the fp32 result)
        y16 = gemm_nt(a, b, alpha=0.5)
        torch.testing.assert_close(y16.float(), (0.5 * y).bfloat16().float(), rtol=1e-2, atol=1e-2)
        if M == 300:
            bias = torch.randn(N, device="cuda").bfloat16()
            yb = gemm_nt(a, b, bias=bias, alpha=0.5)
            torch.testing.assert_close(yb.float(), _ref(a, b, bias, None, 0.5), rtol=2e-2, atol=8e-2)
            c = torch.randn(M, N, device="cuda")
            c0 = c.clone()
            gemm_nt(a, b, out=c, accumulate=True)
            torch.testing.assert_close(c, c0 + _ref(a, b), rtol=2e-3, atol=5e-2)
    finally:
        D.gemm_set_kernel(0)
        D.gemm_set_w4_sched(1)


def test_gemm_asymmetric_identity():
    """A = I with an asymmetric B catches a transposed C write (guide §3)."""
    from collective_communication_mpi_amd.ops import gemm_nt

    n = 64
    a = torch.eye(n, device="cuda").bfloat16()
    b = torch.arange(n * n, device="cuda", dtype=torch.float32).reshape(n, n).remainder(97).bfloat16()
    y = gemm_nt(a, b, out_dtype=torch.float32)
    torch.testing.assert_close(y, b.float().T)
    # same check through the 256x256 kernel (K % 128 == 0)
    from collective_communication_mpi_amd import _native

    n = 256
    a = torch.eye(n, device="cuda").bfloat16()
    b = torch.arange(n * n, device="cuda", dtype=torch.float32).reshape(n, n).remainder(97).bfloat16()
    _native.device().gemm_set_kernel(2)
    try:
        y = gemm_nt(a, b, out_dtype=torch.float32, splitk=1)
    finally:
        _native.device().gemm_set_kernel(0)
    torch.testing.assert_close(y, b.float().T)


@pytest.mark.parametrize("act", [None, "relu", "gelu"])
@pytest.mark.parametrize("bias_dtype", [torch.float32, torch.bfloat16])
def test_gemm_epilogue(act, bias_dtype):
    from collective_communication_mpi_amd.ops import gemm_nt

    a = torch.randn(300, 128, device="cuda").bfloat16()
    b = torch.randn(200, 128, device="cuda").bfloat16()
    bias = torch.randn(200, device="cuda").to(bias_dtype)
    y = gemm_nt(a, b, bias=bias, act=act, alpha=0.5)
    torch.testing.assert_close(y.float(), _ref(a, b, bias, act, 0.5), rtol=2e-2, atol=5e-2)


@pytest.mark.parametrize("out_dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("slice_bn", [128, 256])
def test_gemm_smallk_epilogue(out_dtype, slice_bn):
    """K <= 96 path (LDS-resident B, direct vector stores): bias, act, accumulate, both outputs."""
    from collective_communication_mpi_amd import _native
    from collective_communication_mpi_amd.ops import gemm_nt

    _native.device().gemm_set_smallk(slice_bn, 2048)
    a = torch.randn(700, 72, device="cuda").bfloat16()
    b = torch.randn(520, 72, device="cuda").bfloat16()
    bias = torch.randn(520, device="cuda")
    y = gemm_nt(a, b, bias=bias, act="gelu", alpha=0.5, out_dtype=out_dtype)
    torch.testing.assert_close(y.float(), _ref(a, b, bias, "gelu", 0.5), rtol=2e-2, atol=5e-2)
    c = torch.randn(700, 520, device="cuda").to(out_dtype)
    c0 = c.float().clone()
    gemm_nt(a, b, out=c, accumulate=True, splitk=1)
    _native.device().gemm_set_smallk(128, 2048)
    torch.testing.assert_close(c.float(), c0 + _ref(a, b), rtol=2e-2, atol=8e-2)


def test_gemm_accumulate_strided():
    from collective_communication_mpi_amd.ops import gemm_nt

    big = torch.randn(100, 96, device="cuda").bfloat16()
    a = big[:, 16:80]  # row stride 96, K = 64
    b = torch.randn(40, 64, device="cuda").bfloat16()
    c = torch.randn(100, 40, device="cuda")
    c0 = c.clone()
    gemm_nt(a, b, out=c, accumulate=True)
    torch.testing.assert_close(c, c0 + _ref(a, b), rtol=2e-3, atol=2e-2)


def test_transpose_and_interleave():
    from collective_communication_mpi_amd.ops import deinterleave_lastaxis, interleave_lastaxis, transpose

    x = torch.randn(333, 129, device="cuda").bfloat16()
    torch.testing.assert_close(transpose(x), x.T.contiguous())
    for dt in (torch.float32, torch.bfloat16, torch.float64, torch.int32):
        st = torch.randn(4, 3, 5, 6, device="cuda").to(dt)
        inter = interleave_lastaxis(st, 4)
        torch.testing.assert_close(inter, torch.cat(list(st), dim=-1))
        torch.testing.assert_close(deinterleave_lastaxis(inter, 4), st)


@pytest.mark.parametrize("kind", ["lds", "reg"])
@pytest.mark.parametrize("R,C", [(8, 8), (520, 72), (4096, 1032), (1000, 16), (24, 4104)])
def test_transpose_vectorized(R, C, kind):
    """16-B transpose kernels (R, C % 8 == 0), LDS tile and register transpose (picked by
    CCMPI_TRANSPOSE at the first call in a process: the reg case runs in a child):
    partial workgroups in both dimensions, a strided source view, against torch."""
    if kind == "reg":
        import subprocess
        import sys

        code = (f"import torch, tests.test_gpu_kernels as t; t._transpose_check({R}, {C})")
        env = {**os.environ, "CCMPI_TRANSPOSE": "reg"}
        r = subprocess.run([sys.executable, "-c", code], cwd=REPO, env=env, capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stderr[-2000:]
        return
    _transpose_check(R, C)


def _transpose_check(R, C):
    from collective_communication_mpi_amd.ops import transpose

    x = torch.randn(R, C + 8, device="cuda").bfloat16()[:, :C]
    torch.testing.assert_close(transpose(x), x.T.contiguous(), rtol=0, atol=0)
    out = torch.empty(C, R + 16, device="cuda", dtype=torch.bfloat16)[:, :R]
    transpose(x, out=out)
    torch.testing.assert_close(out, x.T, rtol=0, atol=0)


def test_single_rank_communicator_paths():
    from collective_communication_mpi_amd import MPI, Communicator

    comm = Communicator(MPI.COMM_WORLD)
    x = torch.randn(1 << 20, device="cuda")
    y = torch.empty_like(x)
    comm.Allreduce(x, y, MPI.SUM)
    torch.testing.assert_close(y, x)
    s = comm.empty(1 << 20)
    s.copy_(x)
    comm.myAllreduce(s, y, MPI.MAX, algo="twoshot")
    torch.testing.assert_close(y, x)
    z = torch.empty(3, 1 << 18, device="cuda")
    comm.Allgather(x[: 3 << 18].reshape(3, -1)[0], z[0])
    assert comm.total_bytes_transferred == 0  # p = 1: no traffic in any formula


@pytest.mark.parametrize("nbytes", [(1 << 20) + 16, (1 << 20) + 6, 48 << 20, (4 << 30) + 4096 + 48])
def test_single_rank_allreduce_copy(nbytes):
    """N = 1 all-reduce = the contiguous-slice copy kernel: exact bytes, tails, > 2^20 workgroups' worth."""
    from collective_communication_mpi_amd import MPI, Communicator, _native

    D = _native.device()
    x = torch.randn(nbytes // 2, device="cuda", dtype=torch.float16)
    y = torch.zeros_like(x)
    Communicator(MPI.COMM_WORLD).Allreduce(x, y, MPI.SUM)
    assert torch.equal(x, y)


def test_split_derives_rccl_communicator():
    """Split of a communicator that has RCCL derives the child's via ncclCommSplit."""
    from collective_communication_mpi_amd import MPI, Communicator

    comm = Communicator(MPI.COMM_WORLD)
    comm.dev.ensure_rccl()
    child = comm.Split(key=0, color=0)
    assert child.dev._rccl
    x = torch.arange(4096, device="cuda", dtype=torch.float32)
    y = torch.empty_like(x)
    child.Allreduce(x, y, MPI.SUM, algo="rccl")
    torch.cuda.synchronize()
    torch.testing.assert_close(y, x)


@pytest.mark.parametrize("M,N1,N2", [(64, 16, 128), (32768, 384, 768), (32768, 768, 64), (1000, 136, 72), (7, 8, 8),
                                     (320, 128, 72), (32768, 768, 72)])
@pytest.mark.parametrize("splitk", [1, 4, None])
@pytest.mark.parametrize("pf", [0, 1, 2])  # K tiles in flight: auto, one, two (odd / even tile counts above)
def test_gemm_tn_weight_grad(M, N1, N2, splitk, pf):
    from collective_communication_mpi_amd import _native
    from collective_communication_mpi_amd.ops import gemm_tn

    _native.device().gemm_tn_set_prefetch(pf)
    try:
        g = torch.Generator(device="cuda").manual_seed(M + N1 + N2)
        a = torch.randn(M, N1, device="cuda", generator=g).bfloat16()
        b = torch.randn(M, N2, device="cuda", generator=g).bfloat16()
        ref = a.float().T @ b.float()
        out = gemm_tn(a, b, splitk=splitk)
        torch.testing.assert_close(out, ref, rtol=2e-3, atol=2e-3 * M ** 0.5)
        acc = torch.ones(N1, N2, device="cuda")
        gemm_tn(a, b, out=acc, accumulate=True, alpha=0.5, splitk=splitk)
        torch.testing.assert_close(acc, 1 + 0.5 * ref, rtol=2e-3, atol=2e-3 * M ** 0.5)
        acc.fill_(1.0)
        gemm_tn(a, b, out=acc, accumulate=True, splitk=splitk, workspace=True)
        torch.testing.assert_close(acc, 1 + ref, rtol=2e-3, atol=2e-3 * M ** 0.5)
    finally:
        _native.device().gemm_tn_set_prefetch(0)


@pytest.mark.parametrize("M,N1,c,N2,ldb", [(32768, 768, 768, 840, 896), (4096, 256, 128, 200, 264),
                                            (1000, 136, 64, 72, 72)])
def test_gemm_tn_column_split(M, N1, c, N2, ldb):
    """gemm_tn(tail=...): columns < c accumulate into out, the rest overwrite tail,
    with b a column window of a wider (padded) row buffer."""
    from collective_communication_mpi_amd.ops import gemm_tn

    g = torch.Generator(device="cuda").manual_seed(M + c)
    a = torch.randn(M, N1, device="cuda", generator=g).bfloat16()
    wide = torch.randn(M, ldb, device="cuda", generator=g).bfloat16()
    b = wide[:, :N2]
    ref = a.float().T @ b.float()
    out = torch.full((N1, c), 2.0, device="cuda")
    tail = torch.full((N1, N2 - c), 7.0, device="cuda")
    gemm_tn(a, b, out=out, accumulate=True, tail=tail)
    tol = dict(rtol=2e-3, atol=2e-3 * M ** 0.5)
    torch.testing.assert_close(out, 2 + ref[:, :c], **tol)
    torch.testing.assert_close(tail, ref[:, c:], **tol)


def test_gemm_tn_asymmetric():
    """A^T with A = I and asymmetric B catches row/column swaps in the tr-read path."""
    from collective_communication_mpi_amd.ops import gemm_tn

    n = 128
    a = torch.eye(n, device="cuda").bfloat16()
    b = torch.arange(n * n, device="cuda", dtype=torch.float32).reshape(n, n).remainder(89).bfloat16()
    torch.testing.assert_close(gemm_tn(a, b, splitk=1), b.float())
    torch.testing.assert_close(gemm_tn(b, a, splitk=1), b.float().T)


@pytest.mark.parametrize("splitk", [2, 8])
def test_gemm_nt_splitk(splitk):
    from collective_communication_mpi_amd.ops import gemm_nt

    a = torch.randn(256, 4096, device="cuda").bfloat16()
    b = torch.randn(192, 4096, device="cuda").bfloat16()
    bias = torch.randn(192, device="cuda")
    y = gemm_nt(a, b, bias=bias, out_dtype=torch.float32, splitk=splitk)
    torch.testing.assert_close(y, _ref(a, b, bias), rtol=2e-3, atol=0.15)


def _attn_ref(qkv, B, S, H, D):
    q, k, v = qkv.float().view(B, S, 3, H, D).unbind(2)
    q, k, v = (t.transpose(1, 2) for t in (q, k, v))  # B,H,S,D
    p = torch.softmax(q @ k.transpose(-1, -2) / D ** 0.5, dim=-1)
    return (p @ v).transpose(1, 2).reshape(B * S, H * D)


@pytest.mark.parametrize("B,S,H,D", [(3, 16, 2, 64), (2, 7, 1, 32), (4, 64, 2, 64), (9, 1, 2, 32), (5, 16, 3, 128),
                                     (2048, 16, 4, 64), (4096, 16, 3, 32), (6, 12, 4, 64), (3, 33, 2, 64)])
def test_attn_small_fwd_bwd(B, S, H, D):
    from collective_communication_mpi_amd import _native

    dev = _native.device()
    st = torch.cuda.current_stream().cuda_stream
    qkv = (torch.randn(B * S, 3 * H * D, device="cuda") * 0.5).bfloat16()
    o = torch.empty(B * S, H * D, device="cuda", dtype=torch.bfloat16)
    lse = torch.empty(B * H, S, device="cuda")
    pool = torch.empty(B, H * D, device="cuda", dtype=torch.bfloat16)
    dev.attn_small_fwd(qkv.data_ptr(), o.data_ptr(), lse.data_ptr(), B, S, H, D, qkv.stride(0), o.stride(0),
                       D ** -0.5, pool.data_ptr(), pool.stride(0), st)
    ref_in = qkv.float().requires_grad_(True)
    ref = _attn_ref(ref_in, B, S, H, D)
    torch.testing.assert_close(o.float(), ref.detach(), rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(pool.float(), ref.detach().view(B, S, H * D).mean(1), rtol=2e-2, atol=2e-2)
    if S <= 16 and D in (32, 64, 128):  # pooled-only forward: O is not materialized
        pool2 = torch.empty_like(pool)
        lse2 = torch.empty_like(lse)
        dev.attn_small_fwd(qkv.data_ptr(), 0, lse2.data_ptr(), B, S, H, D, qkv.stride(0), H * D, D ** -0.5,
                           pool2.data_ptr(), pool2.stride(0), st)
        torch.testing.assert_close(pool2, pool, rtol=0, atol=0)
        torch.testing.assert_close(lse2, lse, rtol=0, atol=0)
    do = torch.randn(B * S, H * D, device="cuda").bfloat16()
    ref.backward(do.float())
    dqkv = torch.empty_like(qkv)
    dbias = torch.zeros(3 * H * D, device="cuda")
    dev.attn_small_bwd(qkv.data_ptr(), o.data_ptr(), lse.data_ptr(), do.data_ptr(), dqkv.data_ptr(),
                       dbias.data_ptr(), B, S, H, D, qkv.stride(0), o.stride(0), D ** -0.5, S * do.stride(0),
                       do.stride(0), st)
    torch.testing.assert_close(dqkv.float(), ref_in.grad, rtol=3e-2, atol=3e-2)
    # bias gradient = column sums of the fp32 gradient (not of the bf16-rounded dqkv:
    # rounding noise over B*S rows would dominate at large B)
    ref_b = ref_in.grad.sum(0)
    assert (dbias - ref_b).norm() <= 2e-2 * ref_b.norm() + 1e-3, ((dbias - ref_b).abs().max(), ref_b.abs().max())
    # broadcast form: dO[b, s] = g[b] for every s (pooled-gradient path, row stride 0)
    gpool = torch.randn(B, H * D, device="cuda").bfloat16()
    ref_in.grad = None
    ref2 = _attn_ref(ref_in, B, S, H, D)
    ref2.backward(gpool.float().repeat_interleave(S, dim=0))
    dev.attn_small_bwd(qkv.data_ptr(), o.data_ptr(), lse.data_ptr(), gpool.data_ptr(), dqkv.data_ptr(), 0, B, S,
                       H, D, qkv.stride(0), o.stride(0), D ** -0.5, gpool.stride(0), 0, st)
    torch.testing.assert_close(dqkv.float(), ref_in.grad, rtol=3e-2, atol=3e-2)


@pytest.mark.parametrize("B,S,H,D,n_out", [(2048, 16, 4, 64, 16), (37, 16, 2, 128, 10), (13, 9, 1, 32, 16),
                                            (7, 16, 4, 64, 3)])
def test_attn_fused_fc_o(B, S, H, D, n_out):
    """Pooled fc_o inside the attention kernels: forward logits zp = pool . W_o^T + b_o
    (heads summed in the workgroup) and backward dO = (dz . W_o) / S formed in-kernel,
    against torch fp32 and against the explicit-dO kernel path."""
    from collective_communication_mpi_amd import _native

    dev = _native.device()
    st = torch.cuda.current_stream().cuda_stream
    g = torch.Generator(device="cuda").manual_seed(B * 31 + D)
    qkv = (torch.randn(B * S, 3 * H * D, device="cuda", generator=g) * 0.5).bfloat16()
    lse = torch.empty(B * H, S, device="cuda")
    pool = torch.empty(B, H * D, device="cuda", dtype=torch.bfloat16)
    wo = (torch.randn(n_out, H * D, device="cuda", generator=g) * 0.1).bfloat16()
    bo = torch.randn(n_out, device="cuda", generator=g)
    zp = torch.full((B, 16), float("nan"), device="cuda")
    dev.attn_small_fwd(qkv.data_ptr(), 0, lse.data_ptr(), B, S, H, D, qkv.stride(0), H * D, D ** -0.5,
                       pool.data_ptr(), pool.stride(0), st, wo=wo.data_ptr(), ld_wo=wo.stride(0), n_out=n_out,
                       zp=zp.data_ptr(), ld_zp=zp.stride(0), bo=bo.data_ptr())
    ref_pool = _attn_ref(qkv, B, S, H, D).view(B, S, H * D).mean(1)
    torch.testing.assert_close(pool.float(), ref_pool, rtol=2e-2, atol=2e-2)
    ref_z = pool.float() @ wo.float().T + bo          # from the kernel's own bf16 pooled output
    torch.testing.assert_close(zp[:, :n_out], ref_z, rtol=1e-4, atol=1e-4)
    # backward: in-kernel dO vs the explicit broadcast dO the separate GEMM would produce
    dz = torch.randn(B, 16, device="cuda", generator=g).bfloat16()
    dpool = ((dz[:, :n_out].float() @ wo.float()) / S).bfloat16()
    d1, d2 = torch.empty_like(qkv), torch.empty_like(qkv)
    b1, b2 = torch.zeros(3 * H * D, device="cuda"), torch.zeros(3 * H * D, device="cuda")
    dev.attn_small_bwd(qkv.data_ptr(), 0, lse.data_ptr(), dpool.data_ptr(), d1.data_ptr(), b1.data_ptr(), B, S, H, D,
                       qkv.stride(0), H * D, D ** -0.5, dpool.stride(0), 0, st)
    dev.attn_small_bwd(qkv.data_ptr(), 0, lse.data_ptr(), 0, d2.data_ptr(), b2.data_ptr(), B, S, H, D,
                       qkv.stride(0), H * D, D ** -0.5, 0, 0, st, dz=dz.data_ptr(), ld_dz=dz.stride(0),
                       wo=wo.data_ptr(), ld_wo=wo.stride(0), n_out=n_out, dz_scale=1.0 / S)
    torch.cuda.synchronize()
    # dO rounding can differ in the last bf16 bit (fp32 summation order), nothing more
    torch.testing.assert_close(d2.float(), d1.float(), rtol=2e-2, atol=2e-2)
    assert (b2 - b1).norm() <= 1e-2 * b1.norm() + 1e-3


@pytest.mark.parametrize("B,S,H,D,n_out", [(2048, 16, 2, 64, 16), (2048, 16, 4, 64, 16), (37, 16, 1, 128, 10),
                                            (12, 9, 2, 32, 16)])
def test_attn_token_fc_o(B, S, H, D, n_out):
    """Per-token row-parallel fc_o inside the attention kernel: z[t] = bf16(O[t]) . W_o^T + b_o
    (heads summed in the workgroup, MFMA) against torch fp32 on the kernel's own O; the push
    form (row blocks stored write-through to per-block targets, here local buffers) writes
    bitwise the same rows; the pooled output is still produced."""
    from collective_communication_mpi_amd import _native

    dev = _native.device()
    st = torch.cuda.current_stream().cuda_stream
    g = torch.Generator(device="cuda").manual_seed(B * 7 + H)
    qkv = (torch.randn(B * S, 3 * H * D, device="cuda", generator=g) * 0.5).bfloat16()
    lse = torch.empty(B * H, S, device="cuda")
    o = torch.empty(B * S, H * D, device="cuda", dtype=torch.bfloat16)
    pool = torch.empty(B, H * D, device="cuda", dtype=torch.bfloat16)
    wo = torch.zeros(16, H * D, device="cuda").bfloat16()
    wo[:n_out] = (torch.randn(n_out, H * D, device="cuda", generator=g) * 0.1).bfloat16()
    bo = torch.zeros(16, device="cuda")
    bo[:n_out] = torch.randn(n_out, device="cuda", generator=g)
    z = torch.full((B * S, 16), float("nan"), device="cuda")
    kw = dict(wo=wo.data_ptr(), ld_wo=wo.stride(0), n_out=n_out, bo=bo.data_ptr(), ld_zt=16)
    dev.attn_small_fwd(qkv.data_ptr(), o.data_ptr(), lse.data_ptr(), B, S, H, D, qkv.stride(0), o.stride(0), D ** -0.5,
                       pool.data_ptr(), pool.stride(0), st, ztok=z.data_ptr(), **kw)
    ref_o = _attn_ref(qkv, B, S, H, D)
    torch.testing.assert_close(o.float(), ref_o, rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(pool.float(), ref_o.view(B, S, H * D).mean(1), rtol=2e-2, atol=2e-2)
    ref_z = o.float() @ wo[:n_out].float().T + bo[:n_out]
    torch.testing.assert_close(z[:, :n_out], ref_z, rtol=1e-4, atol=1e-4)
    assert torch.all(z[:, n_out:] == 0)
    # push form: blocks of whole sequences into separate targets
    blocks = 4 if B % 4 == 0 else 1
    zrows = B * S // blocks
    tg = torch.full((blocks, zrows, 16), float("nan"), device="cuda")
    dev.attn_small_fwd(qkv.data_ptr(), 0, lse.data_ptr(), B, S, H, D, qkv.stride(0), H * D, D ** -0.5,
                       pool.data_ptr(), pool.stride(0), st, zrows=zrows,
                       zpush=[tg[j].data_ptr() for j in range(blocks)], **kw)
    torch.cuda.synchronize()
    assert torch.equal(tg.view(B * S, 16), z)
    with pytest.raises(ValueError):  # a block boundary inside a sequence
        dev.attn_small_fwd(qkv.data_ptr(), 0, lse.data_ptr(), B, S, H, D, qkv.stride(0), H * D, D ** -0.5,
                           pool.data_ptr(), pool.stride(0), st, zrows=S + 1, zpush=[tg.data_ptr()], **kw)


@pytest.mark.parametrize("B,S,H,D,kp", [(2048, 16, 4, 64, 72), (2048, 16, 2, 64, 72), (37, 16, 1, 64, 64),
                                        (9, 7, 2, 32, 40), (5, 16, 4, 64, 8), (3001, 16, 4, 32, 72)])
def test_attn_qkv_fused(B, S, H, D, kp):
    """QKV projection + attention + per-token fc_o in one kernel (the harness forward):
    q | k | v = bf16(X W^T + b) against torch fp32 (stored when asked), then lse, pool and z
    against the unfused attention kernel run on that qkv; the push form bitwise equal."""
    from collective_communication_mpi_amd import _native

    dev = _native.device()
    st = torch.cuda.current_stream().cuda_stream
    g = torch.Generator(device="cuda").manual_seed(B * 13 + H * 5 + kp)
    HD = H * D
    xp = (torch.randn(B * S, kp, device="cuda", generator=g) * 0.5).bfloat16()
    w = (torch.randn(3 * HD, kp, device="cuda", generator=g) / kp ** 0.5).bfloat16()
    bq = torch.randn(3 * HD, device="cuda", generator=g) * 0.1
    wo = torch.zeros(16, HD, device="cuda").bfloat16()
    wo[:10] = (torch.randn(10, HD, device="cuda", generator=g) * 0.1).bfloat16()
    bo = torch.zeros(16, device="cuda")
    bo[:10] = torch.randn(10, device="cuda", generator=g)
    qkv = torch.full((B * S, 3 * HD), float("nan"), device="cuda").bfloat16()
    lse = torch.empty(B * H, S, device="cuda")
    pool = torch.empty(B, HD, device="cuda", dtype=torch.bfloat16)
    z = torch.full((B * S, 16), float("nan"), device="cuda")
    common = dict(lse=lse.data_ptr(), B=B, S=S, Hl=H, D=D, scale=D ** -0.5, pool=pool.data_ptr(), ld_pool=pool.stride(0),
                  wo=wo.data_ptr(), ld_wo=wo.stride(0), n_out=16, bo=bo.data_ptr(), ld_zt=16, stream=st)
    dev.attn_qkv_fwd(xq=xp.data_ptr(), ld_xq=xp.stride(0), kq=kp, wq=w.data_ptr(), ld_wq=w.stride(0), bq=bq.data_ptr(),
                     qkv_out=qkv.data_ptr(), ld_qkv=qkv.stride(0), ztok=z.data_ptr(), zrows=0, zpush=[], **common)
    ref_qkv = (xp.float() @ w.float().T + bq).bfloat16()
    torch.testing.assert_close(qkv.float(), ref_qkv.float(), rtol=1e-2, atol=1e-2)
    # the unfused kernel on the fused kernel's own qkv: same lse / pool; z up to fp32 summation
    # order and the fused softmax's hardware reciprocal (1 ulp in P can flip a bf16 rounding of P)
    lse2, pool2 = torch.empty_like(lse), torch.empty_like(pool)
    z2 = torch.empty_like(z)
    dev.attn_small_fwd(qkv.data_ptr(), 0, lse2.data_ptr(), B, S, H, D, qkv.stride(0), HD, D ** -0.5, pool2.data_ptr(),
                       pool2.stride(0), st, wo=wo.data_ptr(), ld_wo=wo.stride(0), n_out=16, bo=bo.data_ptr(),
                       ztok=z2.data_ptr(), ld_zt=16)
    torch.testing.assert_close(lse, lse2, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(pool.float(), pool2.float(), rtol=1e-2, atol=1e-2)
    torch.testing.assert_close(z, z2, rtol=1e-2, atol=2e-3)
    # push form into per-block targets: bitwise the same rows; no qkv written (inference)
    blocks = 2 if B % 2 == 0 else 1
    tg = torch.full((blocks, B * S // blocks, 16), float("nan"), device="cuda")
    qkv.fill_(float("nan"))
    dev.attn_qkv_fwd(xq=xp.data_ptr(), ld_xq=xp.stride(0), kq=kp, wq=w.data_ptr(), ld_wq=w.stride(0), bq=bq.data_ptr(),
                     qkv_out=0, ld_qkv=qkv.stride(0), ztok=0, zrows=B * S // blocks,
                     zpush=[tg[j].data_ptr() for j in range(blocks)], **common)
    torch.cuda.synchronize()
    assert torch.equal(tg.view(B * S, 16), z) and torch.isnan(qkv.float()).all()
    # local form: the token mean of z (+ bias) straight into the logits, z never stored
    zm = torch.full((B, 16), float("nan"), device="cuda")
    dev.attn_qkv_fwd(xq=xp.data_ptr(), ld_xq=xp.stride(0), kq=kp, wq=w.data_ptr(), ld_wq=w.stride(0), bq=bq.data_ptr(),
                     qkv_out=0, ld_qkv=qkv.stride(0), ztok=0, zrows=0, zpush=[], zmean=zm.data_ptr(), ld_zmean=16,
                     **common)
    torch.cuda.synchronize()
    torch.testing.assert_close(zm, z.view(B, S, 16).mean(dim=1), rtol=1e-5, atol=1e-5)
    with pytest.raises(ValueError):  # beyond the register-resident weight + bias columns: kq > 72
        dev.attn_qkv_fwd(xq=xp.data_ptr(), ld_xq=xp.stride(0), kq=80, wq=w.data_ptr(), ld_wq=w.stride(0),
                         bq=bq.data_ptr(), qkv_out=0, ld_qkv=qkv.stride(0), ztok=z.data_ptr(), zrows=0, zpush=[],
                         **common)


@pytest.mark.parametrize("B,H,D", [(2048, 4, 64), (2048, 2, 64), (37, 1, 64), (301, 4, 32)])
def test_attn_qkv_fused_patchify(B, H, D):
    """Fused patchify: the kernel builds the MNIST patch rows from the fp32 images itself --
    the rows it stores for the backward are bitwise k_patchify's, and qkv / lse / pool / z are
    bitwise those of the same kernel reading k_patchify's rows."""
    from collective_communication_mpi_amd import _native

    dev = _native.device()
    st = torch.cuda.current_stream().cuda_stream
    g = torch.Generator(device="cuda").manual_seed(B + H)
    S, kp, HD = 16, 72, H * D
    img = torch.rand(B, 784, device="cuda", generator=g)
    xp = torch.empty(B * S, kp, device="cuda", dtype=torch.bfloat16)
    dev.patchify(img.data_ptr(), xp.data_ptr(), B, 28, 7, kp, st, kp)
    w = (torch.randn(3 * HD, kp, device="cuda", generator=g) / kp ** 0.5).bfloat16()
    bq = torch.randn(3 * HD, device="cuda", generator=g) * 0.1
    wo = (torch.randn(16, HD, device="cuda", generator=g) * 0.1).bfloat16()
    bo = torch.randn(16, device="cuda", generator=g)
    outs = []
    for mode in ("rows", "img"):
        qkv = torch.full((B * S, 3 * HD), float("nan"), device="cuda").bfloat16()
        lse = torch.empty(B * H, S, device="cuda")
        pool = torch.empty(B, HD, device="cuda", dtype=torch.bfloat16)
        z = torch.full((B * S, 16), float("nan"), device="cuda")
        xo = torch.full((B * S, kp), float("nan"), device="cuda").bfloat16()
        dev.attn_qkv_fwd(xq=xp.data_ptr() if mode == "rows" else 0, ld_xq=kp, kq=kp, wq=w.data_ptr(),
                         ld_wq=w.stride(0), bq=bq.data_ptr(), qkv_out=qkv.data_ptr(), ld_qkv=qkv.stride(0),
                         lse=lse.data_ptr(), B=B, S=S, Hl=H, D=D, scale=D ** -0.5, pool=pool.data_ptr(),
                         ld_pool=pool.stride(0), wo=wo.data_ptr(), ld_wo=wo.stride(0), n_out=16, bo=bo.data_ptr(),
                         ztok=z.data_ptr(), ld_zt=16, zrows=0, zpush=[], stream=st,
                         img=img.data_ptr() if mode == "img" else 0, xq_out=xo.data_ptr() if mode == "img" else 0)
        outs.append((qkv, lse, pool, z, xo))
    torch.cuda.synchronize()
    (q0, l0, p0, z0, _), (q1, l1, p1, z1, xo) = outs
    assert torch.equal(xo, xp)
    assert torch.equal(q0, q1) and torch.equal(l0, l1) and torch.equal(p0, p1) and torch.equal(z0, z1)
    with pytest.raises(ValueError):  # image mode is the 16-token MNIST case
        dev.attn_qkv_fwd(xq=0, ld_xq=kp, kq=kp, wq=w.data_ptr(), ld_wq=w.stride(0), bq=bq.data_ptr(), qkv_out=0,
                         ld_qkv=3 * HD, lse=l0.data_ptr(), B=B, S=9, Hl=H, D=D, scale=1.0, pool=p0.data_ptr(),
                         ld_pool=HD, wo=wo.data_ptr(), ld_wo=HD, n_out=16, bo=0, ztok=z0.data_ptr(), ld_zt=16,
                         zrows=0, zpush=[], stream=st, img=img.data_ptr())


@pytest.mark.parametrize("B,H", [(2048, 2), (2048, 4), (1000, 2), (512, 2), (37, 1)])
def test_attn_qkv_fold_schedule(B, H):
    """The fused forward's in-kernel weight fold (the pipelined plan's) with the fold-aware block
    schedule -- fold-owning workgroups take fewer pair blocks; at B = 1000 and 512 (the DP4 x TP2
    per-rank shape) / H = 2 the grid grows by the fold's tiles and their workgroups take none --
    against plain grid-stride and against the forward without the fold: token-mean logits bitwise
    equal, and the folded W_eff bitwise the standalone fp32-MFMA fold kernel's."""
    from collective_communication_mpi_amd import _native

    dev = _native.device()
    st = torch.cuda.current_stream().cuda_stream
    g = torch.Generator(device="cuda").manual_seed(B * 7 + H)
    S, kp, D = 16, 72, 64
    HD = H * D
    img = torch.rand(B, 784, device="cuda", generator=g)
    w = (torch.randn(3 * HD, kp, device="cuda", generator=g) / kp ** 0.5).bfloat16()
    bq = torch.randn(3 * HD, device="cuda", generator=g) * 0.1
    wo = (torch.randn(16, HD, device="cuda", generator=g) * 0.1).bfloat16()
    bo = torch.randn(16, device="cuda", generator=g)
    wq32 = torch.randn(3 * HD, 768, device="cuda", generator=g) / 768 ** 0.5
    we32 = torch.randn(768, kp, device="cuda", generator=g) / 8
    outs = {}
    try:
        for sched in (0, 1, None):
            zm = torch.full((B, 16), float("nan"), device="cuda")
            wn = torch.full((3 * HD, kp), float("nan"), device="cuda").bfloat16()
            kw = dict(xq=0, ld_xq=kp, kq=kp, wq=w.data_ptr(), ld_wq=w.stride(0), bq=bq.data_ptr(), qkv_out=0,
                      ld_qkv=3 * HD, lse=0, B=B, S=S, Hl=H, D=D, scale=D ** -0.5, pool=0, ld_pool=HD,
                      wo=wo.data_ptr(), ld_wo=wo.stride(0), n_out=16, bo=bo.data_ptr(), ztok=0, ld_zt=16, zrows=0,
                      zpush=[], zmean=zm.data_ptr(), ld_zmean=16, stream=st, img=img.data_ptr())
            if sched is not None:
                kw.update(fold_wq=wq32.data_ptr(), ld_fold_wq=768, fold_we=we32.data_ptr(), ld_fold_we=kp,
                          fold_out=wn.data_ptr(), ld_fold_out=kp, fold_R=3 * HD, fold_d=768)
            dev.attn_set_qkv_fold_sched(-1 if sched is None else sched)
            dev.attn_qkv_fwd(**kw)
            outs[sched] = (zm, wn)
    finally:
        dev.attn_set_qkv_fold_sched(-1)
    ref = torch.full((3 * HD, kp), float("nan"), device="cuda").bfloat16()
    dev.fold_set_variant(1)
    try:
        dev.fold_emb_qkv(wq32.data_ptr(), 768, we32.data_ptr(), kp, ref.data_ptr(), kp, 3 * HD, 768, kp, st)
    finally:
        dev.fold_set_variant(-1)
    torch.cuda.synchronize()
    (z0, w0), (z1, w1), (zn, _) = outs[0], outs[1], outs[None]
    assert not torch.isnan(z1).any()
    assert torch.equal(z0, z1) and torch.equal(z0, zn)
    assert torch.equal(w0, w1) and torch.equal(w1, ref)


@pytest.mark.parametrize("img,patch,misalign", [(28, 7, 0), (28, 7, 1), (24, 6, 0)])  # LDS / plain / runtime sizes
def test_patchify_columns(img, patch, misalign):
    from collective_communication_mpi_amd.models.mnist_tp import LayerConfig, patchify

    cfg = LayerConfig(img=img, patch=patch)
    x = torch.rand(5 * img * img + misalign, device="cuda")[misalign:].view(5, img * img)
    xp = patchify(x, cfg).float()
    g = cfg.img // cfg.patch
    ref = x.view(5, g, cfg.patch, g, cfg.patch).permute(0, 1, 3, 2, 4).reshape(5 * g * g, cfg.pixels)
    torch.testing.assert_close(xp[:, : cfg.pixels], ref.bfloat16().float())
    assert torch.all(xp[:, cfg.pixels] == 1)
    onehot = xp[:, cfg.pixels + 1:cfg.pixels + 1 + cfg.seq]
    torch.testing.assert_close(onehot, torch.eye(cfg.seq, device="cuda").repeat(5, 1))
    assert torch.all(xp[:, cfg.pixels + 1 + cfg.seq:] == 0)


def test_embed_patches_fused_matches_patchify_gemm():
    """Patch rows generated inside the small-K GEMM (and stored to xp) == patchify, then the GEMM."""
    from collective_communication_mpi_amd import _native
    from collective_communication_mpi_amd.models.mnist_tp import LayerConfig, patchify
    from collective_communication_mpi_amd.ops import gemm_nt

    cfg = LayerConfig()
    B, d = 37, cfg.d_model  # M = 592: a partial last M tile
    x = torch.rand(B, 784, device="cuda")
    w = (torch.randn(d, cfg.kp, device="cuda") * 0.2).bfloat16()
    ld = d + cfg.kp + 56  # [h | xp] rows, 16-B aligned
    hx = torch.full((B * cfg.seq, ld), float("nan"), device="cuda").bfloat16()
    h, xp = hx[:, :d], hx[:, d:d + cfg.kp]
    _native.device().embed_patches(x.data_ptr(), w.data_ptr(), h.data_ptr(), B, cfg.img, cfg.patch, d, cfg.kp,
                                   w.stride(0), h.stride(0), xp.data_ptr(), xp.stride(0),
                                   torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    xp_ref = patchify(x, cfg)
    assert torch.equal(xp, xp_ref)
    torch.testing.assert_close(h.float(), gemm_nt(xp_ref, w).float(), rtol=1e-2, atol=1e-2)
    torch.testing.assert_close(h.float(), xp_ref.float() @ w.float().t(), rtol=2e-2, atol=3e-2)
    assert torch.isnan(hx[:, d + cfg.kp:].float()).all()  # padding columns untouched


@pytest.mark.parametrize("n", [1000, 1003, 650001])
def test_fused_adamw_matches_torch(n):
    from collective_communication_mpi_amd.parallel.dp import FlatParams

    fp = FlatParams([("w", (n,))], "cuda")
    w0 = torch.randn(n, device="cuda")
    fp.param("w").copy_(w0)
    ref = torch.nn.Parameter(w0.clone())
    opt = torch.optim.AdamW([ref], lr=1e-2, weight_decay=0.1, eps=1e-8)
    for _ in range(3):
        g = torch.randn(n, device="cuda")
        fp.grad("w").copy_(g * 2)
        fp.adamw(1e-2, weight_decay=0.1, grad_scale=0.5)  # grad_scale folds a 1/dp average
        ref.grad = g
        opt.step()
        assert torch.all(fp.grad("w") == 0)  # the kernel zeroes what it consumed
    torch.testing.assert_close(fp.param("w"), ref.detach(), rtol=1e-5, atol=1e-6)
    # the bf16 copy is the rounding of the kernel's own fp32 result (against torch's, values
    # within 1e-7 of a bf16 rounding boundary may land one bf16 ulp apart at this n)
    assert torch.equal(fp.param16("w"), fp.param("w").bfloat16())


@pytest.mark.parametrize("ydtype", [torch.int32, torch.int64])
@pytest.mark.parametrize("C,Cp", [(10, 16), (5, 8), (20, 32)])  # lane-per-class kernel (<= 16) and row kernel
def test_xent_head_fused(ydtype, C, Cp):
    """Fused softmax cross-entropy head vs torch (loss, dZ incl. zero padding, d bias)."""
    from collective_communication_mpi_amd import _native

    B, gb = 777, 3000
    z = torch.randn(B, Cp, device="cuda") * 3
    bias = torch.randn(Cp, device="cuda")
    y = torch.randint(0, C, (B,), device="cuda").to(ydtype)
    loss = torch.empty(1, device="cuda")
    dz = torch.full((B, Cp), 7.0, device="cuda").bfloat16()
    db = torch.ones(Cp, device="cuda")
    ws = torch.zeros(1 + (B + 15) // 16, device="cuda")  # ticket + partials (lane-per-class kernel)
    for it in range(2):  # the second call checks that the kernel re-armed its ticket
        db_in = db.clone()
        _native.device().xent_head(z.data_ptr(), z.stride(0), bias.data_ptr(), y.data_ptr(), ydtype == torch.int64, B,
                                   C, Cp, 1.0 / gb, loss.data_ptr(), dz.data_ptr(), dz.stride(0), db.data_ptr(),
                                   torch.cuda.current_stream().cuda_stream, ws.data_ptr())
        if it == 0:
            first = loss.clone()
    torch.testing.assert_close(loss, first)
    logits = (z[:, :C] + bias[:C]).requires_grad_(True)
    ref = torch.nn.functional.cross_entropy(logits, y.long(), reduction="sum") / gb
    ref.backward()
    torch.testing.assert_close(loss[0], ref.detach(), rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(dz[:, :C].float(), logits.grad, rtol=1e-2, atol=1e-5)
    assert torch.all(dz[:, C:] == 0)
    gsum = logits.grad.sum(0)
    torch.testing.assert_close(db_in[:C], 1 + gsum, rtol=1e-4, atol=1e-6)   # after one call
    torch.testing.assert_close(db[:C], 1 + 2 * gsum, rtol=1e-4, atol=1e-6)  # after two
    torch.testing.assert_close(db[C:], torch.ones(Cp - C, device="cuda"))


@pytest.mark.parametrize("B,HD,C,Cp", [(777, 256, 10, 16), (2048, 128, 10, 16), (130, 100, 5, 8)])
@pytest.mark.parametrize("ydtype", [torch.int32, torch.int64])
def test_xent_head_wo_fused(B, HD, C, Cp, ydtype):
    """Loss head + dW_o = dZ^T pool in one launch vs torch: loss, bf16 dZ (zero padding), d bias,
    and dW_o accumulated into a non-zero buffer from the bf16 dZ and pool."""
    from collective_communication_mpi_amd import _native

    gb = 3000
    g = torch.Generator(device="cuda").manual_seed(B + HD)
    z = torch.randn(B, Cp, device="cuda", generator=g) * 3
    y = torch.randint(0, C, (B,), device="cuda", generator=g).to(ydtype)
    pool = torch.randn(B, HD, device="cuda", generator=g).bfloat16()
    loss = torch.empty(1, device="cuda")
    dz = torch.full((B, Cp), 7.0, device="cuda").bfloat16()
    db = torch.ones(Cp, device="cuda")
    dwo = torch.full((Cp, HD + 4), 0.5, device="cuda")  # padded rows: ld > HD
    ws = torch.zeros(1 + (B + 63) // 64, device="cuda")
    for _ in range(2):  # the second call checks the re-armed ticket
        _native.device().xent_head_wo(z.data_ptr(), z.stride(0), y.data_ptr(), ydtype == torch.int64, B, C, Cp, 1.0 / gb,
                                      loss.data_ptr(), dz.data_ptr(), dz.stride(0), db.data_ptr(), pool.data_ptr(),
                                      pool.stride(0), HD, dwo.data_ptr(), dwo.stride(0),
                                      torch.cuda.current_stream().cuda_stream, ws.data_ptr())
    torch.cuda.synchronize()
    logits = z[:, :C].clone().requires_grad_(True)
    ref = torch.nn.functional.cross_entropy(logits, y.long(), reduction="sum") / gb
    ref.backward()
    torch.testing.assert_close(loss[0], ref.detach(), rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(dz[:, :C].float(), logits.grad, rtol=1e-2, atol=1e-5)
    assert torch.all(dz[:, C:] == 0)
    torch.testing.assert_close(db[:C], 1 + 2 * logits.grad.sum(0), rtol=1e-4, atol=1e-6)
    torch.testing.assert_close(db[C:], torch.ones(Cp - C, device="cuda"))
    wref = dz[:, :C].float().T @ pool.float()  # from the bf16 gradient the kernel stores
    torch.testing.assert_close(dwo[:C, :HD], 0.5 + 2 * wref, rtol=1e-4, atol=1e-5)
    assert torch.all(dwo[C:] == 0.5) and torch.all(dwo[:, HD:] == 0.5)


def test_flat_params_transposed_copies():
    """Fused AdamW / cast keep W^T bf16 copies in sync with the flat master weights."""
    from collective_communication_mpi_amd.parallel.dp import FlatParams

    f = FlatParams([("a", (48, 80)), ("b", (7,)), ("c", (33, 16))], "cuda", transposed=("a", "c"))
    f.p32.copy_(torch.randn(f.numel, device="cuda"))
    f.refresh_bf16()
    for nm in ("a", "c"):
        torch.testing.assert_close(f.param16_t(nm), f.param16(nm).T)
    f.g.copy_(torch.randn(f.numel, device="cuda"))
    f.adamw(1e-2, weight_decay=0.1)
    for nm in ("a", "c"):
        torch.testing.assert_close(f.param16_t(nm), f.param16(nm).T)
        torch.testing.assert_close(f.param16(nm).float(), f.param(nm), rtol=1e-2, atol=1e-2)


@pytest.mark.parametrize("M,N1,N2", [(32768, 768, 768), (4096, 512, 1024), (1024, 296, 520), (256, 256, 256)])
@pytest.mark.parametrize("splitk", [None, 1, 3])
def test_gemm_tn_pingpong(M, N1, N2, splitk):
    """256x256 ping-pong TN kernel (transposed LDS reads, workspace split-K)."""
    from collective_communication_mpi_amd.ops import gemm_tn
    from collective_communication_mpi_amd.ops.kernels import set_tn_variant

    g = torch.Generator(device="cuda").manual_seed(M + 3 * N1 + N2)
    a = torch.randn(M, N1, device="cuda", generator=g).bfloat16()
    b = torch.randn(M, N2, device="cuda", generator=g).bfloat16()
    ref = a.float().T @ b.float()
    set_tn_variant(1)
    try:
        out = gemm_tn(a, b, splitk=splitk)
        torch.testing.assert_close(out, ref, rtol=2e-3, atol=2e-3 * M ** 0.5)
        acc = torch.ones(N1, N2, device="cuda")
        gemm_tn(a, b, out=acc, accumulate=True, alpha=0.5, splitk=splitk)
        torch.testing.assert_close(acc, 1 + 0.5 * ref, rtol=2e-3, atol=2e-3 * M ** 0.5)
    finally:
        set_tn_variant(None)


@pytest.mark.parametrize("ge_mfma", [True, False], ids=["ge-mfma", "ge-atomic"])
@pytest.mark.parametrize("R,d,kp", [(768, 768, 72), (384, 768, 72), (20, 36, 16), (50, 1000, 8), (1000, 64, 16)])
def test_emb_qkv_wgrad_matches_fp32(R, d, kp, ge_mfma):
    """The harness's weight-gradient kernel: Gq += A We^T, Ge += Wq^T A (matrix-core tiles over
    all R rows, or R-split atomic tiles; R = 1000 exceeds the matrix-core path and takes the
    atomic one), Z zeroed -- against fp32 torch."""
    from collective_communication_mpi_amd import _native

    g = torch.Generator(device="cuda").manual_seed(R + d + kp)
    A = torch.randn(R, kp, device="cuda", generator=g)
    We = torch.randn(d, kp, device="cuda", generator=g)
    Wq = torch.randn(R, d, device="cuda", generator=g)
    Gq = torch.randn(R, d, device="cuda", generator=g)
    Ge = torch.randn(d, kp + 4, device="cuda", generator=g)  # padded rows
    Z = torch.ones(R, kp, device="cuda")
    gq_ref = Gq + A @ We.T
    ge_ref = Ge[:, :kp] + Wq.T @ A
    D = _native.device()
    D.wgrad_set_ge_mfma(ge_mfma)
    try:
        D.emb_qkv_wgrad(A.data_ptr(), A.stride(0), We.data_ptr(), We.stride(0), Wq.data_ptr(), Wq.stride(0),
                        Gq.data_ptr(), Gq.stride(0), Ge.data_ptr(), Ge.stride(0), Z.data_ptr(), Z.stride(0), R, d, kp,
                        torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
    finally:
        D.wgrad_set_ge_mfma(True)
    tol = dict(rtol=1e-4, atol=1e-3 * max(R, d) ** 0.5)
    torch.testing.assert_close(Gq, gq_ref, **tol)
    torch.testing.assert_close(Ge[:, :kp], ge_ref, **tol)
    assert torch.all(Z == 0)


@pytest.mark.parametrize("variant", [0, 1], ids=["fma", "mfma"])
@pytest.mark.parametrize("R,d,kp", [(768, 768, 72), (384, 768, 72), (20, 36, 16), (7, 100, 96), (50, 1000, 8)])
def test_fold_emb_qkv_matches_fp32(R, d, kp, variant):
    """W_eff = W_qkv . W_emb (+ bias in one column) against torch fp64, incl. ragged
    row / column / k edges and strided operands (fp32 FMA kernel and fp32 MFMA kernel,
    both fixed order)."""
    from collective_communication_mpi_amd import _native

    _native.device().fold_set_variant(variant)
    try:
        _fold_check(R, d, kp)
    finally:
        _native.device().fold_set_variant(-1)


def _fold_check(R, d, kp):
    from collective_communication_mpi_amd import _native

    torch.manual_seed(R + d)
    wq = torch.randn(R, d + 4, device="cuda")[:, :d]
    we = torch.randn(d, kp + 8, device="cuda")[:, :kp]
    bias = torch.randn(R, device="cuda")
    bcol = kp // 2
    out = torch.full((R, kp + 8), float("nan"), device="cuda").bfloat16()
    dev = _native.device()
    dev.fold_emb_qkv(wq.data_ptr(), wq.stride(0), we.data_ptr(), we.stride(0), out.data_ptr(), out.stride(0), R, d,
                     kp, torch.cuda.current_stream().cuda_stream, bias=bias.data_ptr(), bias_col=bcol)
    torch.cuda.synchronize()
    ref = wq.double() @ we.double()
    ref[:, bcol] += bias.double()
    torch.testing.assert_close(out[:, :kp].double(), ref, rtol=8e-3, atol=8e-3 * ref.abs().max().item())
    assert torch.isnan(out[:, kp:].float()).all()  # columns past kp untouched


@pytest.mark.parametrize("route", ["transpose", "ring", "pair"])
@pytest.mark.parametrize("ta,tb", [(0, 1), (1, 1), (1, 0)], ids=["kA-tB", "tA-tB", "tA-kB"])
def test_gemm_ring_kmajor_routes(monkeypatch, route, ta, tb):
    """A large K-major GEMM every way: transposed copies + the N-layout pair ring, the
    K-major operands read straight by the pair ring (TA / TB forms: no transposes), and the
    4-slot K-major ring; fp32 reference, bf16 out with alpha, and fp32 accumulate (the DDP
    gradient-sink forms)."""
    from collective_communication_mpi_amd import _native
    from collective_communication_mpi_amd.ops import gemm_ring

    monkeypatch.setenv("CCMPI_KMAJOR_ROUTE", route)
    if route == "pair":
        _native.device().gemm_set_pair_ta(1)  # the (1, 0) form on the pair ring too
    M, N, K = 2048, 2048, 2048
    g = torch.Generator(device="cuda").manual_seed(17 + ta + 2 * tb)
    a = torch.randn(K, M, device="cuda", generator=g).bfloat16() if ta else torch.randn(M, K, device="cuda", generator=g).bfloat16()
    b = torch.randn(K, N, device="cuda", generator=g).bfloat16() if tb else torch.randn(N, K, device="cuda", generator=g).bfloat16()
    ref = (a.float().T if ta else a.float()) @ (b.float().T if tb else b.float()).T
    n0 = _native.device().gemm_ring_launches()
    y16 = gemm_ring(a, b, bool(ta), bool(tb), alpha=0.5)
    assert _native.device().gemm_ring_launches() == n0 + 1
    torch.testing.assert_close(y16.float(), 0.5 * ref, rtol=1.6e-2, atol=1.6e-2 * K ** 0.5)
    c = torch.randn(M, N, device="cuda")
    c0 = c.clone()
    gemm_ring(a, b, bool(ta), bool(tb), out=c, accumulate=True)
    _native.device().gemm_set_pair_ta(0)
    torch.testing.assert_close(c, c0 + ref, rtol=2e-3, atol=2e-3 * K ** 0.5)


@pytest.mark.parametrize("ta,tb", [(0, 0), (0, 1), (1, 1), (1, 0)], ids=["kA-kB", "kA-tB", "tA-tB", "tA-kB"])
@pytest.mark.parametrize("M,N,K", [(256, 256, 64), (300, 520, 256), (776, 1000, 512), (2048, 1024, 1024),
                                   (8, 8, 192), (1, 8, 192)])
def test_gemm_ring_layouts(ta, tb, M, N, K):
    """LDS-ring kernel with K-major operands (dX = dY W, dW = dY^T X without transposes)
    against an fp32 reference: fp32 out (generic epilogue), bf16 out (fast epilogue),
    accumulate."""
    from collective_communication_mpi_amd.ops import gemm_ring

    g = torch.Generator(device="cuda").manual_seed(M + 3 * N + 7 * K + 11 * ta + 13 * tb)
    a = torch.randn(K, M, device="cuda", generator=g).bfloat16() if ta else torch.randn(M, K, device="cuda", generator=g).bfloat16()
    b = torch.randn(K, N, device="cuda", generator=g).bfloat16() if tb else torch.randn(N, K, device="cuda", generator=g).bfloat16()
    opa = a.float().T if ta else a.float()
    opb = b.float().T if tb else b.float()
    ref = opa @ opb.T
    y = gemm_ring(a, b, bool(ta), bool(tb), out_dtype=torch.float32)
    if (ta and M % 8) or (tb and N % 8) or (not ta and K % 8):
        assert y is None  # K-major rows must be 16-B multiples: the caller falls back
        return
    assert y is not None
    torch.testing.assert_close(y, ref, rtol=2e-3, atol=2e-3 * K ** 0.5)
    y16 = gemm_ring(a, b, bool(ta), bool(tb), alpha=0.5)
    torch.testing.assert_close(y16.float(), (0.5 * y).bfloat16().float(), rtol=1e-2, atol=1e-2)
    c = torch.randn(M, N, device="cuda")
    c0 = c.clone()
    gemm_ring(a, b, bool(ta), bool(tb), out=c, accumulate=True)
    torch.testing.assert_close(c, c0 + ref, rtol=2e-3, atol=5e-2)


@pytest.mark.parametrize("T,k", [(1, 8), (7, 24), (4096, 1792), (3, 2056), (513, 14336 // 8)])
def test_swiglu_fwd_bwd_vs_fp32(T, k):
    """Fused SwiGLU kernels (csrc/device/swiglu.hip) against fp32 autograd of silu(g) * u."""
    from collective_communication_mpi_amd.ops import swiglu

    g = torch.Generator(device="cuda").manual_seed(T * 31 + k)
    h = (torch.randn(T, 2 * k, device="cuda", generator=g) * 3).bfloat16().requires_grad_(True)
    da = torch.randn(T, k, device="cuda", generator=g).bfloat16()
    a = swiglu(h)
    a.backward(da)
    hf = h.detach().float().requires_grad_(True)
    ref = torch.nn.functional.silu(hf[:, :k]) * hf[:, k:]
    ref.backward(da.float())
    assert a.dtype == torch.bfloat16 and a.shape == (T, k)
    torch.testing.assert_close(a.float(), ref, rtol=1.6e-2, atol=1e-2)
    torch.testing.assert_close(h.grad.float(), hf.grad, rtol=1.6e-2, atol=2e-2)


def test_swiglu_strided_and_batched():
    """3-D input and a row-strided view (the gate|up slice of a wider buffer) take the kernel."""
    from collective_communication_mpi_amd.ops import swiglu

    g = torch.Generator(device="cuda").manual_seed(5)
    wide = torch.randn(2, 64, 3 * 128, device="cuda", generator=g).bfloat16()
    h = wide[..., :256]  # row stride 384 elements, 16-B aligned
    ref = torch.nn.functional.silu(h[..., :128].float()) * h[..., 128:].float()
    torch.testing.assert_close(swiglu(h).float(), ref, rtol=1.6e-2, atol=1e-2)


@pytest.mark.parametrize("ring", [8, 8 | 16384, 9 | 16384], ids=["ring", "pair", "pairp"])
@pytest.mark.parametrize("M,N,K", [(4096, 2048, 512), (300, 520, 128), (1000, 2056, 64), (257, 264, 192)])
def test_gemm_nt_swiglu_epilogue(M, N, K, ring):
    """Ring GEMM with the SwiGLU gate of interleaved column pairs in its epilogue (EPI 2):
    h = A B^T vs fp32, gate vs silu / mul of the bf16 h, edge tiles in M and N; the
    4-slot ring and the pair-slot ring (whole-line DMA pieces)."""
    from collective_communication_mpi_amd import _native
    from collective_communication_mpi_amd.ops import gemm_nt_swiglu

    D = _native.device()
    D.gemm_set_ring_sched(ring)
    try:
        _swiglu_epilogue_check(M, N, K, gemm_nt_swiglu)
    finally:
        D.gemm_set_ring_sched(8 | 16384)


def _swiglu_epilogue_check(M, N, K, gemm_nt_swiglu):

    g = torch.Generator(device="cuda").manual_seed(M + N + K)
    a = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    b = (torch.randn(N, K, device="cuda", generator=g) / K ** 0.5).bfloat16()
    h = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    glu = torch.empty(M, N // 2, device="cuda", dtype=torch.bfloat16)
    assert gemm_nt_swiglu(a, b, h, glu), "the ring kernel's fast form should apply"
    torch.testing.assert_close(h.float(), _ref(a, b), rtol=1.6e-2, atol=2e-2)
    hf = h.float()
    ref = torch.nn.functional.silu(hf[:, 0::2]) * hf[:, 1::2]
    torch.testing.assert_close(glu.float(), ref, rtol=1.6e-2, atol=1e-2)


@pytest.mark.parametrize("T,k", [(8, 4), (4096, 1024), (200, 36), (72, 1000)])
def test_swiglu_pairs_backward_transposed(T, k):
    """The SwiGLU backward that also writes dh^T (for dW on the N-layout ring): both outputs
    bitwise equal to the plain kernel's dh and its transpose; partial tiles both ways."""
    from collective_communication_mpi_amd.ops import swiglu_pairs_backward

    g = torch.Generator(device="cuda").manual_seed(T + k)
    h = torch.randn(T, 2 * k, device="cuda", generator=g).bfloat16()
    da = torch.randn(T, k, device="cuda", generator=g).bfloat16()
    ref = swiglu_pairs_backward(h, da)
    dh, dht = swiglu_pairs_backward(h, da, transposed=True)
    torch.testing.assert_close(dh, ref, rtol=0, atol=0)
    torch.testing.assert_close(dht, ref.T, rtol=0, atol=0)


def test_swiglu_pairs_fwd_bwd():
    from collective_communication_mpi_amd.ops import swiglu_pairs, swiglu_pairs_backward

    g = torch.Generator(device="cuda").manual_seed(9)
    h = (torch.randn(777, 2 * 1028, device="cuda", generator=g) * 3).bfloat16()
    da = torch.randn(777, 1028, device="cuda", generator=g).bfloat16()
    hf = h.float().requires_grad_(True)
    ref = torch.nn.functional.silu(hf[:, 0::2]) * hf[:, 1::2]
    ref.backward(da.float())
    torch.testing.assert_close(swiglu_pairs(h).float(), ref.detach(), rtol=1.6e-2, atol=1e-2)
    torch.testing.assert_close(swiglu_pairs_backward(h, da).float(), hf.grad, rtol=1.6e-2, atol=2e-2)


def test_gemm_nt_long_k_dispatch():
    """Long K over at most one 256x256 tile per CU: gemm_nt auto takes the 256x256 kernel
    (gemm.hip dispatch, profiles/r3_swiglu/gemm_sweep.txt); numerics vs fp32."""
    from collective_communication_mpi_amd.ops import gemm_nt

    g = torch.Generator(device="cuda").manual_seed(77)
    M, N, K = 1024, 1280, 16512
    a = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    b = (torch.randn(N, K, device="cuda", generator=g) / K ** 0.5).bfloat16()
    y = gemm_nt(a, b, out_dtype=torch.bfloat16)
    torch.testing.assert_close(y.float(), _ref(a, b), rtol=1.6e-2, atol=2e-2)


@pytest.mark.parametrize("groups,S,ncol,ld", [(2048, 16, 16, 16), (7, 9, 8, 12), (1, 1, 4, 4)])
def test_rows_mean_ordered(groups, S, ncol, ld):
    """Token mean of the per-token logits (k_rows_mean): the in-order fp32 sum / S -- the
    order DeviceComm.inbox_mean uses, so the plain and push TP forms agree bitwise."""
    from collective_communication_mpi_amd import _native

    z = torch.randn(groups * S, ld, device="cuda")
    out = torch.full((groups, ld + 4), float("nan"), device="cuda")
    _native.device().rows_mean(z.data_ptr(), ld, out.data_ptr(), out.stride(0), groups, S, ncol,
                               torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    zz = z.view(groups, S, ld)[:, :, :ncol]
    ref = torch.zeros(groups, ncol, device="cuda")
    for i in range(S):
        ref = ref + zz[:, i]
    # (a tensor divisor: torch turns division by a Python scalar into a reciprocal multiply)
    assert torch.equal(out[:, :ncol], ref / torch.full_like(ref, float(S)))
    assert torch.isnan(out[:, ncol:]).all()
