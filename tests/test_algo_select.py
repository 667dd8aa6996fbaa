"""`auto` all-reduce selection (DeviceGroup.pick_allreduce): size classes
(LL -> one-shot -> fan-out), group-size-dependent thresholds, tuned overrides,
and the fall-through past algorithms that failed self_test() / were disabled.
Host-only: the method is exercised on a stand-in object, no GPU needed."""
from types import SimpleNamespace

from collective_communication_mpi_amd.device import DeviceGroup


def group(size=8, disabled=(), tuned=None):
    return SimpleNamespace(size=size, tuned=tuned or {}, ll_auto_max=(256 << 10) if size <= 2 else (64 << 10),
                           oneshot_max=(1 << 20) if size <= 2 else (64 << 10), disabled=set(disabled))


def pick(g, n):
    return DeviceGroup.pick_allreduce(g, n)


def test_size_classes(monkeypatch):
    monkeypatch.delenv("CCMPI_ALLREDUCE_ALGO", raising=False)
    g = group(8)
    assert pick(g, 4096) == "ll"
    assert pick(g, 4100) == "oneshot"          # not a 16-B multiple: no LL
    assert pick(g, 1 << 20) == "fanout"
    assert pick(g, 1 << 30) == "fanout"
    g2 = group(2)
    assert pick(g2, 128 << 10) == "ll"
    assert pick(g2, 512 << 10) == "oneshot"
    assert pick(g2, 4 << 20) == "fanout"
    assert pick(group(1), 1 << 20) == "twoshot"  # single rank: a copy


def test_disabled_fall_through(monkeypatch):
    monkeypatch.delenv("CCMPI_ALLREDUCE_ALGO", raising=False)
    assert pick(group(8, {"ll"}), 4096) == "oneshot"
    assert pick(group(8, {"ll", "oneshot"}), 4096) == "fanout"
    assert pick(group(8, {"fanout"}), 1 << 30) == "twoshot"
    assert pick(group(8, {"ll", "oneshot", "fanout", "twoshot", "reduce_bcast"}), 4096) == "rccl"


def test_tuned_and_forced(monkeypatch):
    monkeypatch.delenv("CCMPI_ALLREDUCE_ALGO", raising=False)
    g = group(4, tuned={(4, 20): "twoshot"})
    assert pick(g, 1 << 20) == "twoshot"
    monkeypatch.setenv("CCMPI_ALLREDUCE_ALGO", "push")
    assert pick(group(4), 1 << 24) == "push"


def test_tuning_file_roundtrip(tmp_path):
    from collective_communication_mpi_amd.device import load_tuning, save_tuning, tuning_key

    path = str(tmp_path / "tune.json")
    k8 = tuning_key(8, 1, "AMD Instinct MI355X")
    k2 = tuning_key(2, 2, "AMD Instinct MI355X")
    assert load_tuning(path, k8) == {}  # no file yet
    save_tuning(path, k8, {(8, 20): "fanout", (8, 12): "ll"})
    save_tuning(path, k2, {(2, 20): "oneshot"})  # merged, not overwritten
    assert load_tuning(path, k8) == {(8, 20): "fanout", (8, 12): "ll"}
    assert load_tuning(path, k2) == {(2, 20): "oneshot"}
    assert load_tuning(path, tuning_key(4, 1, "x")) == {}
    g = SimpleNamespace(size=8, tuned=load_tuning(path, k8), ll_auto_max=64 << 10, oneshot_max=64 << 10, disabled=set())
    assert pick(g, 1 << 20) == "fanout" and pick(g, 4096) == "ll"


def test_alltoallv_plan_offsets():
    """Ragged all-to-all offsets (DeviceGroup.alltoallv): every rank's segment for rank j
    lands right after the segments of ranks < it in j's output, and the per-rank plans
    tile every output exactly once."""
    import numpy as np

    from collective_communication_mpi_amd.device import alltoallv_plan

    rng = np.random.default_rng(0)
    for p in (1, 2, 3, 8):
        C = rng.integers(0, 9, (p, p)) * 4
        es = 4
        plans = [alltoallv_plan(C, me, es) for me in range(p)]
        for me, (soff, doff, lens, grid) in enumerate(plans):
            assert lens == [int(c) * es for c in C[me]]
            assert soff == [int(C[me, :j].sum()) * es for j in range(p)]
            assert grid == int(C.sum(axis=1).max()) * es
        for j in range(p):  # rank j's output: [sum_i C[i, j]] covered once, in source order
            segs = sorted((plans[i][1][j], plans[i][2][j]) for i in range(p))
            pos = 0
            for off, ln in segs:
                assert off == pos
                pos += ln
            assert pos == int(C[:, j].sum()) * es


def test_tp_gemm_routing(monkeypatch):
    """TP layers: hand-written MFMA GEMMs for every CUDA bf16 shape by default (the LDS-ring
    kernel for large ones); CCMPI_TP_GEMM=blas routes to hipBLASLt; other dtypes never MFMA."""
    import torch

    from collective_communication_mpi_amd.parallel import tensor_parallel as tpm

    x = SimpleNamespace(is_cuda=True, dtype=torch.bfloat16, shape=(4096, 4096), numel=lambda: 4096 * 4096)
    w_big = SimpleNamespace(dtype=torch.bfloat16, shape=(28672, 4096))
    w_small = SimpleNamespace(dtype=torch.bfloat16, shape=(256, 4096))
    for mode in ("auto", "own"):
        monkeypatch.setattr(tpm, "_TP_GEMM", mode)
        assert tpm._mfma_ok(x, w_small) and tpm._mfma_ok(x, w_big)
    monkeypatch.setattr(tpm, "_TP_GEMM", "blas")
    assert not tpm._mfma_ok(x, w_small) and not tpm._mfma_ok(x, w_big)
    monkeypatch.setattr(tpm, "_TP_GEMM", "auto")
    x32 = SimpleNamespace(is_cuda=True, dtype=torch.float32, shape=(4096, 4096), numel=lambda: 4096 * 4096)
    assert not tpm._mfma_ok(x32, w_small)
