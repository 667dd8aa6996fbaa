"""CPU checks of the backward GEMM routing rule (ops.kernels._kmajor_via_transpose): which
K-major GEMMs of the Llama MLP backward go through transposed copies into the N-layout
pair ring, which stay on the K-major ring, and the CCMPI_KMAJOR_ROUTE switch."""
import torch

from collective_communication_mpi_amd.ops.kernels import _kmajor_via_transpose


def _t(*shape):
    return torch.empty(*shape, dtype=torch.bfloat16)


def test_dw_default_route_reads_kmajor_operands(monkeypatch):
    """Default route ``pair``: the pair ring reads both M-major dW operands itself (no
    transposes, no dh^T); the round-4 transpose route stays selectable."""
    monkeypatch.delenv("CCMPI_KMAJOR_ROUTE", raising=False)
    T, d, f = 4096, 4096, 14336
    assert not _kmajor_via_transpose(2 * f, d, T, _t(T, 2 * f), _t(T, d))
    assert not _kmajor_via_transpose(d, f, T, _t(T, d), _t(T, f))


def test_dw_shapes_take_the_transpose_route(monkeypatch):
    monkeypatch.setenv("CCMPI_KMAJOR_ROUTE", "transpose")
    T, d, f = 4096, 4096, 14336
    # gate|up dW = dh^T X: M = 2f, N = d, K = T
    assert _kmajor_via_transpose(2 * f, d, T, _t(T, 2 * f), _t(T, d))
    # down dW = dY^T A: M = d, N = f, K = T
    assert _kmajor_via_transpose(d, f, T, _t(T, d), _t(T, f))


def test_long_k_small_and_ragged_stay_on_the_ring(monkeypatch):
    monkeypatch.setenv("CCMPI_KMAJOR_ROUTE", "transpose")
    assert not _kmajor_via_transpose(4096, 4096, 28672, _t(28672, 4096), _t(28672, 4096))  # long K
    assert not _kmajor_via_transpose(512, 4096, 4096, _t(4096, 512), _t(4096, 4096))  # M < 1024
    assert not _kmajor_via_transpose(1024, 1024, 1024, _t(1024, 1024), _t(1024, 1024))  # < 2^33 MACs
    assert not _kmajor_via_transpose(4100, 4096, 4096, _t(4096, 4100), _t(4096, 4096))  # M % 8


def test_route_switch(monkeypatch):
    monkeypatch.setenv("CCMPI_KMAJOR_ROUTE", "ring")
    assert not _kmajor_via_transpose(28672, 4096, 4096, _t(4096, 28672), _t(4096, 4096))
    monkeypatch.setenv("CCMPI_KMAJOR_ROUTE", "transpose")
    assert _kmajor_via_transpose(28672, 4096, 4096, _t(4096, 28672), _t(4096, 4096))


def test_row_parallel_auto_mode(monkeypatch):
    """``auto``: the mode the mlp phase measured for this (M, N) on a group
    of the same identity (the group's ``row_modes`` table, loaded from CCMPI_TUNE_FILE);
    "plain" when nothing was measured -- "chunked" is never the unmeasured default; explicit
    modes pass through."""
    from types import SimpleNamespace

    from collective_communication_mpi_amd.parallel import tensor_parallel as tp

    monkeypatch.setattr(tp, "_size_rank", lambda comm: (2, 0))
    monkeypatch.setattr(tp, "device_group_for", lambda comm: SimpleNamespace(shared_device=False, row_modes={}))
    assert tp._row_mode("auto", object(), 16384, 8192) == "plain"
    assert tp._row_mode("auto", object(), 4096, 4096) == "plain"
    table = {(4096, 4096): "push", (8192, 4096): "chunked", (256, 64): "bogus"}
    monkeypatch.setattr(tp, "device_group_for", lambda comm: SimpleNamespace(shared_device=False, row_modes=table))
    assert tp._row_mode("auto", object(), 4096, 4096) == "push"
    assert tp._row_mode("auto", object(), 8192, 4096) == "chunked"
    assert tp._row_mode("auto", object(), 256, 64) == "plain"  # unknown mode names are ignored
    assert tp._row_mode("auto", object(), 2048, 4096) == "plain"
    assert tp._row_mode("fused", object(), 4096, 4096) == "fused"


def test_row_mode_tune_file_switches_auto_to_push(tmp_path):
    """A tune-file entry written by the mlp phase (save_row_modes) is what a device group
    created afterwards loads (load_row_modes) and what ``auto`` then runs; it sits beside the
    collective tables in the same file without disturbing them."""
    from collective_communication_mpi_amd.device import load_row_modes, load_tuning, save_row_modes, save_tuning
    from collective_communication_mpi_amd.parallel import tensor_parallel as tp

    path = str(tmp_path / "tune.json")
    save_tuning(path, "p8-share1-MI355X", {(8, 20): "fanout"})
    save_row_modes(path, "p8-share1-MI355X", {(4096, 4096): "push"})
    assert load_tuning(path, "p8-share1-MI355X") == {(8, 20): "fanout"}
    table = load_row_modes(path, "p8-share1-MI355X")
    assert table == {(4096, 4096): "push"} and load_row_modes(path, "p2-share1-MI355X") == {}
    assert tp.row_mode_from_table(table, 4096, 4096) == "push"
    assert tp.row_mode_from_table({}, 4096, 4096) == "plain"


def test_row_parallel_push_applies(monkeypatch):
    """``push`` (GEMM epilogue into the owners' inboxes) needs whole 256-row tiles per rank
    block, no bias, K % 64, N % 8 and the ring GEMM; otherwise the layer runs plain."""
    from types import SimpleNamespace

    from collective_communication_mpi_amd.parallel import tensor_parallel as tp

    def t(*shape):
        return SimpleNamespace(is_cuda=True, dtype=torch.bfloat16, shape=shape, stride=lambda d: shape[1])

    monkeypatch.setattr(tp, "_size_rank", lambda comm: (4, 0))
    monkeypatch.setattr(tp, "_gpu_shared", lambda comm: False)
    assert "push" in tp.ROW_MODES
    assert tp._push_ok(t(4096, 3584), t(4096, 3584), None, object())
    assert not tp._push_ok(t(4096, 3584), t(4096, 3584), object(), object())  # bias
    assert not tp._push_ok(t(2048 + 256, 3584), t(4096, 3584), None, object())  # M % (256 p)
    assert not tp._push_ok(t(4096, 3600), t(4096, 3600), None, object())  # K % 64
    assert not tp._push_ok(t(4096, 3584), t(4100, 3584), None, object())  # N % 8
    monkeypatch.setattr(tp, "_gpu_shared", lambda comm: True)
    assert not tp._push_ok(t(4096, 3584), t(4096, 3584), None, object())  # ring GEMM off
