"""bench.py's supervisor contract (CPU: the merge logic only).

* the headline comes from the collective phase alone: a crashed harness (rc -11, the
  round-3 HIP-graph segfault) or a failed DP / MLP phase leaves ``value`` intact and
  records the failure under its own key;
* RCCL is the library comparison: even when it is faster it never replaces ``value``
  (``config.rccl`` + ``handwritten_vs_rccl``);
* the phase plan: the harness always runs in a phase of its own."""
import bench


def _coll():
    return {"metric": bench.METRIC, "value": 500.0, "ms_per_step": 2.147, "n_gpus": 8,
            "config": {"allreduce_algo": "fanout:512", "parallelism": "dp4xtp2",
                       "bf16_1GiB": {"algbw_GBps": 480.0}, "alltoall": {"ms": 1.0, "candidates_ms": {}}}}


def _status(**bad):
    st = {ph: {"ok": True, "returncodes": [0] * 8, "seconds": 1.0} for ph in ("coll", "harness", "mlp", "dp", "rccl")}
    for ph, rc in bad.items():
        st[ph] = {"ok": False, "returncodes": [rc] * 8, "seconds": 1.0}
    return st


def test_harness_crash_keeps_headline():
    args = bench.parse([])
    recs = {"coll": _coll(), "harness": None, "mlp": {"tp": 8, "fwd_ms": 0.2}, "dp": {"comm_hidden_fraction": 0.9},
            "rccl": {"algbw_GBps": 400.0, "bf16_algbw_GBps": 400.0, "alltoall_ms": {"rccl": 1.2}}}
    out = bench.merge_results(args, 8, _status(harness=-11), recs.get)
    c = out["config"]
    assert out["value"] == 500.0 and out["ms_per_step"] == 2.147
    assert "error" in c["harness"] and "-11" in c["harness"]["error"]
    assert "tp_fwd_step_ms" not in c
    assert c["tp_mlp"]["tp"] == 8 and c["dp_overlap"]["comm_hidden_fraction"] == 0.9
    assert c["phases"]["harness"]["returncodes"] == [-11] * 8


def test_harness_record_fills_step_time():
    args = bench.parse([])
    recs = {"coll": _coll(), "harness": {"tp": 2, "dp": 4, "fwd_ms": 0.61, "train_ms": 1.2, "global_batch": 8192,
                                         "seq_len": 16}}
    st = {k: v for k, v in _status().items() if k in ("coll", "harness")}
    out = bench.merge_results(args, 8, st, recs.get)
    c = out["config"]
    assert c["tp_fwd_step_ms"] == 0.61 and c["tp_train_step_ms"] == 1.2 and c["parallelism"] == "dp4xtp2"
    assert "fwd_ms" not in c["harness"]


def test_failed_collective_phase_zero_value():
    args = bench.parse([])
    out = bench.merge_results(args, 8, {"coll": {"ok": False, "returncodes": [-11] * 8, "seconds": 1}}, {}.get)
    assert out["value"] == 0.0 and "collective phase failed" in out["config"]["error"]


def test_faster_rccl_never_replaces_handwritten_value():
    args = bench.parse([])
    recs = {"coll": _coll(), "rccl": {"algbw_GBps": 1000.0, "allreduce_ms": 1.07, "bf16_algbw_GBps": 800.0,
                                      "alltoall_ms": {"rccl": 0.5}}}
    st = {k: v for k, v in _status().items() if k in ("coll", "rccl")}
    out = bench.merge_results(args, 8, st, recs.get)
    c = out["config"]
    assert out["value"] == 500.0 and c["allreduce_algo"] == "fanout:512" and out["ms_per_step"] == 2.147
    assert c["rccl"]["algbw_GBps"] == 1000.0 and c["handwritten_vs_rccl"] == 0.5
    assert c["bf16_1GiB"]["handwritten_vs_rccl"] == 0.6 and c["alltoall"]["rccl_ms"] == {"rccl": 0.5}


def test_phase_plan_isolates_harness():
    args = bench.parse([])
    names = [p for p, _ in bench.plan_phases(args, 8)]
    assert names == ["coll", "harness", "mlp", "dp", "rccl"]
    assert [p for p, _ in bench.plan_phases(args, 1)] == ["coll", "harness", "mlp"]
    assert "fanout:1024" not in bench.allreduce_candidates(8, False)


def test_multi_stream_graph_hazard(monkeypatch):
    """The HIP-graph guard of the harness: multi-stream forwards are not captured with fewer
    than 4 hardware queues per process (the runtime's parallel-stream crash)."""
    from types import SimpleNamespace

    from collective_communication_mpi_amd.models.harness import multi_stream_graph_hazard

    layer = SimpleNamespace(tp_dev=object(), _token_chunks=lambda B: 4)
    cfg = SimpleNamespace(fc_o_mode="token", batch=2048, fwd_chunks=1)
    monkeypatch.setenv("GPU_MAX_HW_QUEUES", "1")
    assert multi_stream_graph_hazard(cfg, layer)
    monkeypatch.setenv("CCMPI_FORCE_GRAPH", "1")
    assert multi_stream_graph_hazard(cfg, layer) is None
    monkeypatch.delenv("CCMPI_FORCE_GRAPH")
    monkeypatch.setenv("GPU_MAX_HW_QUEUES", "4")
    assert multi_stream_graph_hazard(cfg, layer) is None
    monkeypatch.setenv("GPU_MAX_HW_QUEUES", "1")
    single = SimpleNamespace(tp_dev=object(), _token_chunks=lambda B: 1)
    assert multi_stream_graph_hazard(cfg, single) is None


def test_tuning_sweep_failure_keeps_headline():
    """The coll phase writes its record (``partial``) once the headline is measured, before
    the secondary tuning sweep: a sweep that crashes or hangs costs the table, not ``value``."""
    args = bench.parse([])
    early = {**_coll(), "partial": "written before the tuning sweep"}
    out = bench.merge_results(args, 8, _status(coll=-11), {"coll": early}.get)
    assert out["value"] == 500.0 and out["config"]["allreduce_algo"] == "fanout:512"
    assert "-11" in out["config"]["coll_phase_error"]
    # no record at all: the zero headline, as before
    out = bench.merge_results(args, 8, _status(coll=-11), {}.get)
    assert out["value"] == 0.0
