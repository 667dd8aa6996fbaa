"""bench.py's supervisor contract (CPU: the merge logic only).

* the headline comes from the collective phase alone: a crashed harness (rc -11, the
  round-3 HIP-graph segfault) or a failed DP / MLP phase leaves ``value`` intact and
  records the failure under its own key;
* RCCL is the library comparison: even when it is faster it never replaces ``value``
  (``config.rccl`` + ``handwritten_vs_rccl``);
* the phase plan: the harness always runs in a phase of its own."""
import os
import sys

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
    assert names == ["coll", "harness", "mlp", "dp", "rccl", "host"]
    assert [p for p, _ in bench.plan_phases(args, 1)] == ["coll", "harness", "mlp", "host"]
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


def _fake_pick(fail, times):
    """pick_candidates with injected failures (``fail``: candidates whose attempt fails on
    'rank 1'), a fake agree over 2 ranks and counted resets."""
    resets = []

    def attempt(c):
        if c in fail:
            raise RuntimeError("device collective timeout/fault code 0x301 on rank 1 (phase 3, peer 0)")
        return None

    def agree(err):
        return f"rank 1: {err}" if err else None

    return attempt, agree, lambda: resets.append(1), lambda c: times[c], resets


def test_failed_first_candidate_keeps_trying():
    """a failing first candidate is reset away and the rest are still
    tried; every outcome is recorded with its error text."""
    cands = ["twoshot:256", "twoshot:512", "fanout:256", "fanout:512", "ring"]
    times = {"twoshot:512": 4e-3, "fanout:256": 3e-3, "fanout:512": 2.5e-3, "ring": 9e-3}
    attempt, agree, reset, timer, resets = _fake_pick({"twoshot:256"}, times)
    out, best = bench.pick_candidates(cands, attempt, agree, reset, timer)
    assert best == "fanout:512" and len(resets) == 1
    assert out["twoshot:256"]["ms"] is None and "0x301" in out["twoshot:256"]["error"]
    assert out["ring"]["ms"] == 9.0 and out["ring"]["error"] is None


def test_every_candidate_failing_returns_none():
    cands = ["fanout:256", "ring"]
    attempt, agree, reset, timer, resets = _fake_pick(set(cands), {})
    out, best = bench.pick_candidates(cands, attempt, agree, reset, timer)
    assert best is None and len(resets) == 2 and all(o["error"] for o in out.values())


def test_timing_failure_is_a_candidate_error():
    def timer(c):
        if c == "a":
            raise RuntimeError("boom")
        return 1e-3

    out, best = bench.pick_candidates(["a", "b"], lambda c: None, lambda e: e, lambda: None, timer)
    assert best == "b" and "during timing" in out["a"]["error"]


def test_candidate_order_follows_self_test():
    cands = bench.allreduce_candidates(8, False)
    order, skipped = bench.order_candidates(cands, {"ll": True, "oneshot": True, "fanout": True, "twoshot": False},
                                            {"twoshot"})
    assert "twoshot:256" in skipped and "twoshot:512" in skipped
    assert order[:3] == ["fanout:256", "fanout:512", "fanout_lds:512"]
    assert order[3:] == ["push:512", "ring", "rhd"]
    # no self test (one rank) keeps the given order
    order, skipped = bench.order_candidates(["b", "a"], None, set())
    assert order == ["b", "a"] and not skipped


def test_injected_candidate_fault_spec(monkeypatch):
    monkeypatch.setenv("CCMPI_RANK", "0")
    monkeypatch.setenv("CCMPI_SIZE", "2")
    monkeypatch.setenv("CCMPI_BENCH_FAULT", "candidate:twoshot:256,candidate_bf16:*")
    assert bench._injected("twoshot:256", "fp32") and bench._injected("twoshot:256", "bf16")
    assert not bench._injected("fanout:512", "fp32") and bench._injected("fanout:512", "bf16")
    monkeypatch.setenv("CCMPI_RANK", "1")
    assert not bench._injected("twoshot:256", "fp32")  # only rank 0 skips its kernel


def test_bf16_exhaustion_keeps_fp32_headline():
    """An exhausted bf16 candidate list records an error in its block; the record (and the
    fp32 value) survive."""
    args = bench.parse([])
    coll = _coll()
    coll["config"]["bf16_1GiB"] = {"error": "no bf16 candidate produced a correct result",
                                   "candidates": {"fanout:512": {"ms": None, "error": "rank 0: injected"}}}
    out = bench.merge_results(args, 8, {"coll": {"ok": True, "returncodes": [0] * 8, "seconds": 1}},
                              {"coll": coll}.get)
    assert out["value"] == 500.0 and "error" in out["config"]["bf16_1GiB"] and "warning" not in out


def test_partial_headline_sets_top_level_warning():
    args = bench.parse([])
    early = {**_coll(), "partial": "written after the fp32 headline, before the secondaries"}
    out = bench.merge_results(args, 8, _status(coll=-11), {"coll": early}.get)
    assert out["value"] == 500.0 and "warning" in out


def test_host_phase_record_merged():
    args = bench.parse([])
    assert [p for p, _ in bench.plan_phases(args, 1)][-1] == "host"
    assert "host" not in [p for p, _ in bench.plan_phases(bench.parse(["--host-ranks", "0"]), 1)]
    st = {"coll": {"ok": True, "returncodes": [0], "seconds": 1}, "host": {"ok": True, "returncodes": [0], "seconds": 3}}
    rec = {"ranks": 8, "allreduce": {"Allreduce_avg_us": 12.0, "myAllreduce_avg_us": 20.0, "all_runs_equal": True}}
    out = bench.merge_results(args, 1, st, {"coll": _coll(), "host": rec}.get)
    assert out["config"]["host_cpu"]["allreduce"]["all_runs_equal"]


def test_host_phase_runs_on_cpu(tmp_path):
    """BASELINE config 1 end to end on the CPU: 8 host-plane processes, library vs
    hand-written all-reduce / all-to-all, every run checked equal."""
    import json
    import os
    import subprocess
    import sys

    res = tmp_path / "host.json"
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-m", "collective_communication_mpi_amd.launch", "-n", "8", "--timeout", "150",
                        sys.executable, "bench.py", "--phase", "host", "--host-runs", "20", "--result", str(res)],
                       cwd=repo, capture_output=True, text=True, timeout=200)
    assert r.returncode == 0, r.stderr[-3000:]
    rec = json.loads(res.read_text())
    assert rec["ranks"] == 8 and rec["allreduce"]["all_runs_equal"] and rec["alltoall"]["all_runs_equal"]
    assert rec["allreduce"]["myAllreduce_avg_us"] > 0 and rec["alltoall"]["myAlltoall_avg_us"] > 0


def test_sweep_curve_from_tune_times():
    """DeviceGroup.tune keeps every algorithm's time per (dtype, size); sweep_curve turns them
    into the algbw / busbw-vs-size curve the bench records (NCCL-tests conventions)."""
    from collective_communication_mpi_amd.device import DeviceGroup

    class G:
        size = 4
        tune_times = {("float32", 4 << 20): {"twoshot": 3e-4},
                      ("float32", 1 << 20): {"twoshot": 1e-4, "ll": None, "fanout": 2e-4},
                      ("bfloat16", 1 << 20): {"ring": 5e-4}}

    curve = DeviceGroup.sweep_curve(G(), "float32")
    assert [c["bytes"] for c in curve] == [1 << 20, 4 << 20]
    assert curve[0]["best"] == "twoshot" and curve[0]["ms"] == {"twoshot": 0.1, "ll": None, "fanout": 0.2}
    alg = (1 << 20) / 1e-4 / 1e9
    assert curve[0]["algbw_GBps"] == round(alg, 2) and curve[0]["busbw_GBps"] == round(alg * 1.5, 2)
    assert [c["best"] for c in DeviceGroup.sweep_curve(G(), "bfloat16")] == ["ring"]


def test_phase_binding_paths(monkeypatch):
    """both launch paths place GPU ranks the same way.  torchrun (nobody
    bound the supervisor): rank 0 reads the GPU-local plan once and every rank takes its
    local rank's set; launch.py (``CCMPI_BOUND_CPUS`` set): the children inherit that
    binding; ``CCMPI_BIND=none``: the OS places them."""
    from collective_communication_mpi_amd import topology

    plan = [[0, 1], [2, 3], [64, 65], [66, 67]]
    monkeypatch.setattr(topology, "gpu_plan", lambda n, **k: plan[:n])

    class World:
        def Get_size(self):
            return 4

        def bcast(self, obj, root=0):
            return obj if obj is not None else plan

    monkeypatch.delenv("CCMPI_BOUND_CPUS", raising=False)
    monkeypatch.delenv("CCMPI_BIND", raising=False)
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "4")
    assert bench.phase_binding(World(), 0, 0) == ([0, 1], "gpu")
    assert bench.phase_binding(World(), 2, 2) == ([64, 65], "gpu")
    monkeypatch.setenv("CCMPI_BIND", "none")
    assert bench.phase_binding(World(), 1, 1) == (None, "none")
    monkeypatch.setenv("CCMPI_BIND", "gpu")
    monkeypatch.setenv("CCMPI_BOUND_CPUS", "8-15")
    monkeypatch.setenv("CCMPI_BIND_EFFECTIVE", "gpu")
    assert bench.phase_binding(World(), 1, 1) == (None, "gpu")


def test_phase_binding_plan_failure_reaches_every_rank(monkeypatch):
    """A placement plan that fails on rank 0 (any exception, not only OSError) must still reach
    the broadcast every other rank waits in -- with None, so every rank falls back to the OS's
    placement -- and a child binding outside the cpuset must not stop the phase child."""
    from collective_communication_mpi_amd import topology

    def boom(n, **k):
        raise KeyError("no such sysfs attribute")

    monkeypatch.setattr(topology, "gpu_plan", boom)
    calls = []

    class World:
        def Get_size(self):
            return 2

        def bcast(self, obj, root=0):
            calls.append(obj)
            return obj

    monkeypatch.delenv("CCMPI_BOUND_CPUS", raising=False)
    monkeypatch.setenv("CCMPI_BIND", "gpu")
    assert bench.phase_binding(World(), 0, 0) == (None, "none")
    assert calls == [None]
    # a CPU set the process may not use: the child starts anyway, placed by the OS
    rc, _ = bench._run_child([sys.executable, "-c", "pass"], dict(os.environ), 60, cpus=[1 << 20])
    assert rc == 0
