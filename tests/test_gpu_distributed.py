"""Multi-rank GPU tests (ranks share the box's one GPU through IPC).

* every device collective vs an fp64/int64 oracle at 2, 3, 4 and 8 ranks (tests/workers/device_worker.py);
* the DP x TP harness: tp=2 (row-parallel and the reference's naive collects),
  dp=2 and dp=2 x tp=2 reproduce the single-rank training run (losses and
  final weights) within bf16 tolerance."""
import os

import numpy as np
import pytest

from _launch import py, run_ranks

pytestmark = pytest.mark.gpu

ENV = {"CCMPI_DEVICE_TIMEOUT_S": "20"}


@pytest.mark.parametrize("n,matrix", [(2, "full"), (4, "full"), (8, "wide"), (3, "quick")])
def test_device_collectives_multi_rank(n, matrix):
    """Every hand-written collective x algorithm x dtype x op (tests/workers/device_worker.py)
    against an fp64/int64 oracle; 3 ranks: non-power-of-two ring and the rhd refusal."""
    r = run_ranks(n, py("tests/workers/device_worker.py", "--matrix", matrix), timeout=600, env=ENV)
    assert "0 failures" in r.stdout


@pytest.mark.parametrize("n,reg", [(2, "0"), (4, "0"), (2, str(1 << 20))])
def test_device_collectives_big(n, reg):
    """>= 96 MiB: staging-chunk loops and ring/rhd inbox pieces (inbox capped at 64 MiB);
    with on-demand registration off (reg 0) the ordinary tensors take the staging loops,
    with it on they are mapped and reduced in place."""
    r = run_ranks(n, py("tests/workers/device_worker.py", "--big"), timeout=400,
                  env=dict(ENV, CCMPI_INBOX_MAX_MB="64", CCMPI_REGISTER_MIN_BYTES=reg))
    assert "0 failures" in r.stdout


@pytest.mark.parametrize("n", [2, 3, 4])
def test_fused_rowparallel_gemm_allreduce(n):
    """the TP all-reduce fused into the row-parallel GEMM (tile tickets,
    last arrival reduces in rank order and writes every rank's output): vs fp32, bitwise
    vs the unfused rank-order sum, identical on every rank, under rank skew, and through
    RowParallelLinear forward + backward (tests/workers/fused_worker.py)."""
    r = run_ranks(n, py("tests/workers/fused_worker.py"), timeout=400, env=ENV)
    assert "fused OK" in r.stdout


@pytest.mark.parametrize("n", [2, 3, 4, 8])
def test_device_ondemand_registration(n):
    """ordinary torch tensors >= 1 MiB are registered on demand (IPC
    handle of their allocator segment, one host all-gather per call, LRU of mapped
    slots) and every collective runs on them in place; slots are reused, and a freed
    and reallocated range is remapped (allocator generation)."""
    r = run_ranks(n, py("tests/workers/device_worker.py", "--register"), timeout=400, env=ENV)
    assert "0 failures" in r.stdout


def test_harness_graph_replay_after_collectives_one_queue():
    """the bench's old one-process sequence -- collective candidates, bf16,
    all-to-all, empty_cache, then the harness forwards (token, pooled, 4-block token pipeline)
    as HIP graphs -- with 8 ranks on the GPU and ONE hardware queue each.  The multi-stream
    pipeline's graph is what crashed the HIP runtime (profiles/r4_bisect); it is timed eagerly
    under few queues, every other forward replays its graph."""
    r = run_ranks(8, py("benchmarks/graph_replay_repro.py", "--prefix", "ar,bf16,a2a,free", "--size-mb", "256",
                        "--variants", "token:1,row:1,token:4"), timeout=400,
                  env=dict(ENV, GPU_MAX_HW_QUEUES="1", CCMPI_SHARED_GRAPH="1"))  # capture despite sharing
    assert "replay OK" in r.stdout
    import json

    rec = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    graphs = {x["variant"]: x["hip_graph"] for x in rec["results"]}
    assert graphs == {"token:1": True, "row:1": True, "token:4": False}, graphs


def test_captured_registration_slot_is_pinned():
    """a slot a captured HIP graph uses is pinned -- more registrations than
    CCMPI_REGISTER_SLOTS afterwards do not evict it, and the replay is still exact."""
    r = run_ranks(2, py("tests/workers/capture_pin_worker.py"), timeout=200, env=ENV)
    assert "capture pin OK" in r.stdout


@pytest.mark.parametrize("n", [2, 4, 8])
def test_device_collectives_random_skew(n):
    """Randomised per-rank host/device delays, back-to-back calls, symmetric and staged
    calls up to 16 MiB."""
    r = run_ranks(n, py("tests/workers/device_worker.py", "--stress", "120"), timeout=400, env=ENV)
    assert "0 failures" in r.stdout


def test_device_collectives_serialized_launches():
    """the quick matrix with every kernel launch serialized
    (AMD_SERIALIZE_KERNEL=3 / AMD_SERIALIZE_COPY=3, HIP's CUDA_LAUNCH_BLOCKING): the flag
    protocol may not depend on launch overlap within a rank."""
    r = run_ranks(2, py("tests/workers/device_worker.py", "--matrix", "quick", "--sizes", "1,1000,65539"),
                  timeout=300, env=dict(ENV, AMD_SERIALIZE_KERNEL="3", AMD_SERIALIZE_COPY="3"))
    assert "0 failures" in r.stdout


def test_trace_records_collectives_and_survives_graph_capture(tmp_path):
    """CCMPI_TRACE=1 over the quick matrix (which also captures collectives in HIP
    graphs): one JSON record per eager call per rank, with device time and bandwidths;
    calls made during a capture keep their roctx range but are not timed."""
    import glob
    import json

    path = str(tmp_path / "trace_{pid}.jsonl")
    r = run_ranks(2, py("tests/workers/device_worker.py", "--matrix", "quick", "--sizes", "1000"), timeout=300,
                  env=dict(ENV, CCMPI_TRACE="1", CCMPI_TRACE_FILE=path))
    assert "0 failures" in r.stdout
    files = glob.glob(str(tmp_path / "trace_*.jsonl"))
    assert len(files) == 2
    recs = [json.loads(ln) for f in files for ln in open(f)]
    assert {"allreduce", "allgather", "alltoall"} <= {x["op"] for x in recs}
    assert all(x["ms"] >= 0 and x["bytes"] >= 0 for x in recs)
    assert {"ll", "fanout", "push"} <= {x["algo"] for x in recs}


def test_rccl_same_gpu_refused_and_recorded(tmp_path):
    """RCCL with two ranks on one GPU: ncclCommInitRank refuses the duplicate device
    ('invalid usage', profiles/r2_coll/rccl_shared_gpu.json) on every rank, and the probe
    records that outcome instead of hanging or swallowing it."""
    import json

    out = tmp_path / "probe.json"
    run_ranks(2, py("benchmarks/rccl_shared_probe.py", "--out", str(out)), timeout=200, env=ENV)
    rec = json.loads(out.read_text())
    assert len(rec["per_rank"]) == 2
    for r in rec["per_rank"]:
        init = r["ncclCommInitRank"]
        assert not init["ok"], init
        assert "RCCL error" in init["error"] and "invalid usage" in init["error"], init


def _bench_line(extra_env, *args):
    import json
    import subprocess
    import sys

    from _launch import REPO

    e = dict(os.environ, **ENV, **extra_env)
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--steps", "2", "--warmup", "1", "--size-mb", "16",
                        "--a2a-mb", "8", "--dp-layers", "0", "--batch", "128", "--no-secondary", *args],
                       cwd=REPO, env=e, capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, r.stderr[-4000:]
    return json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])


@pytest.mark.parametrize("mode", ["error", "hang"])
def test_bench_survives_rccl_failure(mode):
    """the RCCL baseline runs in its own child group after every
    hand-written number is measured; an RCCL error (forced on ranks that share the GPU)
    or a hang (killed at --rccl-timeout) costs only the 'rccl' entry, never the line."""
    env = {"CCMPI_BENCH_RCCL": "force"} if mode == "error" else {"CCMPI_BENCH_RCCL": "hang"}
    # (the injected hang is killed at the phase limit: 20 s is enough to show it costs only 'rccl')
    out = _bench_line(env, "--rccl-timeout", "60" if mode == "error" else "20")
    c = out["config"]
    assert out["value"] > 0 and c["result_exact"] and c["tp_fwd_step_ms"] > 0
    assert "error" in c["rccl"], c["rccl"]
    assert all(v for v in c["candidates_ms"].values()), c["candidates_ms"]


def test_bench_harness_crash_keeps_headline():
    """the harness runs in a supervised phase of its own; a SIGSEGV there
    (injected: CCMPI_BENCH_FAULT=harness) costs only the harness record, never the
    hand-written all-reduce headline."""
    out = _bench_line({"CCMPI_BENCH_FAULT": "harness"}, "--no-rccl")
    c = out["config"]
    assert out["value"] > 0 and c["result_exact"], out
    assert not c["phases"]["harness"]["ok"] and "error" in c["harness"], c["harness"]
    assert "tp_fwd_step_ms" not in c


def test_bench_tuning_crash_keeps_headline():
    """The coll phase writes the headline before its secondary tuning sweep: a SIGSEGV right
    after it (injected: CCMPI_BENCH_FAULT=coll_tuning) keeps ``value`` and the exit status."""
    import json
    import subprocess
    import sys

    from _launch import REPO

    e = dict(os.environ, **ENV, CCMPI_BENCH_FAULT="coll_tuning")
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--steps", "2", "--warmup", "1", "--size-mb", "16",
                        "--a2a-mb", "8", "--dp-layers", "0", "--batch", "128", "--tune-max-mb", "1", "--no-rccl",
                        "--no-harness", "--mlp-tokens", "0"], cwd=REPO, env=e, capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, r.stderr[-4000:]
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    c = out["config"]
    assert out["value"] > 0 and c["result_exact"] and out.get("partial"), out
    assert "-11" in c["coll_phase_error"], c.get("coll_phase_error")


def test_bench_failing_candidates_keep_headline():
    """the first fp32 candidate fails (rank 0 skips its kernel, rank 1 times
    out in it), and so does every bf16 candidate; the bench resets, tries the rest, records
    each failure with its timeout code, and ``value`` comes from the next working algorithm."""
    import json
    import subprocess
    import sys

    from _launch import REPO

    # each injected failure waits out the device timeout on the rank left in the kernel: 6 s
    # here (the collectives themselves take milliseconds at 16 MiB) instead of the suite's 20
    e = dict(os.environ, **ENV, CCMPI_BENCH_FAULT="candidate:twoshot:256,candidate_bf16:*")
    e["CCMPI_DEVICE_TIMEOUT_S"] = "6"
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--steps", "2", "--warmup", "1", "--size-mb", "16",
                        "--a2a-mb", "8", "--dp-layers", "0", "--tune-max-mb", "1", "--no-rccl", "--no-harness",
                        "--mlp-tokens", "0", "--host-ranks", "0"],
                       cwd=REPO, env=e, capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, r.stderr[-4000:]
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    c = out["config"]
    assert out["value"] > 0 and c["result_exact"], out
    cand = c["candidates"]
    assert cand["twoshot:256"]["ms"] is None and "rank" in cand["twoshot:256"]["error"], cand
    assert c["allreduce_algo"] != "twoshot:256" and sum(1 for o in cand.values() if o["ms"]) >= 3, cand
    assert "error" in c["bf16_1GiB"] and all(o["error"] for o in c["bf16_1GiB"]["candidates"].values()), c["bf16_1GiB"]
    assert c["alltoall_pairwise"]["ms"] > 0 and c["alltoall"]["ms"] > 0
    sw = c["sweep"]
    assert sw["float32"] and all(pt["algbw_GBps"] for pt in sw["float32"]), sw
    assert sw["bfloat16"] and sw["float32"][-1]["bytes"] == 16 << 20


@pytest.mark.parametrize("case", ["myallreduce", "myalltoall"])
def test_cli_device_cases(case):
    """The reference CLI cases on device buffers (reference mpi-test.py:42-98,178-239):
    myAllreduce (int64, MIN) and myAlltoall vs the library path, 4 ranks."""
    r = run_ranks(4, py("mpi-test.py", "--device", "cuda", "--test_case", case, "--runs", "5", "--warmup", "1"),
                  timeout=300, env=ENV)
    assert "All runs produced correct results." in r.stdout


def test_device_timeout_watchdog_and_recovery():
    """A rank that skips a collective: bounded spins, host watchdog, reset."""
    run_ranks(2, py("tests/workers/device_worker.py", "--fault"), timeout=120, env=dict(ENV, CCMPI_WATCHDOG="warn"))


@pytest.fixture(scope="module")
def reference_run(tmp_path_factory):
    out = tmp_path_factory.mktemp("h") / "ref.npz"
    run_ranks(1, py("tests/workers/harness_worker.py", "--tp", "1", "--out", str(out)), timeout=300, env=ENV)
    return np.load(out)


@pytest.mark.parametrize("n,tp,mode", [(2, 2, "row"), (2, 2, "naive"), (2, 2, "token"), (2, 1, "row"), (4, 2, "row"),
                                       (4, 2, "token"), (8, 2, "row"), (8, 1, "row")])  # 8 ranks on one GPU: DP4 x TP2
def test_harness_matches_single_rank(reference_run, tmp_path, n, tp, mode):
    out = tmp_path / "run.npz"
    run_ranks(n, py("tests/workers/harness_worker.py", "--tp", str(tp), "--mode", mode, "--out", str(out)),
              timeout=400, env=ENV)
    got = np.load(out)
    np.testing.assert_allclose(got["losses"], reference_run["losses"], rtol=2e-2, atol=2e-3)
    for k in ("q_w", "o_w", "emb_w"):
        np.testing.assert_allclose(got[k], reference_run[k], rtol=5e-2, atol=5e-3)
    assert got["losses"][-1] < got["losses"][0]


def test_harness_train_plan_matches_eager():
    """Training steps re-issued from recorded launch plans (TrainPlan: two alternating
    recordings, device-side AdamW step counter) reproduce eager steps."""
    r = run_ranks(1, py("tests/workers/graph_train_worker.py"), timeout=300,
                  env=dict(ENV, GT_TP="1", GT_MODE="token", GT_PLAN="1"))
    assert "graph train OK" in r.stdout


@pytest.mark.parametrize("n,tp", [(1, 1), (2, 2)])
def test_harness_forward_plan_matches_forward(n, tp):
    """The recorded launch plan of the harness forward (local form at TP = 1, push form at
    TP = 2) reproduces forward_images bitwise, and follows new pixels and new weights."""
    r = run_ranks(n, py("tests/workers/plan_worker.py"), timeout=300, env=dict(ENV, PL_TP=str(tp)))
    assert "plan OK" in r.stdout


@pytest.mark.parametrize("n,tp,mode", [(1, 1, "token"), (2, 2, "token"), (2, 2, "row"), (2, 1, "token")])
def test_harness_graph_train_matches_eager(n, tp, mode):
    """Training steps replayed from HIP graphs (two alternating captures, device-side AdamW
    step counter) reproduce eager steps: losses, weights, step count; TP and DP collectives
    inside the captured step."""
    r = run_ranks(n, py("tests/workers/graph_train_worker.py"), timeout=300,
                  env=dict(ENV, GT_TP=str(tp), GT_MODE=mode))
    assert "graph train OK" in r.stdout


@pytest.mark.parametrize("n", [2, 8])
def test_harness_fc_o_push_equals_plain(n):
    """the per-token fc_o's push form (row blocks stored into the TP
    owners' inboxes by the attention kernel, then inbox-to-local) is bitwise equal to the
    plain form (kernel + all-reduce of z), TP = 2 at 2 and 8 ranks on one GPU."""
    r = run_ranks(n, py("tests/workers/fc_o_push_worker.py"), timeout=300, env=ENV)
    assert "fc_o push OK" in r.stdout


def test_harness_token_push_matches_single_rank(reference_run, tmp_path):
    """The push form's training run reproduces the single-rank run (dp=1 x tp=2, token fc_o)."""
    out = tmp_path / "run.npz"
    run_ranks(2, py("tests/workers/harness_worker.py", "--tp", "2", "--mode", "token", "--out", str(out)),
              timeout=400, env=dict(ENV, CCMPI_TP_FC_O_FORM="push"))
    got = np.load(out)
    np.testing.assert_allclose(got["losses"], reference_run["losses"], rtol=2e-2, atol=2e-3)
    for k in ("q_w", "o_w", "emb_w"):
        np.testing.assert_allclose(got[k], reference_run[k], rtol=5e-2, atol=5e-3)


def test_harness_checkpoint_resume(tmp_path):
    """6 straight steps == 3 steps, checkpoint, resume, 3 more (dp=1 x tp=2)."""
    H = ["-m", "collective_communication_mpi_amd.models.harness", "--tp", "2", "--batch", "128"]
    a = tmp_path / "a.npy"
    c = tmp_path / "c.npy"
    ck = str(tmp_path / "ck")
    run_ranks(2, py(*H, "--steps", "6", "--log", str(a)), timeout=300, env=ENV)
    run_ranks(2, py(*H, "--steps", "3", "--ckpt", ck, "--save-every", "3"), timeout=300, env=ENV)
    r = run_ranks(2, py(*H, "--steps", "6", "--ckpt", ck, "--resume", "--log", str(c)), timeout=300, env=ENV)
    assert "resumed from" in r.stdout and "at step 3" in r.stdout
    la, lc = np.load(a), np.load(c)
    assert lc.shape == (3,)
    np.testing.assert_allclose(lc, la[3:], rtol=2e-3, atol=1e-4)


@pytest.mark.parametrize("n", [1, 2])
def test_parallel_swiglu_mlp_gpu(n):
    """ParallelSwiGLUMLP on the device plane: MFMA GEMMs, fused SwiGLU HIP kernels, TP
    all-reduces, vs single-process fp32 autograd (tests/workers/swiglu_mlp_worker.py)."""
    r = run_ranks(n, py("tests/workers/swiglu_mlp_worker.py", "--device", "cuda"), timeout=300, env=ENV)
    assert "swiglu mlp OK" in r.stdout


@pytest.mark.parametrize("n,route", [(2, "pair"), (4, "pair"), (8, "pair"), (2, "transpose")])
def test_swiglu_mlp_ring_gemm_beside_collectives_gpu(n, route):
    """the kernels an 8-GPU TP run uses (LDS-ring GEMMs, the SwiGLU
    epilogue, K-major backward rings) next to the other ranks' TP collectives on one GPU:
    CCMPI_SHARED_RING=1 keeps the ring on and holds every collective to half the CUs.  The
    worker also checks the push row mode against plain, bit for bit (8 ranks: the driver's
    8-GPU mlp phase runs it at TP = 8)."""
    # (route "pair", the default: dW reads both M-major operands on the pair ring; route
    # "transpose" with CCMPI_KMAJOR_MIN_MACS=1: these small shapes also take the round-4 dW
    # transpose route, with dh^T from the fused SwiGLU backward, across TP ranks)
    env = {**ENV, "CCMPI_SHARED_RING": "1", "CCMPI_RING_MIN_MACS": "1", "CCMPI_KMAJOR_MIN_MACS": "1",
           "CCMPI_KMAJOR_ROUTE": route}
    r = run_ranks(n, py("tests/workers/swiglu_mlp_worker.py", "--device", "cuda", "--big"), timeout=300, env=env)
    assert "swiglu mlp OK" in r.stdout


def test_tp_scratch_reused_across_token_counts():
    """varying token counts reuse one grow-only scratch block per role (no host
    call once the largest shape was seen), results vs fp32 at every M."""
    r = run_ranks(2, py("tests/workers/tp_varm_worker.py"), timeout=300, env=ENV)
    assert "varm OK" in r.stdout


@pytest.mark.parametrize("n", [2, 4])
def test_tensor_parallel_layers_and_ddp_gpu(n):
    """Column/RowParallelLinear (MFMA bf16 GEMMs, device TP collectives) + bucketed DDP
    on the device plane vs a single-process fp32 reference (tests/workers/tp_ddp_worker.py)."""
    r = run_ranks(n, py("tests/workers/tp_ddp_worker.py", "--device", "cuda"), timeout=300, env=ENV)
    assert "tp/ddp OK" in r.stdout


@pytest.mark.gpu
@pytest.mark.parametrize("schedule,steps", [("deferred", 2), ("auto", 7)])
def test_ddp_schedules_gpu(schedule, steps):
    """the deferred schedule (buckets all-reduced after the backward at the
    full CTA budget) matches the fp32 reference like the overlapped one; ``auto`` times both
    over its trial steps and settles on one (every step still checked)."""
    r = run_ranks(4, py("tests/workers/tp_ddp_worker.py", "--device", "cuda", "--schedule", schedule,
                        "--steps", str(steps)), timeout=300, env=ENV)
    assert "tp/ddp OK" in r.stdout
    if schedule == "auto":
        assert "choice={'chosen'" in r.stdout, r.stdout


def test_bench_tuning_table_drives_auto(tmp_path):
    """the bench's tuning sweep writes CCMPI_TUNE_FILE; a device group
    created afterwards loads it and ``auto`` runs what the table says (ring, RHD), 4 ranks."""
    r = run_ranks(4, py("tests/workers/tune_worker.py", "--file", str(tmp_path / "tune.json")), timeout=300, env=ENV)
    assert "tune OK" in r.stdout


@pytest.mark.parametrize("route", ["default", "transpose_all", "pair_all"])
def test_llama_ddp_gradient_sinks_gpu(route):
    """BASELINE config 5's machinery on a tiny Llama: DDP over 2 ranks with the TP layers'
    dW GEMMs writing straight into the buckets (gradient sinks), vs the mean of replica
    gradients; then measure_ddp_overlap's compute / comm / overlapped record.
    ``transpose_all``: every dW takes the transposed route into the pair ring (the sink's
    1/p alpha and bucket view as its output), as the full-size model's do."""
    env = dict(ENV)
    if route == "transpose_all":
        env.update({"CCMPI_SHARED_RING": "1", "CCMPI_RING_MIN_MACS": "1", "CCMPI_KMAJOR_MIN_MACS": "1",
                    "CCMPI_KMAJOR_MIN_DIM": "8", "CCMPI_KMAJOR_ROUTE": "transpose"})
    elif route == "pair_all":  # every dW on the pair ring's TA + TB form (the default route), small shapes too
        env.update({"CCMPI_SHARED_RING": "1", "CCMPI_RING_MIN_MACS": "1"})
    r = run_ranks(2, py("tests/workers/llama_dp_worker.py", "--device", "cuda", "--measure"), timeout=300, env=env)
    assert "llama dp OK" in r.stdout


def test_bench_multi_rank_path_shared_gpu():
    """bench.py's N >= 2 path (candidate loop, bf16, all-to-all, DP overlap, TP harness, TP MLP)
    with 4 ranks on this GPU, so an 8-GPU run is never the first execution of it."""
    import json
    import subprocess
    import sys

    from _launch import REPO

    e = dict(os.environ, **ENV)
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "4", "--steps", "3", "--warmup", "1", "--size-mb", "64",
                        "--a2a-mb", "16", "--dp-layers", "1", "--dp-tokens", "1024", "--dp-vocab", "0", "--batch", "256",
                        "--mlp-tokens", "512"],
                       cwd=REPO, env=e, capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, r.stderr[-4000:]
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    c = out["config"]
    assert out["n_gpus"] == 1 and c["result_exact"] and c["shared_gpu"]  # 4 ranks, one GPU
    assert set(c["candidates_ms"]) >= {"twoshot:256", "fanout:512", "push:512", "ring", "rhd"}
    assert all(v for v in c["candidates_ms"].values()), c["candidates_ms"]
    assert c["bf16_1GiB"]["algbw_GBps"] > 0 and c["alltoall"]["ms"] > 0
    dpo = c["dp_overlap"]
    assert dpo["comm_hidden_fraction"] is not None and dpo["schedule"] in ("overlap", "deferred")
    assert dpo["step_ms"] == min(dpo["overlapped_ms"], dpo["deferred_ms"])  # overlap can never lose
    assert c["parallelism"] == "dp2xtp2" and c["tp_fwd_step_ms"] > 0
    assert c["tp_mlp"]["tp"] == 4 and c["tp_mlp"]["fwd_bwd_ms"] > 0, c["tp_mlp"]  # TP MLP phase over all ranks
