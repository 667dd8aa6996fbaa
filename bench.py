"""Flagship benchmark (driver contract).

    python bench.py --gpus N --steps K --warmup W
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

Metric (BASELINE.json): "all-reduce algbw (GB/s) @1GiB fp32 + DP4xTP2 fwd step time".

* A step = one out-of-place all-reduce (SUM) of a 1 GiB fp32 buffer through the
  framework's HAND-WRITTEN device all-reduce.  Buffers come from the symmetric heap
  (``comm.empty``), the way framework users allocate communication buffers.
  ``value`` = algbw = 1 GiB / (time per all-reduce), the NCCL-tests convention:
  a property of the whole collective, identical for every rank.  Per-GPU work
  is fixed as N grows (weak scaling).  At N = 1 the all-reduce is a local copy,
  so that number is a copy bandwidth (see ``shared_gpu_dry_run`` below).
* The algorithm is picked once per run, like RCCL's tuner does.  Every
  candidate runs once and is checked for an exact result (rank-valued inputs,
  so fp32 sums are exact) before it is timed: the hand-written two-shot and
  fan-out two-shot over IPC-mapped xGMI peer memory at several CTA budgets, the
  push two-shot, the hand-written multi-ring and recursive halving/doubling
  kernels.  Every candidate's time is reported.  At N >= 2 a size sweep
  (``DeviceGroup.tune``) follows, written as a tuning table that every later
  phase's device groups load (``CCMPI_TUNE_FILE``), so ``algo="auto"`` in the TP
  and DDP layers uses what was measured on this node.  At N >= 4 the harness's
  2-rank TP groups (a table key of their own) are swept as well, up to 16 MiB.
* Every measurement runs in a supervised child phase of fresh processes (the
  process that ``bench.py`` starts never touches the GPU), each under its own
  wall-clock budget; rank 0 merges their JSON records into the one output line.
  A phase that crashes, hangs or errors costs only its own entry (the ``coll`` phase
  writes its record as soon as the headline is measured, so a failure in its tuning
  sweep leaves ``value`` in place, marked ``partial``):

  ====================  =========================================================
  ``coll``              the headline (hand-written all-reduce candidates, 1 GiB
                        fp32) + bf16 + all-to-all 256 MiB/rank + tuning sweep
  ``harness``           DP x TP transformer-layer forward (HIP graph) and train
                        step, TP=2 x DP=N/2 for N >= 2 (DP4xTP2 at N = 8)
  ``mlp``               TP Llama-3-8B MLP block over all ranks (hand-written MFMA
                        GEMMs, SwiGLU epilogue, TP all-reduces; unfused, chunked-
                        overlap, fused and push row-parallel variants)
  ``dp``                BASELINE config 5: DP over all ranks of a Llama-3-8B-sized
                        model (16 GB bf16 gradients) through ``DistributedDataParallel``,
                        bucket all-reduces launched from autograd hooks during a real
                        backward (parallel/llama_dp.py), N >= 2
  ``rccl``              the RCCL library baseline (the role MPI's built-ins play in
                        the reference's mpi-test.py:42-98,178-239), N >= 2.  Reported
                        in ``config.rccl`` with ``handwritten_vs_rccl``; it never
                        replaces the hand-written headline.
  ``shared_gpu_dry_run``  (N = 1 only) the N >= 2 bench, 8 ranks on this one GPU, so
                        the 8-GPU path is exercised before any 8-GPU run.  Its numbers
                        measure HBM + protocol, not xGMI.
  ====================  =========================================================

The timed region is W untimed steps, then a barrier + device sync, K steps,
and another device sync + barrier.  The time is the MAX over ranks.  Rank 0
prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

GiB = 1 << 30
XGMI_LINK_GBPS = 153.6  # MI355X xGMI, per link and direction (7 links x 153.6 = 1075 GB/s per GPU)
METRIC = "all-reduce algbw (GB/s) @1GiB fp32 + DP4xTP2 fwd step time, 1/2/4/8 MI355X"
PHASES = ("coll", "harness", "mlp", "dp", "rccl", "host")


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--size-mb", type=int, default=1024)
    ap.add_argument("--algo", default="auto", help="auto | twoshot | push | ring | rhd | oneshot | fanout | ...")
    ap.add_argument("--tp", type=int, default=0, help="TP degree of the harness step (default 2 if N>=2)")
    ap.add_argument("--batch", type=int, default=2048, help="images per DP replica for the harness step")
    ap.add_argument("--fc-o-mode", default="token", choices=["token", "row"],
                    help="harness fc_o: per-token row-parallel (reference shape) or pooled")
    ap.add_argument("--dp-layers", type=int, default=32, help="Llama-3-8B decoder layers of the DP-overlap phase")
    ap.add_argument("--dp-tokens", type=int, default=4096, help="tokens per rank of the DP-overlap phase")
    ap.add_argument("--dp-vocab", type=int, default=1,
                    help="DP overlap: include the LM head and token embedding (Llama-3-8B: 16.06 GB of gradients)")
    ap.add_argument("--dp-scripted", type=int, default=0,
                    help="DP phase: also measure the scripted wgrad-only overlap (parallel/overlap.py) as a secondary")
    ap.add_argument("--a2a-mb", type=int, default=256)
    ap.add_argument("--mlp-tokens", type=int, default=4096,
                    help="tokens of the TP Llama-3-8B MLP record (tp_mlp: TP over all ranks; 0 = off)")
    ap.add_argument("--tune-max-mb", type=int, default=256, help="N >= 2: largest size of the tuning sweep (0 = off)")
    ap.add_argument("--shared-dry-run", type=int, default=8, help="N=1: ranks of the shared-GPU dry run (0 = off)")
    ap.add_argument("--variants", default="fast", choices=["fast", "all"],
                    help="secondary variants: 'fast' skips the ones that cannot win (token_chunks4 fc_o, "
                         "fused MLP row mode: 11x / 3.4x slower than plain, BENCH_r05 / profiles/r5_rehearse8)")
    ap.add_argument("--no-harness", action="store_true")
    ap.add_argument("--no-secondary", action="store_true")
    ap.add_argument("--verbose", action="store_true")
    ap.add_argument("--phase", default="", choices=("",) + PHASES,
                    help="internal: which child phase this process runs (set by the supervisor)")
    ap.add_argument("--result", default="", help="internal: where a child phase writes its JSON")
    ap.add_argument("--coll-timeout", type=float, default=900.0, help="wall-clock budget of the collective phase (s)")
    ap.add_argument("--harness-timeout", type=float, default=300.0, help="wall-clock budget of the harness phase (s)")
    ap.add_argument("--rccl-timeout", type=float, default=300.0, help="wall-clock budget of the RCCL phase (s)")
    ap.add_argument("--dp-timeout", type=float, default=600.0, help="wall-clock budget of the DP-overlap phase (s)")
    ap.add_argument("--mlp-timeout", type=float, default=300.0, help="wall-clock budget of the TP MLP phase (s)")
    ap.add_argument("--no-rccl", action="store_true", help="skip the RCCL baseline phase")
    ap.add_argument("--host-ranks", type=int, default=8,
                    help="BASELINE config 1: CPU processes of the host-plane phase (0 = off)")
    ap.add_argument("--host-count", type=int, default=1024, help="host phase: float32 elements per buffer")
    ap.add_argument("--host-runs", type=int, default=100, help="host phase: timed runs (reference: 100)")
    ap.add_argument("--host-warmup", type=int, default=400,
                    help="host phase: untimed runs between the cold pass and the timed warm pass")
    ap.add_argument("--host-timeout", type=float, default=180.0, help="wall-clock budget of the host phase (s)")
    return ap.parse_args(argv)


# ------------------------------------------------------------------ supervision
def relaunch(n: int) -> int:
    """--gpus N without a launcher: start N ranks with the framework launcher
    (child processes; this process never touches the GPU)."""
    from collective_communication_mpi_amd.launch import launch

    argv = [sys.executable, os.path.abspath(__file__)] + sys.argv[1:]
    # rank r on the CPUs local to the GPU it drives, an L3 domain of its own (topology.py)
    return launch(n, argv, env_extra={"CCMPI_BENCH_CHILD": "1", "CCMPI_BIND": os.environ.get("CCMPI_BIND", "gpu")})


def _env_rank():
    """(rank, size, local rank) from whichever launcher started this process."""
    e = os.environ
    for rk, sk in (("CCMPI_RANK", "CCMPI_SIZE"), ("RANK", "WORLD_SIZE"), ("PMI_RANK", "PMI_SIZE"),
                   ("OMPI_COMM_WORLD_RANK", "OMPI_COMM_WORLD_SIZE")):
        if rk in e and sk in e:
            r, n = int(e[rk]), int(e[sk])
            break
    else:
        r, n = 0, 1
    local = int(e.get("LOCAL_RANK", e.get("CCMPI_LOCAL_RANK", e.get("MPI_LOCALRANKID", r))))
    return r, n, local


def _run_child(cmd, env, budget: float, abort_flag: str = "", cpus=None):
    """Run one phase child in its own session; kill its process group at the budget, or as
    soon as ``abort_flag`` exists (another rank's child of this phase failed: its peers
    would wait for it in their next collective until the budget).  A child that fails
    creates the flag for the others.  ``cpus``: the child's CPU binding (set before it
    starts, so its GPU runtime's threads inherit it).  Returns (returncode or None if
    killed, seconds)."""
    import signal

    t0 = time.monotonic()
    def pre(c=frozenset(cpus or ())):
        try:
            os.sched_setaffinity(0, c)
        except OSError:  # (a set outside this container's cpuset: the OS places the child)
            pass

    p = subprocess.Popen(cmd, env=env, cwd=REPO, start_new_session=True, preexec_fn=pre if cpus else None)
    rc = None
    while True:
        try:
            rc = p.wait(timeout=0.25)
            break
        except subprocess.TimeoutExpired:
            pass
        if time.monotonic() - t0 > budget or (abort_flag and os.path.exists(abort_flag)):
            for sig in (signal.SIGTERM, signal.SIGKILL):
                try:
                    os.killpg(p.pid, sig)
                except ProcessLookupError:
                    break
                try:
                    p.wait(timeout=10)
                    break
                except subprocess.TimeoutExpired:
                    continue
            rc = None
            break
    if rc != 0 and abort_flag:
        try:
            open(abort_flag, "a").close()
        except OSError:
            pass
    return rc, time.monotonic() - t0


def phase_binding(world, rank: int, local: int):
    """(CPU set for this rank's GPU phase children or None, binding mode).  Launched by
    ``launch.py`` (``CCMPI_BOUND_CPUS`` set): the children inherit that binding.  Launched by
    torchrun (nobody bound us): rank 0 reads the GPU-local plan from sysfs once
    (``topology.gpu_plan``, before any GPU call) and every rank takes its local rank's set,
    so both launch paths place ranks the same way.  ``CCMPI_BIND=none`` (or anything other
    than ``gpu``) leaves placement to the OS."""
    mode = os.environ.get("CCMPI_BIND", "gpu")
    if os.environ.get("CCMPI_BOUND_CPUS"):
        return None, os.environ.get("CCMPI_BIND_EFFECTIVE", mode)
    plan = None
    if mode == "gpu" and rank == 0:
        from collective_communication_mpi_amd.launch import _cpu_busy
        from collective_communication_mpi_amd.topology import gpu_plan

        nloc = int(os.environ.get("LOCAL_WORLD_SIZE", os.environ.get("CCMPI_LOCAL_SIZE", world.Get_size())))
        try:
            plan = gpu_plan(nloc, busy=_cpu_busy())
        except Exception as e:  # (any failure: every rank still reaches the bcast below)
            print(f"[bench] GPU-local placement unavailable ({type(e).__name__}: {e}); OS placement", file=sys.stderr)
            plan = None
    plan = world.bcast(plan, root=0) if mode == "gpu" else None
    if not plan or local >= len(plan):
        return None, "none"
    return plan[local], "gpu"


def plan_phases(args, size: int):
    """(phase, budget) in run order for a job of ``size`` ranks."""
    out = [("coll", args.coll_timeout)]
    sec = not args.no_secondary
    if not args.no_harness:
        out.append(("harness", args.harness_timeout))
    if sec and args.mlp_tokens > 0:
        out.append(("mlp", args.mlp_timeout))
    if sec and size > 1 and args.dp_layers > 0:
        out.append(("dp", args.dp_timeout))
    if size > 1 and not args.no_rccl:
        out.append(("rccl", args.rccl_timeout))
    if sec and args.host_ranks > 1:
        out.append(("host", args.host_timeout))
    return out


def empty_headline(args, size: int, why: str) -> dict:
    return {"metric": METRIC, "value": 0.0, "unit": "GB/s", "n_gpus": size, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": None, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "fp32", "data": "synthetic", "config": {"error": why}}


def merge_results(args, size: int, status: dict, load) -> dict:
    """Rank 0: the one output line from the phases' records.  ``load(phase)`` returns a
    phase's JSON or None.  The headline comes only from the ``coll`` phase; every other
    phase fills its own key and a failed phase leaves an error there, nothing else."""
    out = load("coll") if status.get("coll", {}).get("ok") else None
    if out is None:
        # the coll phase writes its record once the headline is measured, before the
        # secondary tuning sweep: a sweep that dies or hangs keeps the headline
        early = load("coll")
        if early and early.get("partial"):
            out = early
            out.setdefault("config", {})["coll_phase_error"] = f"after the headline: {status.get('coll')}"
    if out is None:
        out = empty_headline(args, size, f"collective phase failed: {status.get('coll')}")
    c = out.setdefault("config", {})

    def rec(phase):
        r = load(phase) if status[phase]["ok"] else None
        return r if r is not None else {"error": f"{phase} phase failed or timed out: {status[phase]}"}

    if "harness" in status:
        h = rec("harness")
        c["harness"] = h
        if "error" not in h:
            c["tp_fwd_step_ms"] = h.pop("fwd_ms", None)
            c["tp_train_step_ms"] = h.pop("train_ms", None)
            c["global_batch"] = h.get("global_batch")
            c["seq_len"] = h.get("seq_len")
            c["parallelism"] = f"dp{h.get('dp')}xtp{h.get('tp')}"
    if "mlp" in status:
        c["tp_mlp"] = rec("mlp")
    if "dp" in status:
        c["dp_overlap"] = rec("dp")
    if "rccl" in status:
        merge_rccl(out, load("rccl") if status["rccl"]["ok"] else None, status["rccl"])
    if "host" in status:
        c["host_cpu"] = rec("host")  # BASELINE config 1 (8 CPU processes, 1k float32)
    c["phases"] = status
    if out.get("partial") and not status.get("coll", {}).get("ok"):
        # the headline survived a failure later in the coll phase: say so at the top level
        out["warning"] = "coll phase failed after the headline was measured (config.coll_phase_error)"
    return out


def merge_rccl(out: dict, rr, status: dict) -> None:
    """Fold the RCCL phase into the record as the library comparison.  The headline
    ``value`` stays the hand-written all-reduce (the north star's product); RCCL goes
    to ``config.rccl`` and ``config.handwritten_vs_rccl`` = hand-written / RCCL algbw."""
    c = out.setdefault("config", {})
    if rr is None or "error" in rr:
        c["rccl"] = {"error": (rr or {}).get("error") or f"RCCL phase failed or timed out: {status}"}
        return
    c["rccl"] = rr
    if rr.get("algbw_GBps") and out.get("value"):
        c["handwritten_vs_rccl"] = round(out["value"] / rr["algbw_GBps"], 3)
    b16 = c.get("bf16_1GiB")
    if b16 and rr.get("bf16_algbw_GBps"):
        b16["handwritten_vs_rccl"] = round(b16["algbw_GBps"] / rr["bf16_algbw_GBps"], 3)
    a2a = c.get("alltoall")
    if a2a and rr.get("alltoall_ms"):
        a2a["rccl_ms"] = dict(rr["alltoall_ms"])


def supervise(args) -> int:
    """This process never touches the GPU.  It runs every phase as a child process
    group of ``size`` fresh ranks (each with its own host-plane job id) under a
    wall-clock budget, and rank 0 merges the JSON records into the one output line."""
    import shutil
    import tempfile
    import uuid

    from collective_communication_mpi_amd import mpi as MPI  # host plane only (CPU)

    world = MPI.COMM_WORLD
    rank, size = world.Get_rank(), world.Get_size()
    _, _, local = _env_rank()
    tmp = world.bcast(tempfile.mkdtemp(prefix="ccmpi_bench_") if rank == 0 else None, root=0)
    job = world.bcast(uuid.uuid4().hex[:12] if rank == 0 else None, root=0)
    # the collective phase's tuning sweep -> every later phase's device groups (auto)
    tune_file = os.environ.get("CCMPI_TUNE_FILE") or os.path.join(tmp, "tune.json")
    argv = list(sys.argv[1:])
    from collective_communication_mpi_amd.topology import format_cpu_list

    cpus, bind_mode = phase_binding(world, rank, local)
    bound = world.allgather(format_cpu_list(cpus if cpus else os.sched_getaffinity(0)))
    status = {}
    for phase, budget in plan_phases(args, size):
        env = dict(os.environ, CCMPI_RANK=str(rank), CCMPI_SIZE=str(size), CCMPI_LOCAL_RANK=str(local),
                   CCMPI_LOCAL_SIZE=os.environ.get("LOCAL_WORLD_SIZE", os.environ.get("CCMPI_LOCAL_SIZE", str(size))),
                   LOCAL_RANK=str(local), CCMPI_JOBID=f"{job}-{phase}", CCMPI_BENCH_WORKER="1",
                   CCMPI_TUNE_FILE=tune_file)
        if phase in ("mlp", "dp"):
            # ranks sharing a GPU (a rehearsal) keep the ring GEMMs an 8-GPU run uses, every
            # collective held within half the CUs (device.py); one rank per GPU: no effect
            env.setdefault("CCMPI_SHARED_RING", "1")
        pp = env.get("PYTHONPATH", "")
        env["PYTHONPATH"] = REPO + (os.pathsep + pp if pp else "")
        cmd = [sys.executable, os.path.abspath(__file__), *argv, "--phase", phase,
               "--result", os.path.join(tmp, f"{phase}.json")]
        if rank == 0:
            print(f"[bench] phase {phase} (budget {budget:.0f}s) ...", file=sys.stderr, flush=True)
        if phase == "host":
            # BASELINE config 1 is an 8-process CPU job whatever N is: rank 0 launches it
            # (host plane only, a job of its own), the other ranks wait
            rc, secs = 0, 0.0
            if rank == 0:
                for k in ("CCMPI_RANK", "CCMPI_SIZE", "CCMPI_LOCAL_RANK", "CCMPI_LOCAL_SIZE", "CCMPI_JOBID"):
                    env.pop(k, None)
                # CPU ranks exchange shared-memory cache lines: one CCD (launch.py ``l3``)
                env["CCMPI_BIND"] = os.environ.get("CCMPI_HOST_BIND", "l3")
                for k in ("CCMPI_BOUND_CPUS", "CCMPI_BIND_EFFECTIVE"):
                    env.pop(k, None)
                cmd = [sys.executable, "-m", "collective_communication_mpi_amd.launch", "-n", str(args.host_ranks),
                       "--timeout", str(int(budget)), *cmd]
                rc, secs = _run_child(cmd, env, budget + 15)
        else:
            if cpus:
                env["CCMPI_BOUND_CPUS"] = format_cpu_list(cpus)
                env["CCMPI_BIND_EFFECTIVE"] = bind_mode
            rc, secs = _run_child(cmd, env, budget, abort_flag=os.path.join(tmp, f"{phase}.abort"), cpus=cpus)
        if rank == 0:
            print(f"[bench] phase {phase}: rc {rc}, {secs:.1f}s", file=sys.stderr, flush=True)
        ok = world.allreduce(int(rc == 0), op=MPI.MIN)
        rcs = world.allgather(rc)
        status[phase] = {"ok": bool(ok), "returncodes": rcs, "seconds": round(secs, 1)}
        if phase != "host":
            status[phase].update(binding=bind_mode, bound_cpus=bound)
        world.Barrier()  # no child of this phase is alive anywhere before the next starts
    rc = 0
    if rank == 0:
        def load(name):
            try:
                with open(os.path.join(tmp, f"{name}.json")) as f:
                    return json.load(f)
            except (OSError, ValueError):
                return None

        out = merge_results(args, size, status, load)
        if not status["coll"]["ok"] and not out.get("partial"):
            rc = 1
        if size == 1 and args.shared_dry_run > 1 and not args.no_secondary:
            out["config"]["shared_gpu_dry_run"] = shared_dry_run(args.shared_dry_run, steps=5, warmup=2,
                                                                 verbose=args.verbose)
        print(json.dumps(out), flush=True)
        shutil.rmtree(tmp, ignore_errors=True)
    world.Barrier()
    return rc


def shared_dry_run(n: int, steps: int, warmup: int, verbose: bool):
    """Run this bench with n ranks on this GPU (the N >= 2 path) and return its JSON.

    One hardware queue per process (``GPU_MAX_HW_QUEUES=1``): with HIP's default of 4,
    8 processes ask for up to 32 queues, the scheduler time-slices the ones it cannot
    map and the DP4xTP2 forward measured 1.6-7.0 ms instead of ~0.6 ms
    (profiles/r3_dryrun).  ``CCMPI_DRYRUN_HW_QUEUES`` overrides (empty = HIP default)."""
    cmd = [sys.executable, "-m", "collective_communication_mpi_amd.launch", "-n", str(n), "--timeout", "600",
           sys.executable, os.path.abspath(__file__), "--gpus", str(n), "--steps", str(steps), "--warmup", str(warmup),
           "--dp-layers", "0", "--a2a-mb", "64", "--shared-dry-run", "0", "--no-rccl", "--mlp-tokens", "0",
           "--tune-max-mb", "16", "--host-ranks", "0"]
    env = dict(os.environ, CCMPI_BENCH_CHILD="1")
    # the placement an N-GPU run uses (every rank on its GPU's CPUs, a CCD each);
    # CCMPI_DRYRUN_BIND=l3|none for the A/B (profiles/r6_bind)
    env["CCMPI_BIND"] = os.environ.get("CCMPI_DRYRUN_BIND", "gpu")
    q = os.environ.get("CCMPI_DRYRUN_HW_QUEUES", "1")
    if q:
        env["GPU_MAX_HW_QUEUES"] = q
    try:
        r = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=660)
    except subprocess.TimeoutExpired:
        return {"error": "timeout"}
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    if r.returncode != 0 or not lines:
        return {"error": f"rc={r.returncode}", "stderr_tail": r.stderr[-800:]}
    out = json.loads(lines[-1])
    if verbose:
        print("[bench] shared dry run:", lines[-1][:400], file=sys.stderr)
    keep = {k: out[k] for k in ("value", "ms_per_step", "n_gpus")}
    keep["ranks"] = n
    keep["unit"] = "GB/s (1 GiB fp32 all-reduce algbw)"
    keep["note"] = f"{n} ranks sharing ONE GPU through IPC: HBM + protocol, not xGMI"
    keep["hw_queues_per_rank"] = env.get("GPU_MAX_HW_QUEUES", "HIP default")
    keep["binding"] = env["CCMPI_BIND"]
    keep["placement"] = out["config"].get("placement")
    keep.update({k: out["config"].get(k) for k in ("allreduce_algo", "busbw_GBps", "candidates_ms", "candidates",
                                                     "result_exact", "self_test", "bf16_1GiB", "alltoall",
                                                     "alltoall_pairwise", "sweep", "tuning", "tp_fwd_step_ms",
                                                     "tp_train_step_ms", "parallelism", "harness", "phases")})
    return keep


# ------------------------------------------------------------------ phase helpers
def _setup_phase(timeout_s: str):
    """Common child-phase bring-up: device timeout, crash reporter, communicator, device."""
    os.environ.setdefault("CCMPI_DEVICE_TIMEOUT_S", timeout_s)
    import faulthandler

    faulthandler.enable()
    from collective_communication_mpi_amd import MPI, Communicator, _native

    _native.host().install_crash_handler(2)  # native backtrace if the phase crashes (rc -11 is then explained)
    import torch

    comm = Communicator(MPI.COMM_WORLD)
    local = _env_rank()[2]
    torch.cuda.set_device(local % torch.cuda.device_count())
    _PLACEMENT[:] = comm.comm.allgather(_check_placement(torch))
    return comm


_PLACEMENT: list = []  # per rank, set by _setup_phase: where the phase child runs


def _check_placement(torch) -> str:
    """This rank's CPU binding against the GPU the runtime opened (topology.check_bound:
    a binding with no CPU on the GPU's side is moved there, every thread, and reported)."""
    from collective_communication_mpi_amd.topology import check_bound

    try:
        props = torch.cuda.get_device_properties(torch.cuda.current_device())
        r = check_bound(props)
        gpu = f"{getattr(props, 'pci_domain_id', 0):04x}:{props.pci_bus_id:02x}:{props.pci_device_id:02x}"
        where = {True: "gpu-local", False: "NOT gpu-local", None: "gpu cpus unknown"}[r.get("gpu_local")]
        return (f"cpus={r['bound_cpus']} gpu={gpu} {where}"
                + (f" (re-bound {r['rebound_threads']} threads)" if "rebound_threads" in r else ""))
    except Exception as e:  # noqa: BLE001 - a record field, never a failure
        return f"unknown ({type(e).__name__}: {e})"[:200]


def _fault_injection(phase: str) -> None:
    """Tests: ``CCMPI_BENCH_FAULT=<phase>`` makes that phase's rank 0 die by SIGSEGV
    after its GPU work started, like the round-3 harness crash."""
    if os.environ.get("CCMPI_BENCH_FAULT") == phase and _env_rank()[0] == 0:
        import signal

        os.kill(os.getpid(), signal.SIGSEGV)


def _timers(comm):
    import torch

    from collective_communication_mpi_amd import MPI

    hc = comm.comm

    def sync_barrier():
        torch.cuda.synchronize()
        hc.Barrier()

    def timed(fn, iters) -> float:
        """Seconds per call: barrier + device sync on both sides, MAX over ranks."""
        sync_barrier()
        t0 = time.perf_counter()
        for _ in range(iters):
            fn()
        sync_barrier()
        return hc.allreduce(time.perf_counter() - t0, op=MPI.MAX) / iters

    return sync_barrier, timed


def allreduce_candidates(world: int, shared: bool, algo: str = "auto"):
    """Hand-written all-reduce algorithms the headline tries (CTA budgets after the ':')."""
    if world == 1:
        return ["twoshot"]  # single rank: the all-reduce is a device copy
    if algo != "auto":
        return [algo]
    hand = ["twoshot:256", "twoshot:512", "fanout:256", "fanout:512", "fanout_lds:512", "push:512", "ring"]
    if world & (world - 1) == 0:
        hand.append("rhd")
    return hand


def _base_algo(algo: str) -> str:
    """The self-test family of a candidate (``fanout_lds:512`` -> ``fanout``)."""
    b = algo.split(":")[0]
    return "fanout" if b == "fanout_lds" else b


def order_candidates(cands, self_test, disabled):
    """(candidates in try order, {skipped candidate: reason}).  Candidates whose algorithm
    family failed the bring-up ``self_test`` (``DeviceGroup.disabled``, also
    ``CCMPI_DISABLE_ALGOS``) are skipped; those whose family passed it come first, the
    untested families (push, ring, RHD) after them, each group in the given order."""
    skipped = {a: "disabled (failed self_test or CCMPI_DISABLE_ALGOS)" for a in cands
               if a.split(":")[0] in disabled or _base_algo(a) in disabled}
    st = self_test or {}
    keep = [a for a in cands if a not in skipped]
    return sorted(keep, key=lambda a: 0 if st.get(_base_algo(a)) else 1), skipped


def pick_candidates(cands, attempt, agree, reset, timer, log=lambda *a: None):
    """Try every candidate, whatever happened to the ones before it (collective: every rank
    runs the same sequence).  ``attempt(c)`` runs ``c`` once and returns None or this rank's
    error text (an exception counts as an error); ``agree(err)`` returns None when every rank
    succeeded, else the first failing rank's error (host all-gather); ``reset()`` restores
    the device state after a failure (a timed-out kernel leaves per-CTA epochs
    inconsistent); ``timer(c)`` returns seconds per call, followed by one more ``agree`` on
    the device error state after timing.  Returns ({candidate: {"ms", "error"}}, fastest
    or None).  Like the reference's per-run oracle check (mpi-test.py:75-84): a mismatch
    is reported, the run goes on."""
    out = {}
    for c in cands:
        try:
            err = attempt(c)
        except Exception as e:  # noqa: BLE001 - any failure disqualifies the candidate, not the run
            err = f"{type(e).__name__}: {e}"
        err = agree(err)
        t = None
        if not err:
            try:
                t = timer(c)
                err = None
            except Exception as e:  # noqa: BLE001
                err = f"during timing: {type(e).__name__}: {e}"
            err = agree(err)
        if err:
            log(f"candidate {c} failed: {err}")
            out[c] = {"ms": None, "error": str(err)[:400]}
            reset()
            continue
        out[c] = {"ms": round(t * 1e3, 4), "error": None}
        log(f"candidate {c}: {t * 1e3:.3f} ms")
    good = {c: o["ms"] for c, o in out.items() if o["ms"]}
    return out, (min(good, key=good.get) if good else None)


def _injected(algo: str, kind: str) -> bool:
    """Tests: ``CCMPI_BENCH_FAULT=candidate:<algo>[,candidate_bf16:<algo>,...]`` makes rank 0
    skip that candidate's kernel (its peers then time out in theirs, as on a broken link)
    and report the failure.  ``candidate:`` matches fp32 and bf16, ``candidate_<kind>:``
    only that kind; ``*`` matches every algorithm."""
    if _env_rank()[0] != 0:
        return False
    for ent in os.environ.get("CCMPI_BENCH_FAULT", "").split(","):
        pre, _, a = ent.partition(":")
        if pre in ("candidate", f"candidate_{kind}") and a in ("*", algo):
            return True
    return False


def _device_agree(comm):
    """``agree`` of ``pick_candidates`` over the host plane, with the device's error state
    (a timeout code names phase and peer) folded into this rank's error."""
    dev, hc = comm.dev, comm.comm

    def agree(err):
        try:
            dev.check()
        except Exception as e:  # noqa: BLE001
            err = f"{err}; {e}" if err else str(e)
        errs = hc.allgather(err)
        bad = [(r, e) for r, e in enumerate(errs) if e]
        return "; ".join(f"rank {r}: {e}" for r, e in bad[:3]) if bad else None

    return agree


def _bw(nbytes: int, ms, world: int, ar: bool = True) -> dict:
    if not ms:
        return {"algbw_GBps": None, "busbw_GBps": None}
    alg = nbytes / (ms / 1e3) / 1e9
    f = (2 * (world - 1) / world if ar else (world - 1) / world) if world > 1 else 0.0
    return {"algbw_GBps": round(alg, 2), "busbw_GBps": round(alg * f, 2)}


def run_headline(comm, args, log=lambda *a: None) -> dict:
    """The headline (collective: every rank calls): bring-up self test, every hand-written
    all-reduce candidate on the 1 GiB fp32 buffer (each checked exact, then timed; a failed
    one is reset away and the next is tried), then the K timed steps of the fastest.
    Returns the record fields plus the buffers for the secondaries (``x``, ``y``)."""
    import torch

    from collective_communication_mpi_amd import MPI

    rank, world = comm.Get_rank(), comm.Get_size()
    dev, hc = comm.dev, comm.comm
    sync_barrier, timed = _timers(comm)
    # bring-up check of the algorithms `auto` picks on this fabric: a failing one is
    # disabled on every rank (and its candidates are skipped below)
    self_test = dev.self_test() if world > 1 else None
    log(f"self test: {self_test}")
    nbytes = args.size_mb << 20
    x = dev.empty(nbytes // 4, torch.float32)
    y = dev.empty(nbytes // 4, torch.float32)
    x.fill_(float(rank + 1))
    expect = float(world * (world + 1) // 2)
    cands, skipped = order_candidates(allreduce_candidates(world, dev.shared_device, args.algo), self_test,
                                      dev.disabled)
    outcomes, best = pick_candidates(cands, *allreduce_trial(comm, x, y, expect, "fp32"), log=log)
    outcomes.update({a: {"ms": None, "error": why} for a, why in skipped.items()})
    if best is None:
        raise SystemExit(f"no all-reduce algorithm produced a correct result: {outcomes}")
    for _ in range(args.warmup):
        dev.allreduce(x, y, "SUM", best, symmetric=True)
    t_step = timed(lambda: dev.allreduce(x, y, "SUM", best, symmetric=True), args.steps)
    torch.cuda.synchronize()
    final_ok = bool(hc.allreduce(int(bool(torch.all(y == expect).item())), op=MPI.MIN))
    algbw = nbytes / t_step / 1e9
    busbw = algbw * (2 * (world - 1) / world) if world > 1 else 0.0
    return {"algbw": algbw, "busbw": busbw, "t_step": t_step, "best": best, "outcomes": outcomes,
            "results": {a: o["ms"] for a, o in outcomes.items()}, "final_ok": final_ok, "self_test": self_test,
            "x": x, "y": y, "expect": expect}


def allreduce_trial(comm, xin, yout, expect: float, kind: str):
    """(attempt, agree, reset, timer) of ``pick_candidates`` for all-reduce candidates on the
    symmetric buffers ``xin`` -> ``yout`` (rank-valued input: the exact result is known)."""
    import torch

    dev = comm.dev
    sync_barrier, timed = _timers(comm)

    def attempt(algo):
        yout.zero_()
        sync_barrier()
        if _injected(algo, kind):
            return "injected fault (CCMPI_BENCH_FAULT): kernel skipped on rank 0"
        dev.allreduce(xin, yout, "SUM", algo, symmetric=True)
        torch.cuda.synchronize()
        dev.check()
        return None if bool(torch.all(yout == expect).item()) else "wrong result"

    def timer(algo):
        dev.allreduce(xin, yout, "SUM", algo, symmetric=True)
        return timed(lambda: dev.allreduce(xin, yout, "SUM", algo, symmetric=True), 3)

    return attempt, _device_agree(comm), dev.reset, timer


def run_secondaries(comm, args, h: dict, log=lambda *a: None, groups=("bf16", "a2a")) -> dict:
    """The secondary device collectives after the headline (collective): the 1 GiB bf16
    all-reduce (BASELINE config 2: the three fastest fp32 candidates, plus the hand-written
    ring timed on its own), and the all-to-all of ``--a2a-mb`` per rank (config 3: direct,
    push and pairwise, the pairwise time reported under its own key).  Every block that
    fails records an error instead of raising."""
    import torch

    rank, world = comm.Get_rank(), comm.Get_size()
    dev = comm.dev
    _, timed = _timers(comm)
    x, y, expect = h["x"], h["y"], h["expect"]
    nbytes = x.numel() * 4
    sec = {}
    if "bf16" in groups:
        xb, yb = x.view(torch.bfloat16), y.view(torch.bfloat16)
        xb.fill_(float(rank + 1))  # rank-valued: exact in bf16
        good = {a: o["ms"] for a, o in h["outcomes"].items() if o["ms"]}
        top = sorted(good, key=good.get)[:3]
        if world > 1 and "ring" not in top and args.algo == "auto":
            top.append("ring")  # BASELINE config 2 names the ring: always a bf16 point of its own
        res16, best16 = pick_candidates(top, *allreduce_trial(comm, xb, yb, expect, "bf16"), log=log)
        b16 = {"candidates": res16, "candidates_ms": {a: o["ms"] for a, o in res16.items()}}
        if best16 is None:
            b16["error"] = "no bf16 candidate produced a correct result"
        else:
            t16 = timed(lambda: dev.allreduce(xb, yb, "SUM", best16, symmetric=True), max(3, args.steps // 2))
            b16.update({"algo": best16, "ms": round(t16 * 1e3, 4), **_bw(nbytes, t16 * 1e3, world)})
        if "ring" in res16:
            b16["ring"] = {"ms": res16["ring"]["ms"], "error": res16["ring"]["error"],
                           **_bw(nbytes, res16["ring"]["ms"], world)}
        sec["bf16_1GiB"] = b16
    if "a2a" in groups:
        an = min((args.a2a_mb << 20) // 4, x.numel()) // world * world  # within the 1 GiB buffers
        blk = an // world
        xa, ya = x[:an], y[:an]
        xa.view(world, blk).copy_((rank * world + torch.arange(world, device=dev.device, dtype=torch.float32))
                                  .view(world, 1).expand(world, blk))
        want = (torch.arange(world, device=dev.device, dtype=torch.float32) * world + rank).view(world, 1).expand(world, blk)
        sync_barrier, _ = _timers(comm)

        def attempt(algo):
            ya.zero_()
            sync_barrier()
            if _injected(algo, "a2a"):
                return "injected fault (CCMPI_BENCH_FAULT): kernel skipped on rank 0"
            dev.alltoall(xa, ya, algo)
            torch.cuda.synchronize()
            dev.check()
            return None if torch.equal(ya.view(world, blk), want) else "wrong result"

        res, ba = pick_candidates(["direct", "push", "pairwise"], attempt, _device_agree(comm), dev.reset,
                                  lambda algo: timed(lambda: dev.alltoall(xa, ya, algo), 5), log=log)
        ms = res[ba]["ms"] if ba else None
        sec["alltoall"] = {"bytes_per_rank": an * 4, "algo": ba, "ms": ms,
                           "algbw_GBps": round(an * 4 / (ms / 1e3) / 1e9, 2) if ms else None,
                           "candidates_ms": {a: o["ms"] for a, o in res.items()}, "candidates": res}
        if not ba:
            sec["alltoall"]["error"] = "no all-to-all algorithm produced a correct result"
        pw = res.get("pairwise", {})
        # BASELINE config 3 (pairwise all-to-all, 256 MiB/rank) on its own key
        sec["alltoall_pairwise"] = {"bytes_per_rank": an * 4, "ms": pw.get("ms"), "error": pw.get("error"),
                                    "algbw_GBps": round(an * 4 / (pw["ms"] / 1e3) / 1e9, 2) if pw.get("ms") else None,
                                    "busbw_GBps": _bw(an * 4, pw.get("ms"), world, ar=False)["busbw_GBps"]}
    return sec


def run_collectives(comm, args, log=lambda *a: None, groups=("ar", "bf16", "a2a")) -> dict:
    """The coll phase's device work in one call (benchmarks/graph_replay_repro.py): the
    headline, then the secondaries named in ``groups``; the 1 GiB buffers are released before
    returning.  Returns the headline fields plus ``secondary``."""
    r = run_headline(comm, args, log)
    sec = [g for g in groups if g in ("bf16", "a2a")]
    r["secondary"] = run_secondaries(comm, args, r, log, tuple(sec)) if sec else {}
    r.pop("x", None), r.pop("y", None)
    return r


def tuning_sweep(comm, args, best_1gib: str, log=lambda *a: None) -> dict:
    """N >= 2: ``DeviceGroup.tune`` over 16 KiB .. ``--tune-max-mb`` with every hand-written
    algorithm ``auto`` may pick (ring and RHD included), plus the 1 GiB winner, written to
    ``CCMPI_TUNE_FILE`` for the later phases' groups of the same size."""
    import torch

    dev = comm.dev
    if comm.Get_size() == 1 or args.tune_max_mb <= 0:
        return {}
    algos = ["ll", "oneshot", "fanout", "twoshot", "ring"] + (["rhd"] if comm.Get_size() & (comm.Get_size() - 1) == 0
                                                              else [])
    t0 = time.perf_counter()
    table = dev.tune(max_bytes=args.tune_max_mb << 20, min_bytes=16 << 10, algos=algos, iters=5, dtype=torch.float32,
                     save=None)
    key = (dev.size, (args.size_mb << 20).bit_length() - 1)
    dev.tuned[key] = best_1gib
    if dev.rank == 0 and os.environ.get("CCMPI_TUNE_FILE"):
        from collective_communication_mpi_amd.device import save_tuning

        save_tuning(os.environ["CCMPI_TUNE_FILE"], dev.tune_key, dev.tuned)
    comm.comm.Barrier()
    log(f"tuning sweep {time.perf_counter() - t0:.1f}s: {table}")
    out = {"key": dev.tune_key, "table": {f"2^{lg}": a for (_, lg), a in sorted(dev.tuned.items())},
           "seconds": round(time.perf_counter() - t0, 1)}
    # BASELINE config 2's algbw sweep: the same sizes in bf16 (measured only: the table above
    # stays the fp32 one), every algorithm's time per size in both curves
    try:
        dev.tune(max_bytes=args.tune_max_mb << 20, min_bytes=16 << 10, algos=algos, iters=5, dtype=torch.bfloat16,
                 save=None, apply=False)
    except Exception as e:  # noqa: BLE001 - the bf16 curve is secondary
        out["bf16_error"] = f"{type(e).__name__}: {e}"[:300]
    out["sweep"] = {"float32": dev.sweep_curve("float32"), "bfloat16": dev.sweep_curve("bfloat16")}
    world = comm.Get_size()
    if world >= 4 and world % 2 == 0:
        # the harness's TP pairs (mp-major grid: ranks 2k, 2k + 1, reference func_impl.py:53-62)
        # are 2-rank groups with a table key of their own: sweep them too (every pair at once,
        # up to 16 MiB -- the TP all-reduce is 2 MiB), so their auto is measured, not a default
        t1 = time.perf_counter()
        sub = comm.Split(comm.Get_rank(), comm.Get_rank() // 2)
        sdev = sub.dev
        sdev.tune(max_bytes=min(args.tune_max_mb, 16) << 20, min_bytes=16 << 10,
                  algos=["ll", "oneshot", "fanout", "twoshot", "ring", "rhd"], iters=5, dtype=torch.float32, save=None)
        if comm.Get_rank() == 0 and os.environ.get("CCMPI_TUNE_FILE"):
            from collective_communication_mpi_amd.device import save_tuning

            save_tuning(os.environ["CCMPI_TUNE_FILE"], sdev.tune_key, sdev.tuned)
        comm.comm.Barrier()
        out["tp_pairs"] = {"key": sdev.tune_key,
                           "table": {f"2^{lg}": a for (_, lg), a in sorted(sdev.tuned.items())},
                           "seconds": round(time.perf_counter() - t1, 1)}
        log(f"TP-pair tuning sweep {out['tp_pairs']['seconds']}s: {out['tp_pairs']['table']}")
    return out


# ------------------------------------------------------------------ phases
def coll_phase(args) -> dict:
    comm = _setup_phase("10")
    import torch

    rank, world = comm.Get_rank(), comm.Get_size()
    dev = comm.dev

    def log(*a):
        if rank == 0 and args.verbose:
            print("[bench coll]", *a, file=sys.stderr, flush=True)

    r = run_headline(comm, args, log)
    _fault_injection("coll")
    tuning = {}
    rec = coll_record(args, comm, r, tuning)
    if not args.no_secondary:
        # the fp32 headline is on disk before any secondary runs: a crash or hang in the
        # bf16 / all-to-all / tuning work below keeps ``value`` (marked partial)
        _write_result(args, rank, {**rec, "partial": "written after the fp32 headline, before the secondaries"})
        _fault_injection("coll_secondary")
        try:
            rec["config"].update(run_secondaries(comm, args, r, log))
        except Exception as e:  # noqa: BLE001 - secondary; the headline stands
            rec["config"]["secondary_error"] = f"{type(e).__name__}: {e}"[:300]
        _write_result(args, rank, {**rec, "partial": "written before the tuning sweep"})
        _fault_injection("coll_tuning")
        try:
            tuning.update(tuning_sweep(comm, args, r["best"], log))
        except Exception as e:  # noqa: BLE001 - the sweep is secondary; the headline stands
            tuning["error"] = f"{type(e).__name__}: {e}"[:300]
        sw = tuning.pop("sweep", None)
        if sw:
            # BASELINE config 2: algbw / busbw vs size (fp32 and bf16), the 1 GiB headline
            # and its bf16 counterpart as the last points
            b16 = rec["config"].get("bf16_1GiB", {})
            sw["float32"].append({"bytes": args.size_mb << 20, "best": r["best"], "ms": r["results"],
                                  **_bw(args.size_mb << 20, r["t_step"] * 1e3, world)})
            if b16.get("ms"):
                sw["bfloat16"].append({"bytes": args.size_mb << 20, "best": b16["algo"], "ms": b16["candidates_ms"],
                                       **_bw(args.size_mb << 20, b16["ms"], world)})
            rec["config"]["sweep"] = sw
    r.pop("x", None), r.pop("y", None)
    torch.cuda.synchronize()
    return rec


def coll_record(args, comm, r: dict, tuning: dict) -> dict:
    """The headline record of the coll phase (``tuning`` is filled in place afterwards)."""
    dev = comm.dev
    world = comm.Get_size()
    tp = args.tp or (2 if world >= 2 and world % 2 == 0 else 1)
    return {
        "metric": METRIC,
        "value": round(r["algbw"], 3),
        "unit": "GB/s",
        "n_gpus": world // dev.ranks_per_device,  # distinct GPUs (ranks sharing one GPU count once)
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(r["t_step"] * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "fp32",
        "data": "synthetic (rank-valued 1 GiB fp32 buffer; MNIST-shaped random images, random-init weights)",
        "config": {
            "model": "allreduce-1GiB-fp32 + MNIST-shaped TP transformer layer (768->256 qkv, 256->10 fc_o per token)",
            "global_batch": args.batch * max(1, world // tp),
            "seq_len": 16,
            "parallelism": f"dp{max(1, world // tp)}xtp{tp}",
            "allreduce_algo": r["best"],
            "allreduce_bytes": args.size_mb << 20,
            "busbw_GBps": round(r["busbw"], 3),
            # one xGMI link per GPU pair (fully connected, <= 7 per GPU), ~153.6 GB/s each per
            # direction: the all-reduce's bus bandwidth as a fraction of the links it can drive
            "xgmi_link_frac": (round(r["busbw"] / (min(world - 1, 7) * XGMI_LINK_GBPS), 3)
                               if world > 1 and not dev.shared_device else None),
            "candidates_ms": r["results"],
            # every candidate's outcome: {"ms", "error"} (error: exception / timeout code with
            # phase and peer, per failing rank; or why it was skipped)
            "candidates": r["outcomes"],
            "result_exact": r["final_ok"],
            "self_test": r["self_test"],
            "shared_gpu": dev.shared_device,
            "tuning": tuning,
            "placement": list(_PLACEMENT),
        },
    }


def harness_phase(args) -> dict:
    """The DP x TP transformer-layer forward (HIP graph) and train step, plus the other
    fc_o forms, in a process of its own (a crash here cannot cost the headline)."""
    comm = _setup_phase("20")
    import torch

    from collective_communication_mpi_amd import MPI
    from collective_communication_mpi_amd.models.harness import bench_forward, fc_o_forms_agree

    world, hc = comm.Get_size(), comm.comm
    tp = args.tp or (2 if world >= 2 and world % 2 == 0 else 1)
    mode = args.fc_o_mode
    _fault_injection("harness")
    # headline: the reference's layer shape -- per-token row-parallel fc_o with (B, S, out)
    # outputs (reference model/func_impl.py:94-109), so the TP all-reduce carries
    # B*S x 16 partial outputs every step
    try:
        harness = bench_forward(comm, tp=tp, batch=args.batch, steps=args.steps, warmup=args.warmup, fc_o_mode=mode)
        herr, hok = None, 1
    except Exception as e:  # noqa: BLE001 - recorded; the pooled form is measured instead
        harness, herr, hok = None, f"{type(e).__name__}: {e}"[:300], 0
    if not hc.allreduce(hok, op=MPI.MIN) and mode != "row":
        torch.cuda.synchronize()
        mode = "row"
        harness = bench_forward(comm, tp=tp, batch=args.batch, steps=args.steps, warmup=args.warmup, fc_o_mode=mode)
        harness["token_error"] = herr
    harness["tp_allreduce_bytes"] = (args.batch * 16 * 16 * 4 if mode == "token" else args.batch * 16 * 4) \
        if tp > 1 else 0
    if not args.no_secondary:
        # the other fc_o forms: pooled row-parallel (B x 16 TP all-reduce), the token
        # pipeline in 4 row blocks whose all-reduces run on a side stream under the next
        # block's attention, and the per-token kernel's other TP form (push / plain)
        other = {}
        variants = [("pooled", "row", 1, "")] if args.fc_o_mode == "token" else [("token", "token", 1, "")]
        if tp > 1:
            if args.variants == "all":
                variants.append(("token_chunks4", "token", 4, ""))
            if mode == "token" and harness.get("fc_o_tp_form") in ("plain", "push"):
                alt = "push" if harness["fc_o_tp_form"] == "plain" else "plain"
                variants.append((f"token_{alt}", "token", 1, alt))
                try:
                    # both forms sum the same partials in rank order: bitwise equal, or the
                    # push form's numbers are not trusted (and its variant is not timed)
                    other["push_equals_plain"] = fc_o_forms_agree(comm, tp, args.batch)
                except Exception as e:  # noqa: BLE001
                    other["push_equals_plain"] = {"equal": False, "error": f"{type(e).__name__}: {e}"[:200]}
        for name, vmode, chunks, form in variants:
            if form == "push" and not other.get("push_equals_plain", {}).get("equal"):
                other[f"{name}_error"] = "push form not bitwise equal to plain: not timed"
                continue
            try:
                r = bench_forward(comm, tp=tp, batch=args.batch, steps=args.steps, warmup=args.warmup,
                                  train=False, fc_o_mode=vmode, tp_chunks=chunks, tp_fc_o_form=form)
                other[f"{name}_fwd_ms"] = round(r["fwd_ms"], 4)
                other[f"{name}_hip_graph"] = r["hip_graph"]
                # how the variant was launched: eager / graph / plan / plan_pipelined_fold, the
                # fastest reported, every mode's time on record
                other[f"{name}_fwd_timed"] = r.get("fwd_timed")
                other[f"{name}_fwd_modes_ms"] = {k[len("fwd_ms_"):]: v for k, v in r.items() if k.startswith("fwd_ms_")}
            except Exception as e:  # noqa: BLE001 - a secondary number must not cost the record
                other[f"{name}_error"] = f"{type(e).__name__}: {e}"[:200]
        harness["fc_o_variants"] = other
        if harness.get("fc_o_tp_form") == "push" and not other.get("push_equals_plain", {}).get("equal"):
            # the headline ran the push form but it did not check out: re-measure it plain
            harness = {**bench_forward(comm, tp=tp, batch=args.batch, steps=args.steps, warmup=args.warmup,
                                       fc_o_mode=mode, tp_fc_o_form="plain"), "fc_o_variants": other,
                       "push_rejected": True, "tp_allreduce_bytes": harness["tp_allreduce_bytes"]}
        form = harness.get("fc_o_tp_form")
        if form in ("plain", "push"):
            alt = "push" if form == "plain" else "plain"
            t_alt = other.get(f"token_{alt}_fwd_ms")
            if t_alt and t_alt < harness["fwd_ms"]:
                # both forms compute the same layer (bitwise equal, checked above): the step time
                # is the faster one measured on this node, like the collectives' tuned choice;
                # the other stays on record as a variant (the train step ran the first form)
                other[f"token_{form}_fwd_ms"] = round(harness["fwd_ms"], 4)
                harness["fwd_ms"] = t_alt
                harness["fc_o_tp_form"] = alt
                harness["train_fc_o_tp_form"] = form
                harness[f"fwd_timed_{form}"] = harness.get("fwd_timed")
                harness["fwd_timed"] = other.get(f"token_{alt}_fwd_timed")
    harness["fwd_ms"] = round(harness["fwd_ms"], 4)
    harness["train_ms"] = round(harness.get("train_ms", float("nan")), 4)
    if "train_ms_eager" in harness:
        harness["train_ms_eager"] = round(harness["train_ms_eager"], 4)
    return harness


def dp_phase(args) -> dict:
    """BASELINE config 5: DistributedDataParallel over every rank of a Llama-3-8B-sized
    model, bucket all-reduces launched by autograd hooks during the real backward
    (parallel/llama_dp.py); the scripted wgrad-only overlap (parallel/overlap.py) as a
    secondary number."""
    comm = _setup_phase("30")
    from collective_communication_mpi_amd.parallel.llama_dp import measure_ddp_overlap

    # CTA budgets of the bucket all-reduces: a CU holding one collective CTA cannot start a
    # ring-GEMM workgroup (512-VGPR waves take whole SIMDs), so large budgets can stall the
    # backward (32 was best on the 2-rank rehearsal, profiles/r4_dp); with one rank per GPU
    # 7 links may need more CTAs in flight: 256 / 512 are swept there too
    budgets = [32, 64, 128] + ([] if comm.dev.shared_device else [256, 512])
    out = measure_ddp_overlap(comm, layers=args.dp_layers, tokens=args.dp_tokens, vocab=bool(args.dp_vocab),
                              iters=2, blocks_sweep=budgets, verbose=args.verbose)
    if args.dp_scripted:
        import torch

        from collective_communication_mpi_amd.parallel.overlap import dp_grad_overlap

        torch.cuda.empty_cache()
        try:
            out["scripted_wgrad_only"] = dp_grad_overlap(comm, layers=args.dp_layers, tokens=args.dp_tokens, iters=2,
                                                         algo="auto", verbose=args.verbose, vocab=bool(args.dp_vocab))
        except Exception as e:  # noqa: BLE001 - secondary
            out["scripted_wgrad_only"] = {"error": f"{type(e).__name__}: {e}"[:300]}
    return out


def mlp_phase(args) -> dict:
    """The Llama-3-8B MLP block (ParallelSwiGLUMLP) with TP over every rank: hand-written
    MFMA GEMMs (SwiGLU gate in the gate|up epilogue) and the TP all-reduces of the
    reference's TP layer, over xGMI when each rank has its own GPU; the row-parallel
    variants (plain, chunked overlap, fused epilogue) side by side."""
    comm = _setup_phase("20")
    from collective_communication_mpi_amd.parallel.mlp_bench import measure_tp_mlp

    from collective_communication_mpi_amd.parallel.tensor_parallel import ROW_MODES

    modes = ROW_MODES if args.variants == "all" else tuple(m for m in ROW_MODES if m != "fused")
    return measure_tp_mlp(comm, tokens=args.mlp_tokens, iters=10, warmup=3, variants=True, modes=modes)


def rccl_phase(args) -> dict:
    """The RCCL library collectives on fresh ranks (BASELINE's 'library' comparison).
    Exact-result check before timing, like the hand-written phase."""
    comm = _setup_phase("10")
    import torch

    from collective_communication_mpi_amd import MPI

    rank, world = comm.Get_rank(), comm.Get_size()
    dev, hc = comm.dev, comm.comm
    mode = os.environ.get("CCMPI_BENCH_RCCL", "")  # tests: "force" RCCL on shared GPUs, simulate a "hang"
    if dev.shared_device and mode not in ("force", "hang"):
        return {"skipped": f"{dev.ranks_per_device} ranks share one GPU (RCCL refuses duplicate devices)"}
    if mode == "hang":
        while True:  # the supervisor's --rccl-timeout must end this phase
            time.sleep(1)
    _, timed = _timers(comm)
    t0 = time.perf_counter()
    dev.ensure_rccl()
    res = {"init_s": round(time.perf_counter() - t0, 2)}
    nbytes = args.size_mb << 20
    x = dev.empty(nbytes // 4, torch.float32)
    y = dev.empty(nbytes // 4, torch.float32)
    expect = float(world * (world + 1) // 2)
    for name, xs, ys in (("fp32", x, y), ("bf16", x.view(torch.bfloat16), y.view(torch.bfloat16))):
        xs.fill_(float(rank + 1))
        ys.zero_()
        dev.allreduce(xs, ys, "SUM", "rccl")
        torch.cuda.synchronize()
        ok = hc.allreduce(int(bool(torch.all(ys == expect).item())), op=MPI.MIN)
        for _ in range(args.warmup):
            dev.allreduce(xs, ys, "SUM", "rccl")
        t = timed(lambda: dev.allreduce(xs, ys, "SUM", "rccl"), args.steps)
        key = "" if name == "fp32" else "bf16_"
        res[f"{key}allreduce_ms"] = round(t * 1e3, 4)
        res[f"{key}algbw_GBps"] = round(nbytes / t / 1e9, 3)
        res[f"{key}busbw_GBps"] = round(nbytes / t / 1e9 * 2 * (world - 1) / world, 3)
        res[f"{key}exact"] = bool(ok)
    an = ((args.a2a_mb << 20) // 4) // world * world
    blk = an // world
    xa, ya = x[:an], y[:an]
    xa.view(world, blk).copy_((rank * world + torch.arange(world, device=dev.device, dtype=torch.float32))
                              .view(world, 1).expand(world, blk))
    want = (torch.arange(world, device=dev.device, dtype=torch.float32) * world + rank).view(world, 1).expand(world, blk)
    res["alltoall_ms"] = {}
    for algo in ("rccl", "pairwise_rccl"):
        ya.zero_()
        dev.alltoall(xa, ya, algo)
        torch.cuda.synchronize()
        ok = hc.allreduce(int(torch.equal(ya.view(world, blk), want)), op=MPI.MIN)
        res["alltoall_ms"][algo] = round(timed(lambda: dev.alltoall(xa, ya, algo), 5) * 1e3, 4) if ok else None
    return res


def host_phase(args) -> dict:
    """BASELINE config 1: "myAllreduce 8-proc CPU on a 1k-float32 buffer" -- the reference's
    own benchmark (mpi-test.py:40-98 myallreduce, :178-239 myalltoall) on the C++ host plane:
    ``--host-runs`` runs, each bracketed by Barrier + Wtime (the reference's timing), the
    library collective against the hand-written one on the same input, every run checked
    with ``np.array_equal`` (MIN is exact in any order).  Also the median of back-to-back
    calls (no barrier inside), the per-call cost without the barrier's.  CPU only."""
    import statistics

    import numpy as np

    from collective_communication_mpi_amd import MPI, Communicator

    world = MPI.COMM_WORLD
    comm = Communicator(world)
    rank, p = comm.Get_rank(), comm.Get_size()
    n = args.host_count
    runs = args.host_runs
    rng = np.random.default_rng(1234 + rank)
    out = {"ranks": p, "count": n, "dtype": "float32", "runs": runs, "op": "MIN",
           "timing": "per run: Barrier, Wtime, call, Barrier, Wtime (reference mpi-test.py:59-72); avg over runs; "
                     "*_cold_avg_us: the first runs from process start, *_avg_us: after --host-warmup runs",
           "warmup_runs": args.host_warmup,
           # the launcher's CPU binding (default: one shared set of the fewest L3 domains)
           "binding": os.environ.get("CCMPI_BIND_EFFECTIVE", os.environ.get("CCMPI_BIND", "l3")), "bound_cpus": os.environ.get("CCMPI_BOUND_CPUS")}

    def ref_loop(lib, my, make, nruns):
        """The reference's loop: per run fresh arrays, Barrier / Wtime / call / Barrier / Wtime."""
        t_lib, t_my, ok = [], [], True
        for _ in range(nruns):
            src, d_lib, d_my = make()
            comm.Barrier()
            t0 = MPI.Wtime()
            lib(src, d_lib)
            comm.Barrier()
            t_lib.append(MPI.Wtime() - t0)
            comm.Barrier()
            t0 = MPI.Wtime()
            my(src, d_my)
            comm.Barrier()
            t_my.append(MPI.Wtime() - t0)
            ok &= bool(np.array_equal(d_lib, d_my))
        return t_lib, t_my, ok

    def bench_pair(name_lib, lib, name_my, my, make):
        # first pass from a cold start, exactly the reference's 100 runs (no warm-up); then
        # --host-warmup untimed runs and the same loop again.  The cold pass pays the cores'
        # clock ramp and cold rings: every call ~2-5x slower for the first few hundred runs,
        # whatever the arrays (profiles/r6_host: the "fresh-array penalty" of round 5 was this
        # warm-up -- fresh and reused arrays time the same once warm)
        c_lib, c_my, ok0 = ref_loop(lib, my, make, runs)
        ref_loop(lib, my, make, args.host_warmup)
        t_lib, t_my, ok = ref_loop(lib, my, make, runs)
        ok = bool(world.allreduce(int(ok and ok0), op=MPI.MIN))
        src, d_lib, d_my = make()
        b2b = {}
        for nm, fn, d in ((name_lib, lib, d_lib), (name_my, my, d_my)):
            reps = []
            for _ in range(5):
                comm.Barrier()
                t0 = time.perf_counter()
                for _ in range(200):
                    fn(src, d)
                reps.append((time.perf_counter() - t0) / 200)
            b2b[nm] = round(max(world.allgather(statistics.median(reps))) * 1e6, 3)
        def avg(ts):
            return round(max(world.allgather(statistics.mean(ts))) * 1e6, 3)

        return {f"{name_lib}_avg_us": avg(t_lib), f"{name_my}_avg_us": avg(t_my),
                f"{name_lib}_cold_avg_us": avg(c_lib), f"{name_my}_cold_avg_us": avg(c_my),
                "back_to_back_median_us": b2b, "all_runs_equal": ok}

    def make_ar():
        return (rng.standard_normal(n).astype(np.float32), np.empty(n, np.float32), np.empty(n, np.float32))

    out["allreduce"] = bench_pair("Allreduce", lambda s, d: comm.Allreduce(s, d, op=MPI.MIN),
                                  "myAllreduce", lambda s, d: comm.myAllreduce(s, d, op=MPI.MIN), make_ar)
    na = n // p * p

    def make_a2a():
        return (rng.standard_normal(na).astype(np.float32), np.empty(na, np.float32), np.empty(na, np.float32))

    out["alltoall"] = bench_pair("Alltoall", comm.Alltoall, "myAlltoall", comm.myAlltoall, make_a2a)
    reps = []
    s, d, _ = make_a2a()
    for _ in range(5):
        comm.Barrier()
        t0 = time.perf_counter()
        for _ in range(200):
            comm.myAlltoall2(s, d)
        reps.append((time.perf_counter() - t0) / 200)
    out["alltoall"]["myAlltoall2_back_to_back_median_us"] = round(max(world.allgather(statistics.median(reps))) * 1e6, 3)
    return out


def _write_result(args, rank: int, out: dict) -> None:
    if rank != 0:
        return
    if args.result:
        tmp = args.result + ".tmp"
        with open(tmp, "w") as f:
            json.dump(out, f)
        os.replace(tmp, args.result)
    else:
        print(json.dumps(out), flush=True)


def main() -> int:
    args = parse()
    launched = any(k in os.environ for k in ("RANK", "CCMPI_RANK", "PMI_RANK", "OMPI_COMM_WORLD_RANK"))
    if args.gpus > 1 and not launched:
        return relaunch(args.gpus)
    if not args.phase:
        return supervise(args)  # this process never touches the GPU
    rank = _env_rank()[0]
    fn = {"coll": coll_phase, "harness": harness_phase, "rccl": rccl_phase, "dp": dp_phase, "mlp": mlp_phase,
          "host": host_phase}[args.phase]
    if args.phase == "coll":
        out = fn(args)  # the headline: a failure here fails the phase (rc != 0)
    else:
        try:
            out = fn(args)
        except Exception as e:  # noqa: BLE001 - recorded in the merged line
            out = {"error": f"{type(e).__name__}: {e}"[:400]}
    if _PLACEMENT and isinstance(out, dict) and args.phase != "coll":
        out["placement"] = list(_PLACEMENT)
    _write_result(args, rank, out)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
