"""``mpirun``-compatible single-node launcher.

    python -m collective_communication_mpi_amd.launch -n 8 python mpi-test.py --test_case myallreduce
    scripts/mpirun -n 4 python3 -m pytest tests/test_transformer_forward.py --with-mpi

The reference is launched with ``mpirun -n {4,8} python ...`` (reference
README.md:52-136,189).  This launcher starts N ranks of the command on this
host with ``CCMPI_RANK/CCMPI_SIZE/CCMPI_LOCAL_RANK/CCMPI_JOBID`` set (plus
``LOCAL_RANK`` so GPU ranks pick a device), prefixes nothing, propagates the
first failing exit code and tears down the remaining ranks (no orphaned
spinners), and enforces an optional wall-clock ``--timeout``.

Open MPI style flags that make no sense for a single-host shm runtime
(``--oversubscribe``, ``--allow-run-as-root``, ``-H host``) are accepted and ignored;
``-x VAR[=VAL]`` exports a variable.  Binding (``--bind-to`` / ``CCMPI_BIND``):

* ``l3`` (default): every rank may run on any hardware thread of the fewest L3 domains
  (CCDs) that hold one physical core per rank, the least busy domain first (a 20 ms
  ``/proc/stat`` sample; ties: the launcher's own domain).  The host
  plane's messages are shared-memory cache lines moving between the ranks' cores: on the
  MI355X box's 2 x 64-core EPYC the OS spread 8 ranks over 8 CCDs, and every line crossed
  the IO die (8-rank library Allreduce of 4 KiB 8.1 us unbound, 3.3-3.9 us in one CCD; the
  reference's myAllreduce loop 26.3 -> 14.8-17.3 us; ``profiles/r5_host/``).  A set rather
  than one CPU per rank: a GPU rank's runtime threads (HIP, RCCL proxy) float within it;
* ``gpu``: rank r on the CPUs local to the GPU it drives (local rank r -> visible GPU
  r % ngpu), its own L3 domain within them, least busy first (``topology.gpu_plan``: KFD
  topology + PCI ``local_cpulist`` read from sysfs before any GPU call).  ``bench.py`` uses
  it for every GPU job; with no GPU in sysfs it falls back to ``l3``;
* ``l3core``: rank r on one hardware thread of the r-th physical core of those domains;
* ``core``: rank r on the r-th CPU the launcher may use;
* ``none`` (or any other level): placement left to the OS.
No binding either when there are more ranks than allowed physical cores.
"""
from __future__ import annotations

import os
import signal
import subprocess
import sys
import time
import uuid
from pathlib import Path
from typing import List, Optional

from collective_communication_mpi_amd.topology import format_cpu_list, gpu_plan

REPO = Path(__file__).resolve().parent.parent

_FLAG_WITH_ARG_IGNORED = {"--map-by", "-H", "--host", "--hostfile", "-hostfile", "--mca", "-ppn"}
_FLAG_IGNORED = {"--oversubscribe", "--allow-run-as-root", "-l", "--tag-output", "-prepend-rank"}


def parse(argv: List[str]):
    n = 1
    timeout: Optional[float] = None
    exports = {}
    i = 0
    while i < len(argv):
        a = argv[i]
        if a in ("-n", "-np", "--np", "-c"):
            n = int(argv[i + 1]); i += 2
        elif a.startswith("-n") and a[2:].isdigit():
            n = int(a[2:]); i += 1
        elif a == "--timeout":
            timeout = float(argv[i + 1]); i += 2
        elif a == "-x":
            kv = argv[i + 1]
            if "=" in kv:
                k, v = kv.split("=", 1)
            else:
                k, v = kv, os.environ.get(kv, "")
            exports[k] = v
            i += 2
        elif a == "--bind-to":
            # Open MPI semantics for "core": rank r pinned to the r-th CPU this launcher may
            # use (fewer migrations, shorter tails for the host plane's spin-waits); any other
            # level ("none", "socket", ...) leaves placement to the OS
            exports["CCMPI_BIND"] = argv[i + 1]
            i += 2
        elif a in _FLAG_WITH_ARG_IGNORED:
            i += 2
        elif a in _FLAG_IGNORED:
            i += 1
        elif a == "--mca":
            i += 3
        elif a == "--":
            i += 1
            break
        else:
            break
    cmd = argv[i:]
    if not cmd:
        raise SystemExit("usage: launch -n N [--timeout S] [-x VAR=VAL] command [args...]")
    return n, timeout, exports, cmd


def _current_cpu() -> Optional[int]:
    try:
        with open("/proc/self/stat") as f:
            return int(f.read().rsplit(")", 1)[1].split()[36])  # field 39: processor
    except (OSError, ValueError, IndexError):
        return None


def _read_cpu_list(path: str) -> List[int]:
    with open(path) as f:
        txt = f.read().strip()
    out = []
    for part in txt.split(","):
        if "-" in part:
            a, b = part.split("-")
            out.extend(range(int(a), int(b) + 1))
        elif part:
            out.append(int(part))
    return out


def _cpu_busy(window_s: float = 0.02) -> dict:
    """Per-CPU busy fraction over a short window (/proc/stat), {} if unreadable."""
    def snap():
        out = {}
        with open("/proc/stat") as f:
            for line in f:
                if line.startswith("cpu") and line[3:4].isdigit():
                    parts = line.split()
                    vals = [int(v) for v in parts[1:]]
                    idle = vals[3] + (vals[4] if len(vals) > 4 else 0)
                    out[int(parts[0][3:])] = (sum(vals), idle)
        return out
    try:
        a = snap()
        time.sleep(window_s)
        b = snap()
    except (OSError, ValueError):
        return {}
    busy = {}
    for c, (tot, idle) in b.items():
        if c in a:
            dt, di = tot - a[c][0], idle - a[c][1]
            busy[c] = (dt - di) / dt if dt > 0 else 0.0
    return busy


def _l3_domains():
    """(domains in placement order, allowed CPUs by domain): L3 key -> one allowed hardware
    thread per physical core; the least busy domain first (a short /proc/stat sample: on a
    shared host another job's ranks may be spinning in the launcher's own domain), ties broken
    by the launcher's own domain, then CPU order."""
    allowed = set(os.sched_getaffinity(0))
    sysfs = "/sys/devices/system/cpu"
    cores, threads = {}, {}
    seen_core = set()
    dom_of = {}
    for c in sorted(allowed):
        sib = tuple(_read_cpu_list(f"{sysfs}/cpu{c}/topology/thread_siblings_list"))
        key = tuple(_read_cpu_list(f"{sysfs}/cpu{c}/cache/index3/shared_cpu_list"))
        dom_of[c] = key
        threads.setdefault(key, []).append(c)
        if sib in seen_core:
            continue
        seen_core.add(sib)
        cores.setdefault(key, []).append(c)
    first = dom_of.get(_current_cpu())
    busy = _cpu_busy()
    load = {k: round(sum(busy.get(c, 0.0) for c in threads[k]), 1) for k in cores}
    order = sorted(cores, key=lambda k: (load[k], k != first, min(k)))
    return order, cores, threads


def l3_plan(n: int) -> Optional[List[int]]:
    """CPUs for n ranks: one allowed hardware thread per physical core, the launcher's own L3
    domain first, then the other domains in CPU order; None if that gives fewer than n CPUs
    or the topology is unreadable."""
    try:
        order, cores, _ = _l3_domains()
        plan = [c for k in order for c in cores[k]]
        return plan[:n] if len(plan) >= n else None
    except (OSError, ValueError):
        return None


def l3_set(n: int) -> Optional[List[int]]:
    """One CPU set for all n ranks: every allowed hardware thread of the fewest L3 domains
    (launcher's first) that hold n physical cores; None as for ``l3_plan``."""
    try:
        order, cores, threads = _l3_domains()
        out, ncores = [], 0
        for k in order:
            out += threads[k]
            ncores += len(cores[k])
            if ncores >= n:
                return sorted(out)
        return None
    except (OSError, ValueError):
        return None


def launch(n: int, cmd: List[str], timeout: Optional[float] = None, env_extra=None,
           job_id: Optional[str] = None) -> int:
    job = job_id or uuid.uuid4().hex[:16]
    procs = []
    base = dict(os.environ)
    base.update(env_extra or {})
    pp = base.get("PYTHONPATH", "")
    base["PYTHONPATH"] = str(REPO) + (os.pathsep + pp if pp else "")
    bind = base.get("CCMPI_BIND", "l3")
    plan = None  # per rank: the CPU set it is bound to
    if bind == "gpu":
        try:
            plan = gpu_plan(n, env=base, busy=_cpu_busy())
        except (OSError, ValueError):
            plan = None
        if plan is None:
            bind = "l3"
    if bind == "l3":
        dom = l3_set(n)
        plan = [dom] * n if dom is not None else None
    elif bind == "l3core":
        cpus = l3_plan(n)
        plan = [[c] for c in cpus] if cpus is not None else None
    elif bind == "core":
        cpus = sorted(os.sched_getaffinity(0))
        plan = [[cpus[r % len(cpus)]] for r in range(n)]
    for r in range(n):
        env = dict(base)
        env.update({
            "CCMPI_RANK": str(r), "CCMPI_SIZE": str(n),
            "CCMPI_LOCAL_RANK": str(r), "CCMPI_LOCAL_SIZE": str(n),
            "CCMPI_JOBID": job, "LOCAL_RANK": str(r),
        })
        # Foreign launcher variables would make the runtime pick the wrong rank.
        for k in ("PMI_RANK", "PMI_SIZE", "OMPI_COMM_WORLD_RANK", "OMPI_COMM_WORLD_SIZE", "RANK", "WORLD_SIZE"):
            env.pop(k, None)
        pin = plan[r] if plan is not None else None
        env["CCMPI_BIND_EFFECTIVE"] = bind if pin is not None else "none"
        if pin is not None:
            env["CCMPI_BOUND_CPUS"] = format_cpu_list(pin)
        procs.append(subprocess.Popen(cmd, env=env, start_new_session=True,
                                      preexec_fn=(lambda c=pin: os.sched_setaffinity(0, set(c))) if pin is not None else None))

    def kill_all(sig=signal.SIGTERM):
        for p in procs:
            if p.poll() is None:
                try:
                    os.killpg(p.pid, sig)
                except ProcessLookupError:
                    pass

    def on_signal(signum, _frame):
        kill_all(signal.SIGTERM)

    old = {s: signal.signal(s, on_signal) for s in (signal.SIGINT, signal.SIGTERM)}
    t0 = time.monotonic()
    rc = 0
    try:
        while True:
            alive = False
            for p in procs:
                code = p.poll()
                if code is None:
                    alive = True
                elif code != 0 and rc == 0:
                    rc = code if code > 0 else 128 - code
            if rc != 0:
                break
            if not alive:
                break
            if timeout is not None and time.monotonic() - t0 > timeout:
                sys.stderr.write(f"[launch] timeout after {timeout:.0f}s; killing {n} ranks\n")
                rc = 124
                break
            time.sleep(0.01)
    finally:
        if rc != 0:
            kill_all(signal.SIGTERM)
            deadline = time.monotonic() + 5
            while time.monotonic() < deadline and any(p.poll() is None for p in procs):
                time.sleep(0.05)
            kill_all(signal.SIGKILL)
        for p in procs:
            try:
                p.wait(timeout=10)
            except subprocess.TimeoutExpired:
                pass
        for s, h in old.items():
            # a handler installed outside Python (e.g. by a profiler's preloaded library)
            # reads back as None and cannot be reinstalled from here
            if h is not None:
                signal.signal(s, h)
    return rc


def main(argv=None) -> int:
    n, timeout, exports, cmd = parse(list(sys.argv[1:] if argv is None else argv))
    return launch(n, cmd, timeout, exports)


if __name__ == "__main__":
    raise SystemExit(main())
