"""Host placement of GPU ranks, read from sysfs BEFORE any GPU call.

The reference runs every rank on "one multi-core host" (reference README.md:9,41) and
leaves placement to MPI.  On an MI355X node the host is 2 sockets x 8 CCDs (one L3 each)
and each GPU hangs off one socket's IO die: a rank that drives GPU g from a core of the
other socket pays an IO-die crossing on every doorbell, every kernel-argument copy and
every host-plane cache line.  This module maps rank -> the CPUs local to *its* GPU:

* ``gpu_devices``: the visible GPUs in HIP ordinal order from the KFD topology
  (``/sys/class/kfd/kfd/topology/nodes/*/properties``: GPU nodes have ``simd_count > 0``;
  ``domain`` + ``location_id`` give the PCI address), each with the CPUs of its PCI
  device (``/sys/bus/pci/devices/<bdf>/local_cpulist``, else its NUMA node's cpulist),
  filtered by ``ROCR_VISIBLE_DEVICES`` then ``HIP_VISIBLE_DEVICES`` / ``CUDA_VISIBLE_DEVICES``
  (indices or ``GPU-<uuid>``), and by the render nodes that exist under ``/dev/dri`` (a
  container sees only its own);
* ``gpu_plan``: local rank r drives visible GPU ``r % ngpu`` (``device.py``'s default);
  within that GPU's CPUs the ranks get DISTINCT L3 domains (CCDs), the least busy first,
  so every rank -- its HIP runtime threads, its host-plane spin-waits -- owns a core set
  on the right socket.  More ranks than domains: domains are shared round-robin.
* ``check_bound``: after the GPU is initialised, the phase child compares its binding with
  the PCI address the runtime reports and re-binds every thread of the process if the
  sysfs prediction named the wrong GPU (recorded, never silent).

The CPU host phase (BASELINE config 1) keeps the launcher's ``l3`` policy: there every
message is a shared-memory cache line between the ranks, so one CCD wins
(``profiles/r5_host/README.md``).
"""
from __future__ import annotations

import os
from typing import Dict, Iterable, List, Mapping, Optional, Sequence

KFD_NODES = "class/kfd/kfd/topology/nodes"


# ------------------------------------------------------------------ cpu lists
def parse_cpu_list(txt: str) -> List[int]:
    """'0-3,8,10-11' -> [0, 1, 2, 3, 8, 10, 11]."""
    out: List[int] = []
    for part in txt.strip().split(","):
        part = part.strip()
        if not part:
            continue
        if "-" in part:
            a, b = part.split("-", 1)
            out.extend(range(int(a), int(b) + 1))
        else:
            out.append(int(part))
    return out


def format_cpu_list(cpus: Iterable[int]) -> str:
    """[0, 1, 2, 3, 8] -> '0-3,8' (the kernel's own cpulist form)."""
    cs = sorted(set(cpus))
    runs, i = [], 0
    while i < len(cs):
        j = i
        while j + 1 < len(cs) and cs[j + 1] == cs[j] + 1:
            j += 1
        runs.append(str(cs[i]) if i == j else f"{cs[i]}-{cs[j]}")
        i = j + 1
    return ",".join(runs)


def _read(path: str) -> Optional[str]:
    try:
        with open(path) as f:
            return f.read()
    except OSError:
        return None


# ------------------------------------------------------------------ GPUs
def _kfd_props(txt: str) -> Dict[str, int]:
    out = {}
    for line in txt.splitlines():
        parts = line.split()
        if len(parts) == 2:
            try:
                out[parts[0]] = int(parts[1])
            except ValueError:
                pass
    return out


def _visible(devs: List[dict], spec: Optional[str]) -> List[dict]:
    """Apply one visibility variable (comma list of indices or GPU-<uuid> tokens)."""
    if spec is None:
        return devs
    spec = spec.strip()
    if spec == "":
        return []
    out = []
    for tok in spec.split(","):
        tok = tok.strip()
        if tok.isdigit():
            i = int(tok)
            if i < len(devs):
                out.append(devs[i])
        elif tok:
            want = tok.lower().replace("gpu-", "")
            out.extend(d for d in devs if d["uuid"] and d["uuid"].lower().replace("gpu-", "") == want)
    return out


def gpu_devices(root: str = "/sys", env: Optional[Mapping[str, str]] = None,
                dev_root: str = "/dev") -> List[dict]:
    """Visible GPUs in HIP ordinal order (see module doc); [] when the topology is unreadable."""
    env = os.environ if env is None else env
    base = os.path.join(root, KFD_NODES)
    try:
        nodes = sorted(int(n) for n in os.listdir(base) if n.isdigit())
    except OSError:
        return []
    devs = []
    for n in nodes:
        txt = _read(os.path.join(base, str(n), "properties"))
        if txt is None:
            continue
        p = _kfd_props(txt)
        if p.get("simd_count", 0) <= 0:
            continue  # a CPU node
        loc, dom = p.get("location_id", 0), p.get("domain", 0)
        bdf = f"{dom:04x}:{(loc >> 8) & 0xff:02x}:{(loc >> 3) & 0x1f:02x}.{loc & 0x7}"
        pci = os.path.join(root, "bus/pci/devices", bdf)
        numa_txt = _read(os.path.join(pci, "numa_node"))
        numa = int(numa_txt.strip()) if numa_txt and numa_txt.strip().lstrip("-").isdigit() else -1
        cl = _read(os.path.join(pci, "local_cpulist"))
        if cl is None and numa >= 0:
            cl = _read(os.path.join(root, f"devices/system/node/node{numa}/cpulist"))
        uid = p.get("unique_id", 0)
        devs.append({"node": n, "bdf": bdf, "domain": dom, "bus": (loc >> 8) & 0xff, "numa": numa,
                     "cpus": parse_cpu_list(cl) if cl else [], "uuid": f"GPU-{uid:016x}" if uid else "",
                     "render_minor": p.get("drm_render_minor", -1)})
    # a container sees only its own render nodes: drop GPUs whose node is absent (when
    # /dev/dri exists at all and names at least one of them)
    dri = os.path.join(dev_root, "dri")
    if os.path.isdir(dri):
        have = [d for d in devs if d["render_minor"] >= 0 and os.path.exists(os.path.join(dri, f"renderD{d['render_minor']}"))]
        if have:
            devs = have
    devs = _visible(devs, env.get("ROCR_VISIBLE_DEVICES"))
    hip = env.get("HIP_VISIBLE_DEVICES", env.get("CUDA_VISIBLE_DEVICES"))
    return _visible(devs, hip)


# ------------------------------------------------------------------ L3 domains
def l3_domains(cpus: Sequence[int], root: str = "/sys") -> Dict[tuple, List[int]]:
    """L3 key -> the given CPUs in that domain (one key per CPU when unreadable)."""
    out: Dict[tuple, List[int]] = {}
    for c in sorted(cpus):
        txt = _read(os.path.join(root, f"devices/system/cpu/cpu{c}/cache/index3/shared_cpu_list"))
        key = tuple(parse_cpu_list(txt)) if txt else (c,)
        out.setdefault(key, []).append(c)
    return out


def gpu_plan(n_ranks: int, root: str = "/sys", env: Optional[Mapping[str, str]] = None,
             allowed: Optional[Iterable[int]] = None, busy: Optional[Mapping[int, float]] = None,
             dev_root: str = "/dev") -> Optional[List[List[int]]]:
    """Per local rank, the CPU set it is bound to (see module doc); None when no GPU is
    visible in sysfs.  ``busy``: per-CPU busy fraction (least busy domain first)."""
    gpus = gpu_devices(root, env, dev_root)
    if not gpus or n_ranks <= 0:
        return None
    allowed = set(os.sched_getaffinity(0) if allowed is None else allowed)
    busy = busy or {}
    # ranks by the CPU set local to their GPU (ranks of GPUs on one NUMA node share a pool)
    pools: Dict[frozenset, List[int]] = {}
    for r in range(n_ranks):
        g = gpus[r % len(gpus)]
        local = frozenset(c for c in g["cpus"] if c in allowed) or frozenset(allowed)
        pools.setdefault(local, []).append(r)
    plan: List[Optional[List[int]]] = [None] * n_ranks
    for local, ranks in pools.items():
        doms = l3_domains(sorted(local), root)
        order = sorted(doms, key=lambda k: (round(sum(busy.get(c, 0.0) for c in doms[k]), 1), min(doms[k])))
        for i, r in enumerate(ranks):
            plan[r] = sorted(doms[order[i % len(order)]])
    return plan  # type: ignore[return-value]


# ------------------------------------------------------------------ after GPU init
def pci_cpus(domain: int, bus: int, device: int = 0, root: str = "/sys") -> List[int]:
    """CPUs local to a PCI device given its address ([] when unreadable).  ``device`` is the
    slot (HIP's ``pciDeviceID``); the function number is 0 for a GPU's display function."""
    bdf = f"{domain:04x}:{bus:02x}:{device:02x}.0"
    txt = _read(os.path.join(root, "bus/pci/devices", bdf, "local_cpulist"))
    return parse_cpu_list(txt) if txt else []


def set_process_affinity(cpus: Iterable[int]) -> int:
    """Bind every thread of this process (runtime helper threads included); returns how
    many threads were moved."""
    cs = set(cpus)
    moved = 0
    try:
        tids = [int(t) for t in os.listdir("/proc/self/task")]
    except OSError:
        tids = [0]
    for t in tids:
        try:
            os.sched_setaffinity(t, cs)
            moved += 1
        except OSError:
            pass
    return moved


def check_bound(props, root: str = "/sys") -> dict:
    """Compare this process's CPU binding with the CPUs local to the GPU the runtime
    opened (``props``: torch device properties).  A binding that has no CPU on the GPU's
    side is re-bound to those CPUs (every thread).  Returns a record for the bench."""
    have = sorted(os.sched_getaffinity(0))
    want = pci_cpus(getattr(props, "pci_domain_id", 0), getattr(props, "pci_bus_id", 0),
                    getattr(props, "pci_device_id", 0), root)
    rec = {"bound_cpus": format_cpu_list(have)}
    if not want:
        rec["gpu_local_cpus"] = None
        return rec
    rec["gpu_local_cpus"] = format_cpu_list(want)
    if set(have) & set(want):
        rec["gpu_local"] = True
        return rec
    if os.environ.get("CCMPI_BOUND_CPUS"):
        # the prediction named another GPU's socket: move to the right one, say so
        rec["rebound_threads"] = set_process_affinity(want)
        rec["bound_cpus"] = format_cpu_list(sorted(os.sched_getaffinity(0)))
    rec["gpu_local"] = False
    return rec
