"""Host placement of GPU ranks (topology.py) and GPU identity (device.device_identity), CPU only.

A fake sysfs tree stands in for an 8-GPU MI355X node: 2 sockets (NUMA nodes), 8 CCDs of
8 cores (16 hardware threads) per socket, GPUs 0-3 on socket 0 and 4-7 on socket 1.
"""
import os
import types

import pytest

from collective_communication_mpi_amd import topology as T

CORES_PER_CCD, CCDS_PER_SOCKET, SOCKETS = 8, 8, 2
NCORES = CORES_PER_CCD * CCDS_PER_SOCKET * SOCKETS  # 128 physical, threads c and c + 128


def _write(path, text):
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "w") as f:
        f.write(text)


def _socket_cpus(s):
    lo = s * NCORES // SOCKETS
    hi = lo + NCORES // SOCKETS
    return list(range(lo, hi)) + list(range(lo + NCORES, hi + NCORES))


def make_node(tmp_path, gpus_per_socket=4, domains=None, render_nodes=None):
    sysfs, dev = tmp_path / "sys", tmp_path / "dev"
    for c in range(2 * NCORES):
        core = c % NCORES
        ccd = core // CORES_PER_CCD
        lo = ccd * CORES_PER_CCD
        l3 = T.format_cpu_list(list(range(lo, lo + CORES_PER_CCD)) + list(range(lo + NCORES, lo + NCORES + CORES_PER_CCD)))
        _write(f"{sysfs}/devices/system/cpu/cpu{c}/cache/index3/shared_cpu_list", l3 + "\n")
    for s in range(SOCKETS):
        _write(f"{sysfs}/devices/system/node/node{s}/cpulist", T.format_cpu_list(_socket_cpus(s)) + "\n")
    # KFD: CPU nodes 0, 1 then GPU nodes 2..9
    for s in range(SOCKETS):
        _write(f"{sysfs}/class/kfd/kfd/topology/nodes/{s}/properties", "cpu_cores_count 64\nsimd_count 0\n")
    ngpu = gpus_per_socket * SOCKETS
    for g in range(ngpu):
        bus = 0x05 + 0x20 * g
        dom = (domains or [0] * ngpu)[g]
        loc = bus << 8
        _write(f"{sysfs}/class/kfd/kfd/topology/nodes/{2 + g}/properties",
               f"cpu_cores_count 0\nsimd_count 1024\nlocation_id {loc}\ndomain {dom}\n"
               f"drm_render_minor {128 + g}\nunique_id {0x1000 + g}\n")
        bdf = f"{dom:04x}:{bus:02x}:00.0"
        sock = g // gpus_per_socket
        _write(f"{sysfs}/bus/pci/devices/{bdf}/numa_node", f"{sock}\n")
        _write(f"{sysfs}/bus/pci/devices/{bdf}/local_cpulist", T.format_cpu_list(_socket_cpus(sock)) + "\n")
    for g in (range(ngpu) if render_nodes is None else render_nodes):
        _write(f"{dev}/dri/renderD{128 + g}", "")
    return str(sysfs), str(dev)


def test_cpu_list_round_trip():
    assert T.parse_cpu_list("0-3,8,10-11\n") == [0, 1, 2, 3, 8, 10, 11]
    assert T.format_cpu_list([11, 0, 1, 2, 3, 8, 10]) == "0-3,8,10-11"
    assert T.format_cpu_list([]) == ""


def test_gpu_plan_binds_each_rank_to_its_gpus_socket(tmp_path):
    """8 ranks on 8 GPUs / 2 NUMA nodes: rank r's CPUs are all on GPU r's socket, and each
    rank owns a distinct L3 domain (16 threads of one CCD)."""
    sysfs, dev = make_node(tmp_path)
    allowed = range(2 * NCORES)
    gpus = T.gpu_devices(sysfs, env={}, dev_root=dev)
    assert [g["numa"] for g in gpus] == [0, 0, 0, 0, 1, 1, 1, 1]
    plan = T.gpu_plan(8, root=sysfs, env={}, allowed=allowed, dev_root=dev)
    assert plan is not None and len(plan) == 8
    for r, cpus in enumerate(plan):
        sock = set(_socket_cpus(r // 4))
        assert set(cpus) <= sock, (r, cpus)
        assert len(cpus) == 2 * CORES_PER_CCD
    assert len({tuple(c) for c in plan}) == 8  # distinct core sets
    # the least busy CCD goes first: make socket 0's first CCD busy
    busy = {c: 1.0 for c in range(CORES_PER_CCD)}
    plan2 = T.gpu_plan(4, root=sysfs, env={}, allowed=allowed, busy=busy, dev_root=dev)
    assert all(not (set(p) & set(busy)) for p in plan2)


def test_gpu_plan_visibility_and_sharing(tmp_path):
    sysfs, dev = make_node(tmp_path)
    allowed = range(2 * NCORES)
    # per-rank isolation to GPU 5 (socket 1): every rank uses it
    plan = T.gpu_plan(2, root=sysfs, env={"ROCR_VISIBLE_DEVICES": "5"}, allowed=allowed, dev_root=dev)
    assert all(set(p) <= set(_socket_cpus(1)) for p in plan)
    # HIP_VISIBLE_DEVICES indexes the ROCr-visible list; UUID tokens work too
    g = T.gpu_devices(sysfs, env={"ROCR_VISIBLE_DEVICES": "1,6", "HIP_VISIBLE_DEVICES": "1"}, dev_root=dev)
    assert [d["numa"] for d in g] == [1]
    g = T.gpu_devices(sysfs, env={"CUDA_VISIBLE_DEVICES": f"GPU-{0x1000 + 2:016x}"}, dev_root=dev)
    assert len(g) == 1 and g[0]["numa"] == 0
    # 8 ranks sharing one GPU (the 1-GPU dry run): 8 distinct CCDs of that GPU's socket
    plan = T.gpu_plan(8, root=sysfs, env={"ROCR_VISIBLE_DEVICES": "0"}, allowed=allowed, dev_root=dev)
    assert len({tuple(p) for p in plan}) == 8 and all(set(p) <= set(_socket_cpus(0)) for p in plan)
    # a container that sees only render node 129 (GPU 1) and 134 (GPU 6)
    sysfs2, dev2 = make_node(tmp_path / "c", render_nodes=[1, 6])
    g = T.gpu_devices(sysfs2, env={}, dev_root=dev2)
    assert [d["numa"] for d in g] == [0, 1]


def test_gpu_plan_respects_allowed_cpus_and_missing_topology(tmp_path):
    sysfs, dev = make_node(tmp_path)
    # a cpuset holding only socket 1's first two CCDs: ranks of socket-0 GPUs fall back to it
    allowed = set(range(64, 80)) | set(range(192, 208))
    plan = T.gpu_plan(8, root=sysfs, env={}, allowed=allowed, dev_root=dev)
    assert all(set(p) <= allowed and p for p in plan)
    assert T.gpu_plan(4, root=str(tmp_path / "nothing"), env={}, allowed=allowed) is None


def test_device_identity_uuid_and_domain():
    """Two GPUs with the same bus number in different PCI domains, each rank seeing its
    device as ordinal 0 (per-rank isolation), are NOT one shared GPU."""
    from collective_communication_mpi_amd.device import device_identity

    def props(domain, bus, uuid="", dev=0):
        return types.SimpleNamespace(uuid=uuid, pci_domain_id=domain, pci_bus_id=bus, pci_device_id=dev,
                                     name="AMD Instinct MI355X")

    a, b = props(0, 0x05), props(1, 0x05)
    keys = [device_identity(a), device_identity(b)]
    assert keys.count(keys[0]) == 1
    # same bus and domain but different UUIDs: distinct; same everything: shared
    assert device_identity(props(0, 5, "GPU-aa")) != device_identity(props(0, 5, "GPU-bb"))
    assert device_identity(props(0, 5, "GPU-aa")) == device_identity(props(0, 5, "GPU-aa"))
    # an all-zero UUID falls back to the PCI address
    assert device_identity(props(0, 5, "00000000-0000-0000-0000-000000000000")) == device_identity(props(0, 5))


def test_check_bound_reports_and_rebinds(tmp_path, monkeypatch):
    sysfs, _ = make_node(tmp_path)
    have = sorted(os.sched_getaffinity(0))
    p = types.SimpleNamespace(pci_domain_id=0, pci_bus_id=0x05, pci_device_id=0)
    # fake GPU-local list = the CPUs we already have: gpu_local True
    _write(f"{sysfs}/bus/pci/devices/0000:05:00.0/local_cpulist", T.format_cpu_list(have))
    r = T.check_bound(p, root=sysfs)
    assert r["gpu_local"] is True and r["bound_cpus"] == T.format_cpu_list(have)
    # GPU-local CPUs outside our set, not launcher-bound: reported, not moved
    _write(f"{sysfs}/bus/pci/devices/0000:05:00.0/local_cpulist", "100000")
    monkeypatch.delenv("CCMPI_BOUND_CPUS", raising=False)
    r = T.check_bound(p, root=sysfs)
    assert r["gpu_local"] is False and "rebound_threads" not in r
    assert sorted(os.sched_getaffinity(0)) == have


@pytest.mark.parametrize("mode", ["gpu", "none"])
def test_launcher_gpu_mode_falls_back_without_gpus(mode):
    """No GPU in this container's sysfs: ``gpu`` binding falls back to ``l3`` and says so."""
    from _launch import py, run_ranks

    code = "import os; print('BIND', os.environ.get('CCMPI_BIND_EFFECTIVE'), os.environ.get('CCMPI_BOUND_CPUS'))"
    r = run_ranks(2, py("-c", code), timeout=60, env={"CCMPI_BIND": mode})
    lines = [l.split() for l in r.stdout.splitlines() if l.startswith("BIND")]
    assert len(lines) == 2
    if mode == "none":
        assert all(l[1] == "none" for l in lines)
    elif T.gpu_plan(2) is None:
        assert all(l[1] in ("l3", "none") for l in lines)
