"""Check topology.py's sysfs prediction against the GPU the runtime opens.

    python benchmarks/placement_probe.py [--ranks 8]

Before any GPU call: the visible GPUs read from the KFD topology (PCI address, NUMA node,
local CPUs) and ``gpu_plan`` for ``--ranks`` local ranks.  Then torch initialises the GPU and
the probe prints every device's PCI address and UUID as the runtime reports them, whether
ordinal i is the device the prediction put at index i, and ``check_bound`` for device 0.
One JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from collective_communication_mpi_amd import topology as T  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", type=int, default=8)
    a = ap.parse_args()
    devs = T.gpu_devices()
    plan = T.gpu_plan(a.ranks)
    out = {"sysfs_gpus": [{k: d[k] for k in ("node", "bdf", "numa", "uuid", "render_minor")}
                          | {"cpus": T.format_cpu_list(d["cpus"])} for d in devs],
           "plan": [T.format_cpu_list(p) for p in plan] if plan else None,
           "affinity": T.format_cpu_list(os.sched_getaffinity(0)),
           "visible_env": {k: os.environ.get(k) for k in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES",
                                                          "CUDA_VISIBLE_DEVICES") if os.environ.get(k) is not None}}
    import torch

    from collective_communication_mpi_amd.device import device_identity

    rt = []
    for i in range(torch.cuda.device_count()):
        p = torch.cuda.get_device_properties(i)
        bdf = f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}.0"
        rt.append({"ordinal": i, "bdf": bdf, "uuid": str(p.uuid), "identity": device_identity(p),
                   "matches_sysfs": i < len(devs) and devs[i]["bdf"] == bdf})
    out["runtime_gpus"] = rt
    out["order_ok"] = bool(rt) and all(r["matches_sysfs"] for r in rt)
    out["check_bound_dev0"] = T.check_bound(torch.cuda.get_device_properties(0))
    print(json.dumps(out))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
