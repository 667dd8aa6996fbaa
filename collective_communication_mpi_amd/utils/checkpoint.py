"""Sharded checkpoint / resume for DP x TP training state.

The reference has no model state; the harness here does: per TP shard the flat
fp32 master weights, AdamW moments and the optimizer step.  Layout of a
checkpoint directory::

    manifest.json            step, tp, dp, parameter specs, user metadata
    tp{t}.safetensors        {"p32", "m", "v"} of TP shard t (written by dp_idx 0)

* DP replicas hold identical state after every synchronised step, so only the
  ``dp_idx == 0`` rank of each TP group writes; every rank reads its TP shard.
* Tensors go through safetensors (no pickle: loading executes nothing from the
  file).  Each file is written to a temporary name and renamed, and the
  manifest is written last by rank 0 after a barrier, so a directory with a
  manifest is always complete.
* Loading checks the parameter specs and the TP degree (a TP-``t`` shard is
  only meaningful for the same TP layout); the DP degree may change.
"""
from __future__ import annotations

import json
import os
from typing import Any, Dict, Optional

import torch

FORMAT = "ccmpi-flat-v1"


def _hc(comm):
    return comm.comm if hasattr(comm, "comm") else comm


def save_sharded(path: str, flat, comm, tp_idx: int, dp_idx: int, tp: int, dp: int,
                 meta: Optional[Dict[str, Any]] = None) -> None:
    """Collective over ``comm`` (the world communicator of the job)."""
    from safetensors.torch import save_file

    hc = _hc(comm)
    os.makedirs(path, exist_ok=True)
    if hc.Get_rank() == 0:
        man = os.path.join(path, "manifest.json")
        if os.path.exists(man):  # invalidate before shards change underneath it
            os.remove(man)
    hc.Barrier()
    if dp_idx == 0:
        tensors = {k: getattr(flat, k).detach().to("cpu").contiguous() for k in ("p32", "m", "v")}
        fn = os.path.join(path, f"tp{tp_idx}.safetensors")
        tmp = fn + f".tmp{os.getpid()}"
        save_file(tensors, tmp, metadata={"format": FORMAT, "step": str(flat.step_count)})
        os.replace(tmp, fn)
    hc.Barrier()
    if hc.Get_rank() == 0:
        man = {"format": FORMAT, "step": int(flat.step_count), "tp": tp, "dp": dp, "numel": int(flat.numel),
               "specs": [[n, list(s)] for n, s in flat.specs], "meta": meta or {}}
        tmp = os.path.join(path, f"manifest.json.tmp{os.getpid()}")
        with open(tmp, "w") as f:
            json.dump(man, f, indent=1)
        os.replace(tmp, os.path.join(path, "manifest.json"))
    hc.Barrier()


def load_sharded(path: str, flat, comm, tp_idx: int, tp: int) -> Dict[str, Any]:
    """Collective: restore ``flat`` (p32, m, v, step, bf16 copy); returns the manifest."""
    from safetensors.torch import load_file

    hc = _hc(comm)
    with open(os.path.join(path, "manifest.json")) as f:
        man = json.load(f)
    if man.get("format") != FORMAT:
        raise ValueError(f"{path}: unknown checkpoint format {man.get('format')!r}")
    if man["tp"] != tp:
        raise ValueError(f"{path}: checkpoint has tp={man['tp']}, job has tp={tp}")
    specs = [[n, list(s)] for n, s in flat.specs]
    if man["specs"] != specs or man["numel"] != flat.numel:
        raise ValueError(f"{path}: parameter layout differs from the model's")
    tensors = load_file(os.path.join(path, f"tp{tp_idx}.safetensors"))
    for k in ("p32", "m", "v"):
        getattr(flat, k).copy_(tensors[k].to(getattr(flat, k).device))
    flat.step_count = int(man["step"])
    if flat.p32.is_cuda:
        flat.refresh_bf16()
    else:
        flat.p16.copy_(flat.p32.to(flat.p16.dtype))
    hc.Barrier()
    return man


def latest(path: str) -> Optional[str]:
    """``path`` itself if it holds a complete checkpoint, else None."""
    return path if os.path.exists(os.path.join(path, "manifest.json")) else None
