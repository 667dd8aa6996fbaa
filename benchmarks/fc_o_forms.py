"""DP x TP harness forward with the per-token fc_o's two TP forms (plain: kernel + all-reduce
of z; push: kernel stores row blocks into the TP owners' inboxes + inbox-to-local), same
process, HIP-graph replays, max over ranks.  Rank 0 prints one JSON line.

    python -m collective_communication_mpi_amd.launch -n 2 python benchmarks/fc_o_forms.py
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

from collective_communication_mpi_amd import MPI, Communicator  # noqa: E402
from collective_communication_mpi_amd.models.harness import bench_forward, fc_o_forms_agree  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--tp", type=int, default=2)
ap.add_argument("--batch", type=int, default=2048)
ap.add_argument("--steps", type=int, default=20)
args = ap.parse_args()
comm = Communicator(MPI.COMM_WORLD)
torch.cuda.set_device(int(os.environ.get("CCMPI_LOCAL_RANK", "0")) % torch.cuda.device_count())
out = {"ranks": comm.Get_size(), "tp": args.tp, "batch_per_replica": args.batch,
       "agree": fc_o_forms_agree(comm, args.tp, 128)}
for form in ("plain", "push", "plain", "push"):
    r = bench_forward(comm, tp=args.tp, batch=args.batch, steps=args.steps, warmup=3, train=False,
                      fc_o_mode="token", tp_fc_o_form=form)
    out.setdefault(f"{form}_fwd_ms", []).append(round(r["fwd_ms"], 4))
    out[f"{form}_hip_graph"] = r["hip_graph"]
if comm.Get_rank() == 0:
    print(json.dumps(out), flush=True)
