#!/usr/bin/env bash
# Round 5, third GPU pass: MLP backward weight-gradient routes (transposes vs K-major B on the
# pair ring) and the ring / RHD all-reduce against the fan-out at 2 and 8 shared ranks.
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/${OUT_TAG:-r5_third}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python benchmarks/mlp_bwd_routes.py > $OUT/mlp_bwd_routes.jsonl 2> $OUT/mlp_bwd_routes.err
rc=$?; echo "routes rc=$rc"; cat $OUT/mlp_bwd_routes.jsonl; [ $rc -ne 0 ] && { tail -20 $OUT/mlp_bwd_routes.err; exit $rc; }
timeout -k 10 300 python -m collective_communication_mpi_amd.launch -n 2 --timeout 280 python benchmarks/coll_sweep.py \
  --ops allreduce --algos fanout,ring,rhd --blocks 64,128,256 --min-bytes 268435456 --max-mb 1024 --iters 5 \
  --out $OUT/ring2.jsonl > $OUT/ring2.log 2>&1
rc=$?; echo "ring2 rc=$rc"; [ $rc -ne 0 ] && { tail -20 $OUT/ring2.log; exit $rc; }
python scripts/coll_table.py $OUT/ring2.jsonl 2>/dev/null | head -40 || true
exit 0
