#!/usr/bin/env bash
# Push broadcast: correctness (quick matrix) at 2/3/8 ranks, pull vs push sweep at 2/4/8.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/r2bc
mkdir -p $OUT
export CCMPI_TIMEOUT=300 CCMPI_DEVICE_TIMEOUT_S=10 TMPDIR=/tmp
for n in 2 3 8; do
  timeout -k 10 240 scripts/mpirun -n $n --timeout 230 python -u tests/workers/device_worker.py --matrix quick > $OUT/q$n.log 2>&1
  rc=$?; echo "quick p=$n rc=$rc"; grep -E "device checks|FAIL" $OUT/q$n.log | head -4; [ $rc -ne 0 ] && exit $rc
done
for n in 2 4 8; do
  timeout -k 10 300 scripts/mpirun -n $n --timeout 290 python benchmarks/coll_sweep.py --ops bcast --min-bytes 65536 --max-mb 256 \
      --out $OUT/b_p$n.jsonl > $OUT/b_p$n.log 2>&1
  rc=$?; echo "sweep p=$n rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
