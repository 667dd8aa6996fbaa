#!/usr/bin/env bash
# LL all-reduce: quick matrix at 2/3/4/8 ranks, then small-message sweep vs oneshot/twoshot.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/r2ll
mkdir -p $OUT
export CCMPI_TIMEOUT=200 CCMPI_DEVICE_TIMEOUT_S=5 TMPDIR=/tmp
for n in 2 3 4 8; do
  timeout -k 10 200 scripts/mpirun -n $n --timeout 190 python -u tests/workers/device_worker.py --matrix quick > $OUT/q$n.log 2>&1
  rc=$?; echo "quick p=$n rc=$rc $(grep -h 'device checks' $OUT/q$n.log | head -1)"; grep FAIL $OUT/q$n.log | head -5; [ $rc -ne 0 ] && exit $rc
done
for n in 2 4 8; do
  timeout -k 10 200 scripts/mpirun -n $n --timeout 190 python benchmarks/coll_sweep.py --ops allreduce --algos ll,oneshot,twoshot \
     --min-bytes 1024 --max-mb 1 --factor 2 --out $OUT/small_p$n.jsonl > $OUT/small_p$n.log 2>&1
  rc=$?; echo "sweep p=$n rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
