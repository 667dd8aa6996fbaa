#!/usr/bin/env bash
# LDS-staged reduction experiment (CCMPI_LDS_REDUCE=1, fan-out all-reduce):
# correctness at 2/8 ranks, then register vs LDS sweep at 2/4/8 ranks.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/r2lds
mkdir -p $OUT
export CCMPI_TIMEOUT=300 CCMPI_DEVICE_TIMEOUT_S=10 TMPDIR=/tmp
for n in 2 8; do
  CCMPI_LDS_REDUCE=1 timeout -k 10 240 scripts/mpirun -n $n --timeout 230 python -u tests/workers/device_worker.py --matrix quick > $OUT/q$n.log 2>&1
  rc=$?; echo "quick lds p=$n rc=$rc"; grep -E "device checks|FAIL" $OUT/q$n.log | head -4; [ $rc -ne 0 ] && exit $rc
done
for n in 2 4 8; do
  for lds in 0 1; do
    CCMPI_LDS_REDUCE=$lds timeout -k 10 300 scripts/mpirun -n $n --timeout 290 python benchmarks/coll_sweep.py --ops allreduce --min-bytes 1048576 --max-mb 256 \
        --algos fanout --out $OUT/ar_p${n}_lds$lds.jsonl > $OUT/ar_p${n}_lds$lds.log 2>&1
    rc=$?; echo "sweep p=$n lds=$lds rc=$rc"; [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
