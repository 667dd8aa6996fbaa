#!/usr/bin/env bash
# Quick matrix (incl. HIP graph capture / replay of the collectives) at 2/3/8 ranks.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/r2g
mkdir -p $OUT
export CCMPI_TIMEOUT=300 CCMPI_DEVICE_TIMEOUT_S=10 TMPDIR=/tmp
for n in 2 3 8; do
  timeout -k 10 240 scripts/mpirun -n $n --timeout 230 python -u tests/workers/device_worker.py --matrix quick > $OUT/q$n.log 2>&1
  rc=$?; echo "quick p=$n rc=$rc"; grep -E "device checks|FAIL|Error" $OUT/q$n.log | head -12; [ $rc -ne 0 ] && exit $rc
done
exit 0
