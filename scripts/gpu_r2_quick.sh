#!/usr/bin/env bash
# Quick multi-rank smoke of the device collectives (short device timeout).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r2q
export CCMPI_TIMEOUT=200 CCMPI_DEVICE_TIMEOUT_S=5 TMPDIR=/tmp
for n in ${RANKS:-2 3 4}; do
  timeout -k 10 200 scripts/mpirun -n $n --timeout 190 python -u tests/workers/device_worker.py --matrix ${MATRIX:-quick} ${EXTRA:-} > gpurun_out/r2q/q$n.log 2>&1
  rc=$?; echo "quick p=$n rc=$rc"; grep -E "device checks|FAIL|Error|error" gpurun_out/r2q/q$n.log | head -12; [ $rc -ne 0 ] && exit $rc
done
exit 0
