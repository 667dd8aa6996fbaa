#!/usr/bin/env bash
# Peer-major CTA mapping for all-gather / all-to-all (CCMPI_PEER_MAJOR=1, experiment):
# correctness at 2/3/8 ranks, then default vs peer-major sweeps at 2/4/8 ranks.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/r2pm
mkdir -p $OUT
export CCMPI_TIMEOUT=300 CCMPI_DEVICE_TIMEOUT_S=10 TMPDIR=/tmp
for n in 2 3 8; do
  CCMPI_PEER_MAJOR=1 timeout -k 10 240 scripts/mpirun -n $n --timeout 230 python -u tests/workers/device_worker.py --matrix quick > $OUT/q$n.log 2>&1
  rc=$?; echo "quick pm p=$n rc=$rc"; grep -E "device checks|FAIL" $OUT/q$n.log | head -4; [ $rc -ne 0 ] && exit $rc
done
for n in 2 4 8; do
  for pm in 0 1; do
    CCMPI_PEER_MAJOR=$pm timeout -k 10 300 scripts/mpirun -n $n --timeout 290 python benchmarks/coll_sweep.py --ops allgather,alltoall --min-bytes 1048576 --max-mb 256 \
        --out $OUT/m_p${n}_pm$pm.jsonl > $OUT/m_p${n}_pm$pm.log 2>&1
    rc=$?; echo "sweep p=$n pm=$pm rc=$rc"; [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
