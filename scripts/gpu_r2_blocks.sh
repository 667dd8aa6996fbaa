#!/usr/bin/env bash
# CTA-budget sweep of the hand-written collectives with ranks sharing the GPU.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r2b
export CCMPI_TIMEOUT=300 CCMPI_DEVICE_TIMEOUT_S=5 TMPDIR=/tmp
OUT=gpurun_out/r2b
declare -A BL=([2]="48,128,256,512" [4]="24,64,128,256" [8]="12,32,64,128")
for n in 2 4 8; do
  timeout -k 10 400 scripts/mpirun -n $n --timeout 390 python benchmarks/coll_sweep.py --ops allreduce,alltoall,lastaxis \
      --algos ${ALGOS:-oneshot,twoshot,push,direct,gather,rscatter} --blocks ${BL[$n]} --min-bytes 1048576 --max-mb 256 \
      --out $OUT/p$n.jsonl > $OUT/p$n.log 2>&1
  rc=$?; echo "blocks sweep p=$n rc=$rc"; tail -1 $OUT/p$n.log; [ $rc -ne 0 ] && exit $rc
done
exit 0
