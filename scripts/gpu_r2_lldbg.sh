#!/usr/bin/env bash
# Kernel-internal durations (rocprofv3 kernel trace) of the LL vs one-shot all-reduce.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/r2lld
rm -rf $OUT; mkdir -p $OUT
export CCMPI_TIMEOUT=100 CCMPI_DEVICE_TIMEOUT_S=5 TMPDIR=/tmp
for n in ${RANKS:-2 8}; do
  timeout -k 10 100 scripts/mpirun -n $n --timeout 90 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof$n -o rank%pid% -- \
     python benchmarks/coll_sweep.py --ops allreduce --algos ll,oneshot,twoshot --min-bytes 4096 --max-mb 1 --factor 16 --iters 50 > $OUT/prof$n.log 2>&1
  echo "p=$n rc=$?"
done
