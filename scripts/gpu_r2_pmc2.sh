#!/usr/bin/env bash
# TCC HBM bytes (FETCH_SIZE, WRITE_SIZE; one counter per pass) of the fan-out
# all-reduce and the push all-gather next to their pull forms: 2 ranks, 64 MiB.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/r2pmc2
mkdir -p $OUT
export CCMPI_TIMEOUT=120 CCMPI_DEVICE_TIMEOUT_S=5 TMPDIR=/tmp
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 100 scripts/mpirun -n 2 --timeout 90 rocprofv3 --pmc $ctr --output-format csv -d $OUT/pmc_$ctr -o rank%pid% -- \
      python benchmarks/coll_sweep.py --ops allreduce,allgather --algos twoshot,fanout,direct,push --min-bytes 67108864 --max-mb 64 --iters 3 > $OUT/pmc_$ctr.log 2>&1
  rc=$?; echo "pmc $ctr rc=$rc"; [ $rc -ne 0 ] && { tail -5 $OUT/pmc_$ctr.log; exit $rc; }
done
python scripts/pmc_bytes.py $OUT/pmc_FETCH_SIZE $OUT/pmc_WRITE_SIZE
