#!/usr/bin/env bash
# TCC HBM bytes (FETCH_SIZE, WRITE_SIZE; one counter per pass) of the ragged all-to-all
# kernels next to the fixed-size pull / push all-to-all: 2 ranks sharing the GPU, 64 MiB/rank.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/pmc_a2av
rm -rf $OUT; mkdir -p $OUT
export CCMPI_TIMEOUT=120 CCMPI_DEVICE_TIMEOUT_S=5 TMPDIR=/tmp
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 100 scripts/mpirun -n 2 --timeout 90 rocprofv3 --pmc $ctr --output-format csv -d $OUT/pmc_$ctr -o rank%pid% -- \
      python benchmarks/alltoall_moe.py --mb 64 --iters 3 --warmup 1 > $OUT/pmc_$ctr.log 2>&1
  rc=$?; echo "pmc $ctr rc=$rc"; [ $rc -ne 0 ] && { tail -5 $OUT/pmc_$ctr.log; exit $rc; }
done
python scripts/pmc_bytes.py $OUT/pmc_FETCH_SIZE $OUT/pmc_WRITE_SIZE > $OUT/bytes.md; cat $OUT/bytes.md
