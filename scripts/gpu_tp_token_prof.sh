#!/usr/bin/env bash
# Kernel stats of the TP=2 per-token forward at 2 ranks sharing the GPU (where does the
# time over the pooled forward go?).
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/tptok
rm -rf $OUT; mkdir -p $OUT
export CCMPI_TIMEOUT=300 CCMPI_DEVICE_TIMEOUT_S=10 TMPDIR=/tmp
timeout -k 10 200 scripts/mpirun -n 2 --timeout 190 python benchmarks/tp_overlap.py --steps 50 --chunks 1 > $OUT/tp2.json 2> $OUT/tp2.err
rc=$?; cat $OUT/tp2.json; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 scripts/mpirun -n 2 --timeout 190 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o rank%pid% -- \
    python benchmarks/tp_overlap.py --steps 20 --chunks 1 > $OUT/prof.log 2>&1
rc=$?; echo "prof rc=$rc"; exit $rc
