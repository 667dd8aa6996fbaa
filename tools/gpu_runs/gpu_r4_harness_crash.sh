#!/usr/bin/env bash
# The round-3 / dry-run harness crash as bench.py runs it: the harness PHASE (first
# bench_forward + the fc_o variants) with 8 ranks on the one GPU and one hardware queue
# each, native crash reporter and per-step progress on.
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/${OUT_TAG:-r4_hcrash}
mkdir -p $OUT
export TMPDIR=/tmp GPU_MAX_HW_QUEUES=${Q:-1} CCMPI_HARNESS_VERBOSE=1 AMD_LOG_LEVEL=${LOG:-1}
timeout -k 10 300 python -m collective_communication_mpi_amd.launch -n 8 --timeout 280 \
  python bench.py --gpus 8 --steps 5 --warmup 2 --phase harness --result $OUT/harness.json --verbose \
  > $OUT/out.txt 2> $OUT/err.txt
rc=$?; echo "harness phase rc=$rc"; cat $OUT/harness.json 2>/dev/null | cut -c1-400; echo
grep -E "\[harness rank 0\]" $OUT/err.txt | tail -12
grep -m1 -A70 "ccmpi crash" $OUT/err.txt
exit $rc
