#!/usr/bin/env bash
# Round 5, seventh GPU pass: rocprofv3 kernel statistics of the N = 1 bench (which kernels the
# MLP backward runs now: no transpose), then the N = 8 rehearsal of the driver's launch.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
OUT=gpurun_out/${OUT_TAG:-r5_seventh}
mkdir -p $OUT
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run_%pid% -- \
  python3 bench.py --shared-dry-run 0 --host-ranks 0 > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "benchprof rc=$rc"; cut -c1-200 $OUT/bench.json; [ $rc -ne 0 ] && { tail -20 $OUT/bench.err; exit $rc; }
OUT_TAG=r5_rehearse8 bash tools/gpu_runs/gpu_r5_rehearse8.sh
