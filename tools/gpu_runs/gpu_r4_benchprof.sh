#!/usr/bin/env bash
# rocprofv3 kernel statistics of the N=1 bench (the driver's command), final kernels.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
OUT=gpurun_out/r4_benchprof
mkdir -p $OUT
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run_%pid% -- \
  python3 bench.py --shared-dry-run 0 > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "rc=$rc"; cut -c1-300 $OUT/bench.json; exit $rc
