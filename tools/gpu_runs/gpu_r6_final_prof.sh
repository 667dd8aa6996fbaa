#!/usr/bin/env bash
# Round 6: rocprofv3 kernel statistics of the N = 1 bench after the attention work (every phase
# child is profiled: coll, harness, mlp), summarised with tools/kernel_stats_md.py.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
OUT=gpurun_out/${OUT_TAG:-r6_final_prof}
mkdir -p $OUT
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run_%pid% -- \
  python3 bench.py --shared-dry-run 0 --host-ranks 0 > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "benchprof rc=$rc"; cut -c1-200 $OUT/bench.json; [ $rc -ne 0 ] && { tail -20 $OUT/bench.err; exit $rc; }
python3 tools/kernel_stats_md.py $OUT/prof 14 > $OUT/kernels.md
echo done
