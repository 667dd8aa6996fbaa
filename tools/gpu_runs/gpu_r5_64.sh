#!/usr/bin/env bash
# Round 5: the forward plan with / without the pipelined fold, timed and under a kernel trace.
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/${OUT_TAG:-r5_64}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 python3 benchmarks/fwd_pipe_probe.py > $OUT/probe.json 2> $OUT/probe.err
rc=$?; cat $OUT/probe.json; [ $rc -ne 0 ] && { tail -20 $OUT/probe.err; exit $rc; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
  python3 benchmarks/fwd_pipe_probe.py > $OUT/probe_prof.json 2> $OUT/probe_prof.err
rc=$?; echo "prof rc=$rc"; exit $rc
