#!/usr/bin/env bash
# Round 5, twentieth GPU pass: why the graph-replayed training step is slower than eager --
# timings, then a kernel trace of the replays.
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/r5_twentieth
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 python3 benchmarks/train_graph_probe.py > $OUT/probe.log 2>&1
rc=$?; tail -3 $OUT/probe.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
  python3 benchmarks/train_graph_probe.py > $OUT/probe_prof.log 2>&1
rc=$?; tail -2 $OUT/probe_prof.log; exit $rc
