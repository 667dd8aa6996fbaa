#!/usr/bin/env bash
# Round 5: launch plans with the allocation guard (plan / graph tests), then the training step's
# kernels (eager, graph, plan) under a kernel trace.
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/${OUT_TAG:-r5_29}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_distributed.py -k "plan or graph_train" tests/test_gpu_kernels.py -k "plan or graph_train or adam" > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -ne 0 ] && { grep -E "FAILED|^E |Error" $OUT/tests.log | head -30; exit $rc; }
timeout -k 10 200 python3 benchmarks/train_graph_probe.py > $OUT/probe.txt 2> $OUT/probe.err
rc=$?; cat $OUT/probe.txt; [ $rc -ne 0 ] && { tail -20 $OUT/probe.err; exit $rc; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
  python3 benchmarks/train_graph_probe.py > $OUT/probe_prof.txt 2> $OUT/probe_prof.err
rc=$?; echo "prof rc=$rc"; exit $rc
