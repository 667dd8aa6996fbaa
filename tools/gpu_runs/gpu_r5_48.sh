#!/usr/bin/env bash
# Round 5: fused loss head + dW_o (xent_head_wo): kernel numerics, harness train / graph / plan
# tests, train-step probe under a kernel trace.
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/${OUT_TAG:-r5_48}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_kernels.py -k "xent or adam or wgrad or fold" > $OUT/tests_k.log 2>&1
rc=$?; tail -2 $OUT/tests_k.log; [ $rc -ne 0 ] && { grep -E "FAILED|^E |Error" $OUT/tests_k.log | head -30; exit $rc; }
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_distributed.py tests/test_gpu_harness_grad.py -k "harness or graph or plan or grad" > $OUT/tests_h.log 2>&1
rc=$?; tail -2 $OUT/tests_h.log; [ $rc -ne 0 ] && { grep -E "FAILED|^E |Error" $OUT/tests_h.log | head -30; exit $rc; }
timeout -k 10 200 python3 benchmarks/train_graph_probe.py > $OUT/probe.txt 2> $OUT/probe.err
rc=$?; cat $OUT/probe.txt; [ $rc -ne 0 ] && { tail -20 $OUT/probe.err; exit $rc; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
  python3 benchmarks/train_graph_probe.py > $OUT/probe_prof.txt 2> $OUT/probe_prof.err
rc=$?; echo "prof rc=$rc"; exit $rc
