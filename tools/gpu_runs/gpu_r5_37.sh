#!/usr/bin/env bash
# Round 5: wgrad kernel with the old dW_qkv tile prefetched (numerics + micro), harness tests.
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/${OUT_TAG:-r5_37}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_kernels.py -k "fold_emb or harness or graph or adam" > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -ne 0 ] && { grep -E "FAILED|^E |Error" $OUT/tests.log | head -30; exit $rc; }
timeout -k 10 300 python3 benchmarks/train_kernels_micro.py wgrad > $OUT/micro.jsonl 2> $OUT/micro.err
rc=$?; cat $OUT/micro.jsonl; [ $rc -ne 0 ] && { tail -20 $OUT/micro.err; exit $rc; }
timeout -k 10 200 python3 benchmarks/train_graph_probe.py > $OUT/probe.txt 2> $OUT/probe.err
rc=$?; cat $OUT/probe.txt; exit $rc
