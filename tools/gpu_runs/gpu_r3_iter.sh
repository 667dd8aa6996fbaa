#!/usr/bin/env bash
# Round-3 iteration: targeted GPU tests (pytest -k expression in $TESTS), then the
# four-wave GEMM sweep ($W4 variants on $SHAPES).  Every step under its own limit;
# the first failing step ends the script.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
OUT=gpurun_out/r3_iter${TAG:+_$TAG}
mkdir -p $OUT
if [ -n "$TESTS" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-600} python -u -m pytest -x -v --timeout 450 --timeout-method thread \
    tests/${TEST_FILE:-test_gpu_distributed.py} -k "$TESTS" > $OUT/tests.log 2>&1
  rc=$?; tail -25 $OUT/tests.log; [ $rc -ne 0 ] && { echo "tests failed rc=$rc"; exit $rc; }
fi
if [ -n "$W4" ]; then
  timeout -k 10 400 python3 benchmarks/gemm_bench.py --rounds 3 --w4 $W4 \
    --shapes ${SHAPES:-4096x4096x14336,4096x28672x4096,4096x4096x28672,4096x14336x4096} > $OUT/gemm_bench.txt 2>&1
  rc=$?; cat $OUT/gemm_bench.txt; [ $rc -ne 0 ] && { echo "gemm bench failed rc=$rc"; exit $rc; }
fi
if [ -n "$EXTRA" ]; then
  timeout -k 10 ${EXTRA_TIMEOUT:-300} bash -c "$EXTRA" > $OUT/extra.log 2>&1
  rc=$?; tail -30 $OUT/extra.log; [ $rc -ne 0 ] && { echo "extra failed rc=$rc"; exit $rc; }
fi
echo iter done
