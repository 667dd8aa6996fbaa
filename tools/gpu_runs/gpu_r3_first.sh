#!/usr/bin/env bash
# Round-3 re-entry check: GPU suite, smoke, 1-GPU bench, four-wave GEMM A/B on the
# Llama MLP shapes.  Each step time-limited; the first failure ends the script.
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/r3_first
mkdir -p $OUT
export CCMPI_TIMEOUT=600 CCMPI_DEVICE_TIMEOUT_S=20 TMPDIR=/tmp
[ -z "$NOGEMM" ] && timeout -k 10 400 python3 benchmarks/gemm_bench.py --rounds 3 --w4 0:8,1:8,3:8 \
  --shapes 4096x4096x14336,4096x28672x4096,4096x4096x28672,4096x14336x4096,8192x8192x8192 > $OUT/gemm_bench.txt 2>&1
rc=$?; [ -z "$NOGEMM" ] && tail -8 $OUT/gemm_bench.txt; [ -z "$NOGEMM" ] && [ $rc -ne 0 ] && { echo "gemm rc=$rc"; exit $rc; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 700 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 $OUT/pytest_gpu.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error" $OUT/pytest_gpu.log | head; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 $OUT/smoke.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 700 python bench.py --verbose > $OUT/bench1.json 2> $OUT/bench1.err
rc=$?; echo "bench rc=$rc"; cat $OUT/bench1.json; exit $rc
