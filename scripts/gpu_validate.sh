#!/usr/bin/env bash
# Round-end rehearsal: GPU tests, smoke(), 1-GPU bench (each step time-limited, chained).
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/val
mkdir -p $OUT
export CCMPI_TIMEOUT=600 CCMPI_DEVICE_TIMEOUT_S=20 TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 700 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 $OUT/pytest_gpu.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error" $OUT/pytest_gpu.log | head; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 $OUT/smoke.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 700 python bench.py --verbose > $OUT/bench1.json 2> $OUT/bench1.err
rc=$?; echo "bench rc=$rc"; cat $OUT/bench1.json; exit $rc
