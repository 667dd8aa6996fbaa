#!/usr/bin/env bash
# Round-end style validation: full GPU suite, smoke, 1-GPU bench (the driver's three tiers).
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${OUT_TAG:-r3_valid}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest_gpu.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error" $OUT/pytest_gpu.log | head; exit $rc; }
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 $OUT/smoke.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 500 python bench.py > $OUT/bench1.json 2> $OUT/bench1.err
rc=$?; echo "bench rc=$rc"; cut -c1-400 $OUT/bench1.json
exit $rc
