#!/usr/bin/env bash
# The driver's round-end GPU tiers on this tree: pytest -m gpu, smoke().
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/${OUT_TAG:-r4_suite}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest_gpu.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error|error" $OUT/pytest_gpu.log | head -20; exit $rc; }
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 $OUT/smoke.log
exit $rc
