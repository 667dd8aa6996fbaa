#!/usr/bin/env bash
# Round 6 validation: the whole GPU test suite (one pytest process), smoke(), then the N = 1 bench
# exactly as the driver runs it.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp CCMPI_TIMEOUT=300 CCMPI_DEVICE_TIMEOUT_S=20
OUT=gpurun_out/${OUT_TAG:-r6_valid}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 $OUT/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "bench rc=$rc"; tail -1 $OUT/bench.json | cut -c1-600
exit $rc
