#!/usr/bin/env bash
# Round-end rehearsal: GPU tests, smoke(), 1-GPU bench (each step time-limited, chained).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export CCMPI_TIMEOUT=300 CCMPI_DEVICE_TIMEOUT_S=20 TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --verbose > gpurun_out/bench1.json 2> gpurun_out/bench1.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench1.json; exit $rc
