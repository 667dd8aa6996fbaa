#!/usr/bin/env bash
# Multi-rank device tests (new matrix, ring/rhd, push all-to-all), each pytest step time-limited.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r2t
export CCMPI_TIMEOUT=600 CCMPI_DEVICE_TIMEOUT_S=20 TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_symheap.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r2t/pytest_heap.log 2>&1
rc=$?; echo "pytest heap rc=$rc"; tail -3 gpurun_out/r2t/pytest_heap.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 1000 python -u -m pytest tests/test_gpu_distributed.py -x -v --timeout 700 --timeout-method thread ${PYARGS:-} > gpurun_out/r2t/pytest_dist.log 2>&1
rc=$?; echo "pytest dist rc=$rc"; grep -E "PASSED|FAILED|ERROR" gpurun_out/r2t/pytest_dist.log | head -40; tail -30 gpurun_out/r2t/pytest_dist.log; exit $rc
