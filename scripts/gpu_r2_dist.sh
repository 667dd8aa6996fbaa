#!/usr/bin/env bash
# Multi-rank device tests (new matrix, ring/rhd, push all-to-all), each pytest step time-limited.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r2t
export CCMPI_TIMEOUT=600 CCMPI_DEVICE_TIMEOUT_S=20 TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests/test_gpu_distributed.py -x -v --timeout 700 --timeout-method thread ${PYARGS:-} > gpurun_out/r2t/pytest_dist.log 2>&1
rc=$?; echo "pytest dist rc=$rc"; tail -30 gpurun_out/r2t/pytest_dist.log; exit $rc
