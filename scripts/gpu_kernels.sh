#!/usr/bin/env bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export CCMPI_TIMEOUT=300 CCMPI_DEVICE_TIMEOUT_S=20
timeout -k 10 400 python -m pytest tests/test_gpu_kernels.py -x -q > gpurun_out/kernels.log 2>&1
rc=$?; echo "kernels rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python benchmarks/copy_gemm_micro.py > gpurun_out/micro.log 2>&1
echo "micro rc=$?"
