#!/usr/bin/env bash
# Pair-slot ring GEMM (whole-line LDS-DMA pieces): numerics tests, then A/B against the
# 4-slot ring and hipBLASLt on the Llama MLP shapes.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
mkdir -p gpurun_out/r4_pair
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_kernels.py \
  -k "ringpair or pair" > gpurun_out/r4_pair/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r4_pair/pytest.log; [ $rc -ne 0 ] && exit $rc
SCHEDS=${SCHEDS:-8,16392} PMC=${PMC:-0} OUT_TAG=r4_pair bash tools/gpu_runs/gpu_r4_gemm.sh
