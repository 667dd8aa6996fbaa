#!/usr/bin/env bash
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
mkdir -p gpurun_out/r4_swiglu_t
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "transposed or swiglu" > gpurun_out/r4_swiglu_t/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/r4_swiglu_t/pytest.log; [ $rc -ne 0 ] && exit $rc
for r in 64 128 64 128; do
  CCMPI_SWIGLU_T_ROWS=$r timeout -k 10 120 python benchmarks/swiglu_bwd_bench.py >> gpurun_out/r4_swiglu_t/bench.jsonl 2>> gpurun_out/r4_swiglu_t/bench.err || exit 1
done
cat gpurun_out/r4_swiglu_t/bench.jsonl
