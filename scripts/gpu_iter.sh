#!/usr/bin/env bash
# Iteration run: new/changed GPU tests, TN split-K/order sweep, 1-GPU bench.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export CCMPI_TIMEOUT=300 CCMPI_DEVICE_TIMEOUT_S=20 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_harness_grad.py tests/test_gpu_kernels.py -k "harness or gemm_tn" -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_iter.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_iter.log; [ $rc -ne 0 ] && exit $rc
for o in 0 1; do
  CCMPI_TN_ORDER=$o timeout -k 10 200 python benchmarks/gemm_tn_splitk.py > gpurun_out/tn_order$o.txt 2>&1 || exit 1
done
echo "tn sweeps done"; cat gpurun_out/tn_order0.txt gpurun_out/tn_order1.txt
timeout -k 10 300 python bench.py --verbose > gpurun_out/bench1.json 2> gpurun_out/bench1.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench1.json; exit $rc
