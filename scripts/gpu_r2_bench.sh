#!/usr/bin/env bash
# bench.py at N=1 (with the 8-rank shared-GPU dry run) + the multi-rank bench-path test.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r2bench
export CCMPI_TIMEOUT=600 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_distributed.py -k bench_multi_rank -x -v --timeout 280 --timeout-method thread > gpurun_out/r2bench/pytest_bench.log 2>&1
rc=$?; echo "bench-path test rc=$rc"; tail -15 gpurun_out/r2bench/pytest_bench.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 700 python bench.py --verbose > gpurun_out/r2bench/bench1.json 2> gpurun_out/r2bench/bench1.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/r2bench/bench1.json; tail -5 gpurun_out/r2bench/bench1.err; exit $rc
