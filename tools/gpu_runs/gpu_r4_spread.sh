#!/usr/bin/env bash
# Pair ring: DMA pieces spread over 1.5 phases (PAIR 3, sched bit 16) vs the default.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
mkdir -p gpurun_out/r4_spread
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "w4_shapes and ringpair" > gpurun_out/r4_spread/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/r4_spread/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python benchmarks/gemm_ps_ab.py --scheds 16392,81928 > gpurun_out/r4_spread/ps_ab.jsonl 2> gpurun_out/r4_spread/ps_ab.err
rc=$?; echo "rc=$rc"; cat gpurun_out/r4_spread/ps_ab.jsonl; exit $rc
