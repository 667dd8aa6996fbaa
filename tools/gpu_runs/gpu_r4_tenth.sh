#!/usr/bin/env bash
# Multi-rank tests of the dW transpose route (fused dh^T, DDP sinks), then the N=1 bench
# with the back-to-back tp_mlp timing.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
OUT=gpurun_out/r4_ten
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_distributed.py::test_swiglu_mlp_ring_gemm_beside_collectives_gpu \
  tests/test_gpu_distributed.py::test_llama_ddp_gradient_sinks_gpu \
  tests/test_gpu_distributed.py::test_parallel_swiglu_mlp_gpu > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 $OUT/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py --verbose > $OUT/bench1.json 2> $OUT/bench1.err
rc=$?; echo "bench rc=$rc"; python3 -c "import json;d=json.load(open('$OUT/bench1.json'));print(d['value'], d['config']['tp_mlp'])"; [ $rc -ne 0 ] && exit $rc
[ "${WITH_ELEVENTH:-1}" = 1 ] && exec_eleventh=1
[ -n "$exec_eleventh" ] && bash tools/gpu_runs/gpu_r4_eleventh.sh
