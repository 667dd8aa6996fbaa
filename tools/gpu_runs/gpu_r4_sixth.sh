#!/usr/bin/env bash
# Pair-slot ring as the default: ring GEMM tests (incl. beside other ranks' collectives on
# the shared GPU), a kernel trace of the TP=1 MLP block, PMC of the pair kernel vs hipBLASLt.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
OUT=gpurun_out/r4_six
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_distributed.py::test_swiglu_mlp_ring_gemm_beside_collectives_gpu \
  tests/test_gpu_kernels.py -k "ring or swiglu or pair" > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/mlp_trace -o run -- \
  python3 benchmarks/tp_mlp.py --iters 5 --warmup 2 > $OUT/mlp_trace.json 2> $OUT/mlp_trace.err
rc=$?; echo "mlp trace rc=$rc: $(cut -c1-300 $OUT/mlp_trace.json)"; [ $rc -ne 0 ] && exit $rc
PMC_VARIANTS='-1:0 0:16392' SCHEDS=16392 OUT_TAG=r4_six bash tools/gpu_runs/gpu_r4_gemm.sh
