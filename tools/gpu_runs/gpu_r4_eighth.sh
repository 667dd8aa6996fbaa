#!/usr/bin/env bash
# Transpose kernels (LDS tile vs register), then the TP=1 MLP block with the dW-only
# transpose route, and a kernel trace of it.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
OUT=gpurun_out/r4_bwd2
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_kernels.py \
  -k "transpose or kmajor" > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest.log; [ $rc -ne 0 ] && exit $rc
for k in lds reg; do
  CCMPI_TRANSPOSE=$k timeout -k 10 120 python benchmarks/transpose_bench.py > $OUT/transpose_$k.json 2> $OUT/transpose_$k.err
  rc=$?; echo "transpose $k rc=$rc: $(cat $OUT/transpose_$k.json)"; [ $rc -ne 0 ] && exit $rc
done
for route in ring transpose; do
  CCMPI_KMAJOR_ROUTE=$route timeout -k 10 200 python benchmarks/tp_mlp.py > $OUT/tp_mlp_$route.json 2> $OUT/tp_mlp_$route.err
  rc=$?; echo "tp_mlp $route rc=$rc: $(cut -c1-420 $OUT/tp_mlp_$route.json)"; [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/mlp_trace -o run -- \
  python3 benchmarks/tp_mlp.py --iters 5 --warmup 2 > $OUT/mlp_trace.json 2> $OUT/mlp_trace.err
rc=$?; echo "mlp trace rc=$rc"; exit $rc
