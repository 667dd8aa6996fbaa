#!/usr/bin/env bash
# Backward GEMM routes (K-major ring vs transposes + pair ring), the persistent pair ring,
# the vectorized transpose, and the TP=1 MLP block under each; kernel trace of the default.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
OUT=gpurun_out/r4_bwd
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_kernels.py \
  tests/test_gpu_distributed.py::test_parallel_swiglu_mlp_gpu \
  -k "transpose or ring or swiglu or pair" > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python benchmarks/gemm_ps_ab.py --scheds 16392,16393 > $OUT/ps_ab.jsonl 2> $OUT/ps_ab.err
rc=$?; echo "ps_ab rc=$rc"; cat $OUT/ps_ab.jsonl; [ $rc -ne 0 ] && exit $rc
for v in ring:16392 transpose:16392 transpose:16393; do
  route=${v%%:*}; rs=${v##*:}
  CCMPI_KMAJOR_ROUTE=$route CCMPI_RING_SCHED=$rs timeout -k 10 200 python benchmarks/tp_mlp.py > $OUT/tp_mlp_${route}_$rs.json 2> $OUT/tp_mlp_${route}_$rs.err
  rc=$?; echo "tp_mlp $v rc=$rc: $(cut -c1-420 $OUT/tp_mlp_${route}_$rs.json)"; [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/mlp_trace -o run -- \
  python3 benchmarks/tp_mlp.py --iters 5 --warmup 2 > $OUT/mlp_trace.json 2> $OUT/mlp_trace.err
rc=$?; echo "mlp trace rc=$rc"; exit $rc
