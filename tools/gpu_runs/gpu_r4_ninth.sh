#!/usr/bin/env bash
# Full GPU suite + smoke on the round's final kernels, then the backward-path A/B records
# (transpose kernels, pair ring with K-major B vs the 4-slot ring, K-major routes), the
# TP=1 MLP block with a kernel trace, the N=1 bench and the long-K probe.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
OUT=gpurun_out/r4_suite2
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 $OUT/smoke.log; [ $rc -ne 0 ] && exit $rc
for k in lds reg; do
  CCMPI_TRANSPOSE=$k timeout -k 10 120 python benchmarks/transpose_bench.py > $OUT/transpose_$k.json 2> $OUT/transpose_$k.err
  rc=$?; echo "transpose $k rc=$rc: $(cat $OUT/transpose_$k.json)"; [ $rc -ne 0 ] && exit $rc
done
for rs in 16392 8; do
  CCMPI_KMAJOR_ROUTE=ring CCMPI_RING_SCHED=$rs timeout -k 10 200 python benchmarks/gemm_ring_bench.py > $OUT/ring_bwd_$rs.json 2> $OUT/ring_bwd_$rs.err
  rc=$?; echo "ring bwd sched $rs rc=$rc"; cat $OUT/ring_bwd_$rs.json | cut -c1-300; [ $rc -ne 0 ] && exit $rc
done
for route in transpose ring; do
  CCMPI_KMAJOR_ROUTE=$route timeout -k 10 200 python benchmarks/tp_mlp.py > $OUT/tp_mlp_$route.json 2> $OUT/tp_mlp_$route.err
  rc=$?; echo "tp_mlp $route rc=$rc: $(cut -c1-420 $OUT/tp_mlp_$route.json)"; [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/mlp_trace -o run -- \
  python3 benchmarks/tp_mlp.py --iters 5 --warmup 2 > $OUT/mlp_trace.json 2> $OUT/mlp_trace.err
rc=$?; echo "mlp trace rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py --verbose > $OUT/bench1.json 2> $OUT/bench1.err
rc=$?; echo "bench rc=$rc"; cut -c1-400 $OUT/bench1.json; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python benchmarks/gemm_longk_probe.py > $OUT/longk.json 2> $OUT/longk.err
rc=$?; echo "longk rc=$rc: $(cat $OUT/longk.json)"; exit $rc
