#!/usr/bin/env bash
# Push row-parallel mode (GEMM epilogue -> owners' inboxes, then inbox-to-local two-shot):
# correctness beside other ranks' collectives, the ring GEMM tests after the epilogue change,
# then the TP = 2 Llama MLP block with every row mode side by side (one GPU, ring GEMMs on).
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
OUT=gpurun_out/r4_push
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_distributed.py::test_swiglu_mlp_ring_gemm_beside_collectives_gpu \
  tests/test_gpu_distributed.py::test_parallel_swiglu_mlp_gpu > $OUT/pytest_dist.log 2>&1
rc=$?; echo "pytest dist rc=$rc"; tail -4 $OUT/pytest_dist.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_kernels.py \
  -k "ring or gemm or swiglu" > $OUT/pytest_kern.log 2>&1
rc=$?; echo "pytest kernels rc=$rc"; tail -3 $OUT/pytest_kern.log; [ $rc -ne 0 ] && exit $rc
CCMPI_SHARED_RING=1 timeout -k 10 300 scripts/mpirun -n 2 --timeout 280 python benchmarks/tp_mlp.py --variants \
  > $OUT/tp2_variants.json 2> $OUT/tp2_variants.err
rc=$?; echo "tp2 rc=$rc"; tail -c 1500 $OUT/tp2_variants.json; exit $rc
