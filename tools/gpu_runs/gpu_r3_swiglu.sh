#!/usr/bin/env bash
# Fused SwiGLU: GPU numerics (kernel + ParallelSwiGLUMLP at 1 and 2 ranks), then the
# Llama-3-8B MLP block at TP = 1 with the fused gate vs the eager torch gate, and a
# rocprofv3 kernel-stats run of the fused block.  First failing step ends the script.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
OUT=gpurun_out/${OUT_TAG:-r3_swiglu}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  tests/test_gpu_kernels.py tests/test_gpu_distributed.py -k "swiglu" > $OUT/tests.log 2>&1
rc=$?; tail -12 $OUT/tests.log; [ $rc -ne 0 ] && { echo "tests failed rc=$rc"; exit $rc; }
for gate in fused eager; do
  flag=""; [ $gate = eager ] && flag="--eager-gate"
  timeout -k 10 200 python -u benchmarks/tp_mlp.py --iters 20 $flag > $OUT/tp_mlp_$gate.json 2> $OUT/tp_mlp_$gate.err
  rc=$?; cat $OUT/tp_mlp_$gate.json; [ $rc -ne 0 ] && { tail -5 $OUT/tp_mlp_$gate.err; exit $rc; }
done
CCMPI_TP_GEMM=blas timeout -k 10 200 python -u benchmarks/tp_mlp.py --iters 20 > $OUT/tp_mlp_fused_blas.json 2> $OUT/tp_mlp_blas.err
rc=$?; cat $OUT/tp_mlp_fused_blas.json; [ $rc -ne 0 ] && exit $rc
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python3 benchmarks/tp_mlp.py --iters 5 \
  > $OUT/prof.log 2>&1
rc=$?; tail -3 $OUT/prof.log; [ $rc -ne 0 ] && exit $rc
echo swiglu done
