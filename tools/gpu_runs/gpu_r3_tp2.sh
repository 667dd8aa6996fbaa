#!/usr/bin/env bash
# TP = 2 Llama MLP on 2 ranks sharing the GPU: fused row-parallel GEMM + all-reduce vs the
# unfused layer, a kernel trace of the fused step (copy kernels around the TP all-reduce?),
# and the full-size DP gradient overlap (BASELINE config 5) at 2 ranks.
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/r3_tp2
mkdir -p $OUT
export CCMPI_DEVICE_TIMEOUT_S=30 TMPDIR=/tmp
L="python -m collective_communication_mpi_amd.launch -n 2 --timeout 280"
timeout -k 10 300 env CCMPI_TP_FUSED=1 $L python benchmarks/tp_mlp.py > $OUT/tp2_fused.json 2>> $OUT/err.log || { echo "tp2 fused rc=$?"; tail -20 $OUT/err.log; exit 1; }
timeout -k 10 300 $L python benchmarks/tp_mlp.py > $OUT/tp2_unfused.json 2>> $OUT/err.log || { echo "tp2 unfused rc=$?"; tail -20 $OUT/err.log; exit 1; }
cat $OUT/tp2_fused.json $OUT/tp2_unfused.json
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace_tp2 -o out -- \
  python -m collective_communication_mpi_amd.launch -n 2 --timeout 280 python benchmarks/tp_mlp.py --iters 3 --warmup 1 \
  > $OUT/trace_tp2.log 2>&1 || { echo "trace failed"; tail $OUT/trace_tp2.log; exit 1; }
timeout -k 10 600 $L python benchmarks/dp_grad_overlap.py --verbose > $OUT/dp2_overlap.json 2>> $OUT/dp2_progress.log || { echo "dp overlap rc=$?"; tail -20 $OUT/err.log; exit 1; }
cat $OUT/dp2_overlap.json
echo tp2 done
