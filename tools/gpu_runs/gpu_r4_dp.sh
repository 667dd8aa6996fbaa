#!/usr/bin/env bash
# BASELINE config 5 rehearsal on a REAL backward (DDP + autograd over the Llama-3-8B-shaped
# model of the framework's layers): 2 ranks sharing the GPU, 2 layers first (function check),
# then the full 16 GB model, then a rocprofv3 kernel trace of a 4-layer run for the
# bucket-all-reduce / backward-GEMM concurrency.
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/${OUT_TAG:-r4_dp}
mkdir -p $OUT
export CCMPI_DEVICE_TIMEOUT_S=60 TMPDIR=/tmp
L="python -m collective_communication_mpi_amd.launch -n 2 --timeout 500"
timeout -k 10 300 $L python benchmarks/llama_ddp.py --verbose --layers 2 --blocks 64 > $OUT/l2.json 2>> $OUT/progress.log || { echo "l2 rc=$?"; tail -20 $OUT/progress.log; exit 1; }
cat $OUT/l2.json
timeout -k 10 560 $L python benchmarks/llama_ddp.py --verbose --blocks 32,64,128 > $OUT/full.json 2>> $OUT/progress.log || { echo "full rc=$?"; tail -20 $OUT/progress.log; exit 1; }
cat $OUT/full.json
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace -o run -- \
  python -m collective_communication_mpi_amd.launch -n 2 --timeout 280 python benchmarks/llama_ddp.py --layers 4 --blocks 64 \
  > $OUT/trace.json 2>> $OUT/progress.log || { echo "trace rc=$?"; tail -20 $OUT/progress.log; exit 1; }
python3 scripts/overlap_from_trace.py $OUT/trace --comm k_allreduce --compute gemm > $OUT/overlap.md 2>&1
cat $OUT/overlap.md | head -30
echo dp done
