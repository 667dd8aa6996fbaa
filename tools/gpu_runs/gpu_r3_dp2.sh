#!/usr/bin/env bash
# BASELINE config 5 rehearsal: DP gradient all-reduce overlapped with the weight-gradient
# GEMMs at 2 ranks sharing the GPU, 4 layers first (function check), then the full
# Llama-3-8B size (32 layers + LM head + embedding, 16.06 GB of bf16 gradients).
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/r3_dp2
mkdir -p $OUT
export CCMPI_DEVICE_TIMEOUT_S=60 TMPDIR=/tmp
L="python -m collective_communication_mpi_amd.launch -n 2 --timeout 560"
timeout -k 10 300 $L python benchmarks/dp_grad_overlap.py --verbose --layers 4 > $OUT/dp2_l4.json 2>> $OUT/progress.log || { echo "l4 rc=$?"; tail -20 $OUT/progress.log; exit 1; }
cat $OUT/dp2_l4.json
timeout -k 10 600 $L python benchmarks/dp_grad_overlap.py --verbose > $OUT/dp2_full.json 2>> $OUT/progress.log || { echo "full rc=$?"; tail -20 $OUT/progress.log; exit 1; }
cat $OUT/dp2_full.json
echo dp2 done
