#!/usr/bin/env bash
# GEMM variants (persistent prefetch-before-epilogue, parity-staggered phases), then the
# harness-graph crash bisect (stops at the first crash, which ends the call).
set -o pipefail
cd "$(dirname "$0")/../.."
OUT_TAG=r4_gemm2 SCHEDS=8,9,2056,2057 PMC=0 bash tools/gpu_runs/gpu_r4_gemm.sh || exit 1
bash tools/gpu_runs/gpu_r4_bisect.sh
