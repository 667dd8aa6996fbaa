#!/usr/bin/env bash
set -o pipefail
cd "$(dirname "$0")/../.."
PMC_VARIANTS='0:16392 0:16393' SCHEDS=16392,16393 OUT_TAG=r4_pmc_persist bash tools/gpu_runs/gpu_r4_gemm.sh
