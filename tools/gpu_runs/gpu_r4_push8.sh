#!/usr/bin/env bash
# The push row mode (and the rest of the --big MLP checks) with 8 ranks sharing the GPU:
# the rank count of the driver's 8-GPU mlp phase.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
OUT=gpurun_out/r4_push8
mkdir -p $OUT
CCMPI_SHARED_RING=1 CCMPI_RING_MIN_MACS=1 CCMPI_KMAJOR_MIN_MACS=1 timeout -k 10 400 \
  scripts/mpirun -n 8 --timeout 380 python tests/workers/swiglu_mlp_worker.py --device cuda --big > $OUT/worker8.log 2>&1
rc=$?; echo "worker n=8 rc=$rc"; tail -5 $OUT/worker8.log; exit $rc
