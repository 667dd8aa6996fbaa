#!/usr/bin/env bash
# Pair-slot ring GEMM check + A/B, the config-5 rehearsal with the shared-GPU overlap cap,
# then the runtime crash once more with the guard off and HIP error logging on (expected
# to crash: it ends the call).
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
bash tools/gpu_runs/gpu_r4_pair.sh || exit 1
bash tools/gpu_runs/gpu_r4_dp.sh || exit 1
mkdir -p gpurun_out/r4_fix
export CCMPI_FORCE_GRAPH=1 AMD_LOG_LEVEL=1 GPU_MAX_HW_QUEUES=1 CCMPI_HARNESS_VERBOSE=1
timeout -k 10 200 python -m collective_communication_mpi_amd.launch -n 8 --timeout 180 \
  python benchmarks/graph_replay_repro.py --prefix "" --train 0 --variants token:4 \
  > gpurun_out/r4_fix/forced.out 2> gpurun_out/r4_fix/forced.err
rc=$?; echo "forced multi-stream graph, one queue: rc=$rc"
grep -m3 -i "parallel stream\|hipGraph" gpurun_out/r4_fix/forced.err
grep -m2 "ccmpi crash" gpurun_out/r4_fix/forced.err
exit 0
