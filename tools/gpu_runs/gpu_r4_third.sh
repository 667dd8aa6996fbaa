#!/usr/bin/env bash
# Full GPU suite + smoke, then the chained-M0 GEMM A/B, the host-overhead record at 2 and 8
# ranks, and last the bench harness phase at 8 ranks / one queue (may crash: ends the call).
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
bash tools/gpu_runs/gpu_r4_suite.sh || exit 1
OUT_TAG=r4_gemm3 SCHEDS=8,4104,8200 PMC=0 bash tools/gpu_runs/gpu_r4_gemm.sh || exit 1
mkdir -p gpurun_out/r4_host
for n in 2 8; do
  timeout -k 10 200 python -m collective_communication_mpi_amd.launch -n $n --timeout 180 \
    python benchmarks/host_overhead.py > gpurun_out/r4_host/host_p$n.json 2> gpurun_out/r4_host/host_p$n.err || { echo "host p$n failed"; tail -20 gpurun_out/r4_host/host_p$n.err; exit 1; }
  cat gpurun_out/r4_host/host_p$n.json
done
bash tools/gpu_runs/gpu_r4_harness_crash.sh
