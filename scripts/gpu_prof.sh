#!/usr/bin/env bash
# rocprofv3 kernel-trace + stats of (a) the single-rank bench (copy + harness)
# and (b) the hand-written collectives at 2 ranks sharing the GPU.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/prof
export CCMPI_TIMEOUT=300 CCMPI_DEVICE_TIMEOUT_S=20 TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/bench1 -o bench1 -- python bench.py --steps 10 --warmup 3 > gpurun_out/prof_bench1.log 2>&1
rc=$?; echo "prof bench1 rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 scripts/mpirun -n 2 --timeout 390 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/ar2 -o rank%pid% -- python benchmarks/sweep.py --op all --max-mb 64 --iters 5 --warmup 2 > gpurun_out/prof_ar2.log 2>&1
rc=$?; echo "prof ar2 rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 scripts/mpirun -n 2 --timeout 390 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/harness_tp2 -o rank%pid% -- python -m collective_communication_mpi_amd.models.harness --tp 2 --batch 2048 --steps 10 > gpurun_out/prof_harness.log 2>&1
echo "prof harness rc=$?"
