#!/usr/bin/env bash
# GPU tests, then harness profile at tp=2 (2 ranks share the GPU) + 1-rank bench.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/prof
export CCMPI_TIMEOUT=300 CCMPI_DEVICE_TIMEOUT_S=20 TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 scripts/mpirun -n 2 --timeout 390 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/harness_tp2_v2 -o rank%pid% -- python -m collective_communication_mpi_amd.models.harness --tp 2 --batch 2048 --steps 10 > gpurun_out/prof_harness2.log 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --verbose > gpurun_out/bench1.json 2> gpurun_out/bench1.err
echo "bench rc=$?"
