#!/usr/bin/env bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export CCMPI_TIMEOUT=300 CCMPI_DEVICE_TIMEOUT_S=20
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --verbose > gpurun_out/bench1.json 2> gpurun_out/bench1.err
rc=$?; echo "bench1 rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --gpus 2 --steps 10 --warmup 3 --size-mb 256 --batch 1024 --verbose > gpurun_out/bench2_shared.json 2> gpurun_out/bench2_shared.err
echo "bench2 rc=$?"
