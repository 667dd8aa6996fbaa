#!/usr/bin/env bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export CCMPI_TIMEOUT=300 CCMPI_DEVICE_TIMEOUT_S=20 TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --gpus 2 --steps 10 --warmup 3 --size-mb 256 --verbose > gpurun_out/bench2_shared.json 2> gpurun_out/bench2_shared.err
rc=$?; echo "bench2 rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 scripts/mpirun -n 2 --timeout 290 python benchmarks/alltoall_moe.py --mb 64 > gpurun_out/moe2.json 2> gpurun_out/moe2.err
rc=$?; echo "moe rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python benchmarks/dp_grad_overlap.py --layers 4 > gpurun_out/overlap1.json 2> gpurun_out/overlap1.err
rc=$?; echo "overlap1 rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 scripts/mpirun -n 2 --timeout 390 python benchmarks/dp_grad_overlap.py --layers 2 --tokens 2048 > gpurun_out/overlap2.json 2> gpurun_out/overlap2.err
echo "overlap2 rc=$?"
CCMPI_TRACE=1 timeout -k 10 200 scripts/mpirun -n 2 --timeout 190 python benchmarks/sweep.py --op allreduce --max-mb 4 --iters 3 --algos twoshot,push > gpurun_out/trace2.log 2>&1
echo "trace rc=$?"
