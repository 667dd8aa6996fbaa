#!/usr/bin/env bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/prof
export CCMPI_TIMEOUT=300 CCMPI_DEVICE_TIMEOUT_S=20
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --verbose --no-harness > gpurun_out/bench1.json 2> gpurun_out/bench1.err &&
timeout -k 10 300 python bench.py --gpus 2 --steps 10 --warmup 3 --verbose --no-harness --size-mb 256 > gpurun_out/bench2_shared.json 2> gpurun_out/bench2_shared.err &&
timeout -k 10 400 scripts/mpirun -n 2 --timeout 390 python benchmarks/sweep.py --op all --max-mb 64 --iters 10 > gpurun_out/sweep2_shared.jsonl 2> gpurun_out/sweep2_shared.err &&
timeout -k 10 400 scripts/mpirun -n 1 --timeout 390 python benchmarks/sweep.py --op allreduce --max-mb 1024 --iters 10 --algos twoshot > gpurun_out/sweep1.jsonl 2> gpurun_out/sweep1.err &&
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/ar2 -o ar2 -- python benchmarks/sweep.py --op allreduce --max-mb 64 --iters 5 --algos twoshot,oneshot > gpurun_out/prof_ar1.log 2>&1
echo "rc=$?"
