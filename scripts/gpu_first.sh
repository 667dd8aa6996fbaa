#!/usr/bin/env bash
# First GPU probe: device plane correctness at 1/2/4 ranks sharing one GPU.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export CCMPI_TIMEOUT=300 CCMPI_DEVICE_TIMEOUT_S=20
timeout -k 10 400 python -c "import torch; print(torch.__version__, torch.cuda.device_count(), torch.cuda.get_device_name(0)); p=torch.cuda.get_device_properties(0); print(p)" > gpurun_out/probe.log 2>&1 &&
timeout -k 10 300 scripts/mpirun -n 1 --timeout 290 python tests/workers/device_worker.py --quick > gpurun_out/dev1.log 2>&1 &&
timeout -k 10 300 scripts/mpirun -n 2 --timeout 290 python tests/workers/device_worker.py --quick > gpurun_out/dev2.log 2>&1 &&
timeout -k 10 400 scripts/mpirun -n 4 --timeout 390 python tests/workers/device_worker.py --quick > gpurun_out/dev4.log 2>&1
rc=$?
echo "main rc=$rc"
[ $rc -ne 0 ] && exit $rc
# RCCL with 2 ranks on one GPU (expected to be refused: duplicate GPU)
timeout -k 10 200 scripts/mpirun -n 2 --timeout 190 python tests/workers/device_worker.py --quick --rccl --sizes 16 > gpurun_out/dev2_rccl.log 2>&1
echo "rccl rc=$?"
exit $rc
