#!/usr/bin/env bash
# Harness-graph fix check (GPU test), the 1-GPU bench with the 8-rank dry run, the config-5
# rehearsal on a real backward, then the runtime crash once more with the guard off and HIP
# error logging on (expected to crash: ends the call).
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
mkdir -p gpurun_out/r4_fix
timeout -k 10 500 python -u -m pytest -x -v --timeout 450 --timeout-method thread \
  "tests/test_gpu_distributed.py::test_harness_graph_replay_after_collectives_one_queue" > gpurun_out/r4_fix/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r4_fix/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py --verbose > gpurun_out/r4_fix/bench1.json 2> gpurun_out/r4_fix/bench1.err
rc=$?; echo "bench rc=$rc"; cut -c1-300 gpurun_out/r4_fix/bench1.json; [ $rc -ne 0 ] && exit $rc
bash tools/gpu_runs/gpu_r4_dp.sh || exit 1
export CCMPI_FORCE_GRAPH=1 AMD_LOG_LEVEL=1 GPU_MAX_HW_QUEUES=1 CCMPI_HARNESS_VERBOSE=1
timeout -k 10 200 python -m collective_communication_mpi_amd.launch -n 8 --timeout 180 \
  python benchmarks/graph_replay_repro.py --prefix "" --train 0 --variants token:4 \
  > gpurun_out/r4_fix/forced.out 2> gpurun_out/r4_fix/forced.err
rc=$?; echo "forced multi-stream graph, one queue: rc=$rc"
grep -m3 -i "parallel stream\|hipGraph" gpurun_out/r4_fix/forced.err
grep -m2 "ccmpi crash" gpurun_out/r4_fix/forced.err
exit 0
