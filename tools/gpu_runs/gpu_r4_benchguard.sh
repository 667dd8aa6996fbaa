#!/usr/bin/env bash
# The coll phase's headline written before the tuning sweep: a crash injected right after it
# keeps the value; then the driver's N=2 invocation end to end with the new bench.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
OUT=gpurun_out/r4_benchguard
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread \
  tests/test_gpu_distributed.py::test_bench_tuning_crash_keeps_headline \
  tests/test_gpu_distributed.py::test_bench_harness_crash_keeps_headline > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 $OUT/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29537 bench.py --gpus 2 --steps 10 --warmup 3 > $OUT/bench2.json 2> $OUT/bench2.err
rc=$?; echo "torchrun N=2 rc=$rc"; cut -c1-400 $OUT/bench2.json; exit $rc
