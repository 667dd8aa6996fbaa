#!/usr/bin/env bash
# Round-end validation after the push row mode: full GPU suite + smoke, the N=1 bench (with the 8-rank dry run) and
# the driver's N=2 invocation rehearsed with both ranks on the one GPU.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
OUT=gpurun_out/r4_final2
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 $OUT/smoke.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py --verbose > $OUT/bench1.json 2> $OUT/bench1.err
rc=$?; echo "bench N=1 rc=$rc"; cut -c1-300 $OUT/bench1.json; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 3 --verbose > $OUT/bench2.json 2> $OUT/bench2.err
rc=$?; echo "torchrun N=2 rc=$rc"; cut -c1-300 $OUT/bench2.json; exit $rc
