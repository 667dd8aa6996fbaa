#!/usr/bin/env bash
# The driver's N=2 invocation, rehearsed with both ranks on the one GPU.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
OUT=gpurun_out/r4_torchrun2
mkdir -p $OUT
timeout -k 10 1000 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29531 bench.py --gpus 2 --steps 10 --warmup 3 --verbose > $OUT/bench2.json 2> $OUT/bench2.err
rc=$?; echo "torchrun bench N=2 rc=$rc"; cut -c1-1500 $OUT/bench2.json; tail -5 $OUT/bench2.err; exit $rc
