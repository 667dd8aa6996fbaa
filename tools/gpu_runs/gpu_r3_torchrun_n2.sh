#!/usr/bin/env bash
# The driver's N >= 2 bench command at N = 2 (torch.distributed.run, both ranks on this one
# GPU): supervisor, hand-written phase, DP-overlap phase at the full Llama-3-8B size, TP MLP
# phase, RCCL phase (skipped on a shared GPU).  One JSON line expected.
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/r3_torchrun_n2
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 5 > $OUT/bench2.json 2> $OUT/bench2.err
rc=$?; echo "torchrun bench rc=$rc"; cut -c1-1500 $OUT/bench2.json
exit $rc
