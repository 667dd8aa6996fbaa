#!/usr/bin/env bash
# Round 6: HIP_FORCE_DEV_KERNARG A/B on the N = 1 bench's harness and its 8-rank dry run
# (device-memory kernargs help the GPU side of short kernels; do they cost eager launches?).
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
OUT=gpurun_out/${OUT_TAG:-r6_kernarg_ab}
mkdir -p $OUT
for K in 0 1 0 1; do
  HIP_FORCE_DEV_KERNARG=$K timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 --mlp-tokens 0 --host-ranks 0 \
    >> $OUT/ab_k$K.jsonl 2>> $OUT/ab_k$K.err || exit $?
done
echo done
