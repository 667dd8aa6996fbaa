#!/usr/bin/env bash
# Round 5: vectorized AdamW + attention-backward grid / bias-gradient micro, then the train tests.
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/${OUT_TAG:-r5_55}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python3 benchmarks/train_kernels_micro.py bwd adamw > $OUT/micro.jsonl 2> $OUT/micro.err
rc=$?; cat $OUT/micro.jsonl; [ $rc -ne 0 ] && { tail -20 $OUT/micro.err; exit $rc; }
OUT_TAG=${OUT_TAG:-r5_55}_t bash tools/gpu_runs/gpu_r5_48.sh
