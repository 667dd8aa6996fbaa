#!/usr/bin/env bash
# Round 6: phase stamps of the fused forward at the N = 8 per-rank shape (B = 512, H = 2), with and without the fold.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
OUT=gpurun_out/${OUT_TAG:-r6_trace512}
mkdir -p $OUT
for F in "" "--fold"; do
  timeout -k 10 120 python benchmarks/qkv_fused_micro.py --H 2 --B 512 --grid 256 --train 0 --iters 300 --nolse $F --only img --trace \
    >> $OUT/trace.jsonl 2>> $OUT/trace.err || exit $?
done
echo done
