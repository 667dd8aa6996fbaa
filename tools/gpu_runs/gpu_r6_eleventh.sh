#!/usr/bin/env bash
# Round 6: where the in-kernel weight fold's ~3.3 us goes (phase stamps with and without --fold).
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
OUT=gpurun_out/${OUT_TAG:-r6_eleventh}
mkdir -p $OUT
for H in 2 4; do
  for F in "" "--fold"; do
    timeout -k 10 120 python benchmarks/qkv_fused_micro.py --H $H --B 2048 --grid 256 --train 0 --iters 300 --nolse --only img --trace $F \
      >> $OUT/trace.jsonl 2>> $OUT/trace.err || exit $?
  done
done
echo done
