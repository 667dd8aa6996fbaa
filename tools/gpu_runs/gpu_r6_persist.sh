#!/usr/bin/env bash
# Round 6: the pair-slot ring GEMM with / without the persistent grid on the MLP forward shapes.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
OUT=gpurun_out/${OUT_TAG:-r6_persist}
mkdir -p $OUT
timeout -k 10 400 python3 benchmarks/gemm_persist_ab.py --rounds 5 --shapes 4096x28672x4096,4096x4096x14336,4096x14336x4096,28672x4096x4096 \
  > $OUT/persist.jsonl 2> $OUT/err.log || exit $?
echo done
