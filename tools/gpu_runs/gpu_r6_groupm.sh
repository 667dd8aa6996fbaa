#!/usr/bin/env bash
# Round 6: tile order (group-M) of the pair ring on the backward K-major shapes (dW: both operands
# K-major, dX: K-major B) and the forward NT shapes, against hipBLASLt.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
OUT=gpurun_out/${OUT_TAG:-r6_groupm}
mkdir -p $OUT
ROUTE=dW SHAPES=28672x4096x4096,4096x14336x4096,14336x4096x4096 timeout -k 10 300 python3 benchmarks/gemm_groupm.py > $OUT/groupm.jsonl 2> $OUT/err.log || exit $?
ROUTE=dX SHAPES=4096x4096x28672,4096x14336x4096 timeout -k 10 300 python3 benchmarks/gemm_groupm.py >> $OUT/groupm.jsonl 2>> $OUT/err.log || exit $?
ROUTE=nt SHAPES=4096x28672x4096,28672x4096x4096 timeout -k 10 300 python3 benchmarks/gemm_groupm.py >> $OUT/groupm.jsonl 2>> $OUT/err.log || exit $?
echo done
