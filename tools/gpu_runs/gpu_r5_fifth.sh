#!/usr/bin/env bash
# Round 5, fifth GPU pass: the pair ring's barrier-skew upper bound (no-barrier ablation vs
# default vs hipBLASLt), then the 1-GPU bench with the token fc_o kernel and the no-transpose
# dW route.
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/${OUT_TAG:-r5_fifth}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python benchmarks/gemm_nobar_ab.py > $OUT/nobar.jsonl 2> $OUT/nobar.err
rc=$?; echo "nobar rc=$rc"; cat $OUT/nobar.jsonl; [ $rc -ne 0 ] && { tail -20 $OUT/nobar.err; exit $rc; }
timeout -k 10 700 python bench.py --verbose > $OUT/bench1.json 2> $OUT/bench1.err
rc=$?; echo "bench rc=$rc"; cut -c1-300 $OUT/bench1.json; [ $rc -ne 0 ] && { tail -30 $OUT/bench1.err; exit $rc; }
exit 0
