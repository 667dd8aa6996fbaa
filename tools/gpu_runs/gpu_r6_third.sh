#!/usr/bin/env bash
# Round 6: phase stamps of the fused QKV + attention + fc_o kernel (k_qkv_attn16_fwd) at the
# DP4xTP2 per-rank shape (H = 2, B = 2048) and H = 4; with / without the lse store.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
OUT=gpurun_out/${OUT_TAG:-r6_third}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "attn or qkv or fold" > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for H in 2 4; do
  for B in 512 2048; do
    timeout -k 10 120 python benchmarks/qkv_fused_micro.py --H $H --B $B --grid 512 --train 0 --iters 300 --trace \
      >> $OUT/trace.jsonl 2>> $OUT/trace.err || exit $?
    timeout -k 10 120 python benchmarks/qkv_fused_micro.py --H $H --B $B --grid 512 --train 0 --iters 300 --nolse --trace \
      >> $OUT/trace.jsonl 2>> $OUT/trace.err || exit $?
  done
done
echo done
