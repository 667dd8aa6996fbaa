#!/usr/bin/env bash
# Round 6: fused attention kernel v5 (hoisted W_h / bias loads, branchless X build, DPP token
# mean) -- correctness, timing and prologue phase stamps.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
OUT=gpurun_out/${OUT_TAG:-r6_fourth}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "attn or qkv or fold" > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for H in 2 4; do
  for G in 512 256; do
    timeout -k 10 120 python benchmarks/qkv_fused_micro.py --H $H --B 2048 --grid $G --train 0 --iters 300 --nolse --trace \
      >> $OUT/trace.jsonl 2>> $OUT/trace.err || exit $?
  done
done
timeout -k 10 120 python benchmarks/qkv_fused_micro.py --H 2 --B 2048 --iters 300 --only img > $OUT/micro_h2.jsonl 2>&1 || exit $?
echo done
