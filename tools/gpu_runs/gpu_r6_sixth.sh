#!/usr/bin/env bash
# Round 6: fused attention v6 (8-wave workgroups, W_h staged once per workgroup) -- tests, phase
# stamps at the DP4xTP2 (H = 2) and TP = 1 (H = 4) shapes, grid sweep, fold tail cost.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
OUT=gpurun_out/${OUT_TAG:-r6_sixth}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "attn or qkv or fold" > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for H in 2 4; do
  timeout -k 10 120 python benchmarks/qkv_fused_micro.py --H $H --B 2048 --grid 256 --train 0 --iters 300 --nolse --trace \
    >> $OUT/trace.jsonl 2>> $OUT/trace.err || exit $?
  timeout -k 10 120 python benchmarks/qkv_fused_micro.py --H $H --B 2048 --grid 256 --train 0 --iters 300 --nolse --fold --only img --trace \
    >> $OUT/trace.jsonl 2>> $OUT/trace.err || exit $?
done
for G in 128 192 256 512; do
  timeout -k 10 120 python benchmarks/qkv_fused_micro.py --H 2 --B 2048 --grid $G --iters 300 --only img --nolse >> $OUT/grid.jsonl 2>&1 || exit $?
done
echo done
