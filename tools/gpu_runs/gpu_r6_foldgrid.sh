#!/usr/bin/env bash
# Round 6: fold workgroups of their own at small per-rank batches (grid widened by the fold's
# tiles; fold-only workgroups skip the attention prologue) -- kernel tests, micro at B = 512 / 2048
# (fold schedule on / off), the N = 1 harness.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
OUT=gpurun_out/${OUT_TAG:-r6_foldgrid}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_harness_grad.py -x -q --timeout 120 --timeout-method thread -k "attn or qkv or fold or plan or harness or patchify" > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for B in 512 2048; do
  for H in 2 4; do
    timeout -k 10 120 python benchmarks/qkv_fused_micro.py --H $H --B $B --grid 256 --train 0 --iters 300 --nolse --fold --only img \
      >> $OUT/micro.jsonl 2>> $OUT/micro.err || exit $?
  done
done
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 --mlp-tokens 0 --host-ranks 0 > $OUT/bench.json 2> $OUT/bench.err || exit $?
echo done
