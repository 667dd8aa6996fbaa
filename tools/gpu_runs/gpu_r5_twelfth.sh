#!/usr/bin/env bash
# Round 5, twelfth GPU pass: fused patchify via LDS-DMA image staging, the tiled fp32-MFMA
# fold -- numerics tests, harness tests, then the harness forward / train step with kernel
# statistics for: fused QKV + fused patchify, fused QKV alone, unfused; fold FMA vs MFMA.
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/r5_twelfth
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_kernels.py -k "attn_qkv_fused or attn_token_fc_o or fold_emb" > $OUT/tests_k.log 2>&1
rc=$?; tail -3 $OUT/tests_k.log; [ $rc -ne 0 ] && { grep -E "FAILED|^E " $OUT/tests_k.log | head -30; exit $rc; }
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_distributed.py -k "harness" > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -ne 0 ] && { grep -E "FAILED|^E " $OUT/tests.log | head -20; exit $rc; }
for v in "1 1 mfma" "1 0 mfma" "0 0 mfma" "1 1 fma"; do
  set -- $v
  tag=q$1p$2$3
  CCMPI_FUSE_QKV=$1 CCMPI_FUSE_PATCHIFY=$2 CCMPI_FOLD=$3 timeout -k 10 300 rocprofv3 --kernel-trace --stats \
    --output-format csv -d $OUT/prof_$tag -o run_%pid% -- \
    python3 bench.py --no-secondary --shared-dry-run 0 --host-ranks 0 --size-mb 64 > $OUT/bench_$tag.json 2> $OUT/bench_$tag.err
  rc=$?; echo "$tag rc=$rc"; [ $rc -ne 0 ] && { tail -20 $OUT/bench_$tag.err; exit $rc; }
  python3 -c "
import json; d=json.loads(open('$OUT/bench_$tag.json').read().strip().splitlines()[-1]); c=d['config']
print('$tag tp_fwd', c.get('tp_fwd_step_ms'), 'train', c.get('tp_train_step_ms'))"
done
exit 0
