#!/usr/bin/env bash
# Round 5, fourteenth GPU pass: transposed projection / register-chained z in the fused QKV
# kernel, packed bf16 conversions -- kernel + harness tests, the isolated kernel timings, and
# the harness forward / train step (fused patchify on and off).
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/${OUT_TAG:-r5_fourteenth}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_kernels.py -k "attn or fold_emb or gemm_bias or cast or rows_mean or harness" > $OUT/tests_k.log 2>&1
rc=$?; tail -3 $OUT/tests_k.log; [ $rc -ne 0 ] && { grep -E "FAILED|^E " $OUT/tests_k.log | head -30; exit $rc; }
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_distributed.py -k "harness" > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -ne 0 ] && { grep -E "FAILED|^E " $OUT/tests.log | head -20; exit $rc; }
for H in 4 2; do
  timeout -k 10 200 python3 benchmarks/qkv_fused_micro.py --H $H > $OUT/micro_h$H.jsonl 2> $OUT/micro_h$H.err
  rc=$?; echo "micro h$H rc=$rc"; [ $rc -ne 0 ] && { tail -20 $OUT/micro_h$H.err; exit $rc; }
done
for v in "1 1" "1 0"; do
  set -- $v
  tag=q$1p$2
  CCMPI_FUSE_QKV=$1 CCMPI_FUSE_PATCHIFY=$2 timeout -k 10 300 rocprofv3 --kernel-trace --stats \
    --output-format csv -d $OUT/prof_$tag -o run_%pid% -- \
    python3 bench.py --no-secondary --shared-dry-run 0 --host-ranks 0 --size-mb 64 > $OUT/bench_$tag.json 2> $OUT/bench_$tag.err
  rc=$?; echo "$tag rc=$rc"; [ $rc -ne 0 ] && { tail -20 $OUT/bench_$tag.err; exit $rc; }
  python3 -c "
import json; d=json.loads(open('$OUT/bench_$tag.json').read().strip().splitlines()[-1]); c=d['config']
print('$tag tp_fwd', c.get('tp_fwd_step_ms'), 'train', c.get('tp_train_step_ms'))"
done
exit 0
