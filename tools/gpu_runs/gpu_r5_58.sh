#!/usr/bin/env bash
# Round 5: fold-in-kernel placement (start vs end of the fused forward): plan tests + bench each.
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/${OUT_TAG:-r5_58}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_distributed.py -k "forward_plan" > $OUT/tests.log 2>&1
rc=$?; tail -2 $OUT/tests.log; [ $rc -ne 0 ] && { grep -E "FAILED|^E |Error|assert" $OUT/tests.log | head -30; exit $rc; }
for at in start end start end; do
  CCMPI_FOLD_TAIL_AT=$at timeout -k 10 300 python3 bench.py --no-secondary --shared-dry-run 0 --host-ranks 0 --size-mb 64 > $OUT/bench_$at.json 2> $OUT/bench_$at.err
  rc=$?; [ $rc -ne 0 ] && { echo "bench $at rc=$rc"; tail -20 $OUT/bench_$at.err; exit $rc; }
  python3 -c "
import json; d=json.loads(open('$OUT/bench_$at.json').read().strip().splitlines()[-1]); c=d['config']; h=c.get('harness', {})
print('$at', 'tp_fwd', c.get('tp_fwd_step_ms'), {k: h.get(k) for k in ('fwd_timed', 'fwd_ms_plan', 'fwd_ms_plan_pipelined_fold')})"
done
