#!/usr/bin/env bash
# Round 5: weight fold pipelined into the fused forward's tail -- plan tests (1 and 2 ranks),
# harness tests, bench harness phase, forward kernels under a trace.
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/${OUT_TAG:-r5_57}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_distributed.py -k "plan or harness" > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -ne 0 ] && { grep -E "FAILED|^E |Error|assert" $OUT/tests.log | head -30; exit $rc; }
timeout -k 10 300 python3 bench.py --no-secondary --shared-dry-run 0 --host-ranks 0 --size-mb 64 > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "bench rc=$rc"; [ $rc -ne 0 ] && { tail -20 $OUT/bench.err; exit $rc; }
python3 -c "
import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]); c=d['config']; h=c.get('harness', {})
print('tp_fwd', c.get('tp_fwd_step_ms'), {k: h.get(k) for k in ('fwd_timed', 'fwd_ms_plan', 'fwd_ms_plan_pipelined_fold', 'fwd_ms_graph', 'fwd_ms_eager')})"
