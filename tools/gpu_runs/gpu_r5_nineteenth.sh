#!/usr/bin/env bash
# Round 5, nineteenth GPU pass: HIP-graph-captured training steps (GraphedTrainStep, device-side
# AdamW step counter) -- graph-vs-eager tests, the harness tests, the bench harness phase.
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/${OUT_TAG:-r5_nineteenth}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_distributed.py -k "harness or graph" tests/test_gpu_kernels.py -k "harness or graph or adam" \
  > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -ne 0 ] && { grep -E "FAILED|^E |Error" $OUT/tests.log | head -30; exit $rc; }
timeout -k 10 300 python3 bench.py --no-secondary --shared-dry-run 0 --host-ranks 0 --size-mb 64 > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "bench rc=$rc"; [ $rc -ne 0 ] && { tail -20 $OUT/bench.err; exit $rc; }
python3 -c "
import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]); c=d['config']; h=c.get('harness', {})
print('tp_fwd', c.get('tp_fwd_step_ms'), 'train', c.get('tp_train_step_ms'), 'eager', h.get('train_ms_eager'), 'graph', h.get('train_hip_graph'), h.get('train_graph_skipped'))"
