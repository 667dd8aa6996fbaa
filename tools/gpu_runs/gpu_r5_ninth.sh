#!/usr/bin/env bash
# Round 5, ninth GPU pass: kernel times of the harness forward / train step with the fused QKV
# kernel on and off (rocprofv3 kernel statistics of the harness phase only).
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/${OUT_TAG:-r5_ninth}
mkdir -p $OUT
export TMPDIR=/tmp
for f in 1 0; do
  CCMPI_FUSE_QKV=$f timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_fuse$f -o run_%pid% -- \
    python3 bench.py --no-secondary --shared-dry-run 0 --host-ranks 0 --size-mb 64 > $OUT/bench_fuse$f.json 2> $OUT/bench_fuse$f.err
  rc=$?; echo "fuse=$f rc=$rc"; [ $rc -ne 0 ] && { tail -20 $OUT/bench_fuse$f.err; exit $rc; }
  python3 -c "
import json; d=json.loads(open('$OUT/bench_fuse$f.json').read().strip().splitlines()[-1]); c=d['config']
print('tp_fwd', c.get('tp_fwd_step_ms'), 'train', c.get('tp_train_step_ms'))"
done
exit 0
