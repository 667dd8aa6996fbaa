#!/usr/bin/env bash
# The driver's N=4 invocation rehearsed with 4 ranks on the one GPU (smaller all-reduce and DP
# model): the coll phase's world tuning sweep plus the new TP-pair sweep, then the harness
# (DP2 x TP2) on the pair table.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
OUT=gpurun_out/r4_tune4
mkdir -p $OUT
timeout -k 10 1000 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
  --master-port 29541 bench.py --gpus 4 --steps 5 --warmup 2 --size-mb 256 --dp-layers 2 --tune-max-mb 16 --verbose \
  > $OUT/bench4.json 2> $OUT/bench4.err
rc=$?; echo "torchrun N=4 rc=$rc"; python3 -c "
import json; d=json.load(open('$OUT/bench4.json')); c=d['config']
print(d['value'], c['parallelism'], c.get('tp_fwd_step_ms'), {k: v['ok'] for k, v in c.get('phases', {}).items()})
print(json.dumps(c.get('tuning'))[:1500])"; exit $rc
