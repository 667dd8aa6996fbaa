#!/usr/bin/env bash
# 6 ranks on the one GPU (not a driver case): the TP-pair sweep with three pairs at once, then the
# DP3 x TP2 harness on the pair table.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
OUT=gpurun_out/r4_tune6
mkdir -p $OUT
timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 6 --master-addr 127.0.0.1 \
  --master-port 29543 bench.py --gpus 6 --steps 5 --warmup 2 --size-mb 64 --dp-layers 0 --mlp-tokens 0 --no-rccl \
  --tune-max-mb 4 --verbose > $OUT/bench6.json 2> $OUT/bench6.err
rc=$?; echo "torchrun N=6 rc=$rc"; python3 -c "
import json; d=json.load(open('$OUT/bench6.json')); c=d['config']
print(d['value'], 'partial' in d, c['parallelism'], c.get('tp_fwd_step_ms'), {k: v['ok'] for k, v in c.get('phases', {}).items()})
t = c.get('tuning', {}); print({k: t[k] for k in ('tp_pairs', 'dp_groups') if k in t})"; exit $rc
