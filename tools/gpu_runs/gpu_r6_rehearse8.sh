#!/usr/bin/env bash
# Round 6: the driver's N = 8 launch (torch.distributed.run, 8 ranks) rehearsed on the one GPU with
# reduced sizes -- every phase of the N >= 2 path must finish and merge into one line, now with
# the GPU-local placement (torchrun path), the DDP overlapped / deferred choice and the agreed
# MLP row-mode choice.  Not a performance number (8 processes share one GPU; no xGMI).
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
OUT=gpurun_out/${OUT_TAG:-r6_rehearse8}
mkdir -p $OUT
GPU_MAX_HW_QUEUES=1 timeout -k 10 1000 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
  --master-addr 127.0.0.1 --master-port 29547 bench.py --gpus 8 --steps 5 --warmup 2 --size-mb 256 --a2a-mb 32 \
  --dp-layers 2 --dp-tokens 1024 --dp-vocab 0 --mlp-tokens 2048 --tune-max-mb 16 --batch 512 --verbose \
  > $OUT/bench8.json 2> $OUT/bench8.err
rc=$?; echo "torchrun N=8 rc=$rc"; python3 -c "
import json; d=json.loads(open('$OUT/bench8.json').read().strip().splitlines()[-1]); c=d['config']
print(d['value'], d.get('partial'), d.get('warning'), c['parallelism'], c.get('tp_fwd_step_ms'))
print({k: (v['ok'], v.get('binding'), (v.get('bound_cpus') or [''])[:2]) for k, v in c.get('phases', {}).items()})
print('placement', c.get('placement', [])[:3])
print('mlp', {k: c['tp_mlp'].get(k) for k in ('row_mode', 'fwd_ms', 'fwd_bwd_ms')}, c['tp_mlp'].get('row_mode_variants', {}).get('auto_choice'))
print('dp', {k: c['dp_overlap'].get(k) for k in ('compute_ms', 'comm_ms', 'overlapped_ms', 'deferred_ms', 'step_ms', 'schedule', 'comm_hidden_fraction', 'comm_full_ms')})
print('harness', c['harness'].get('fc_o_tp_form'), c['harness'].get('fwd_timed'), c['harness'].get('fc_o_variants'))
print('host', c.get('host_cpu', {}).get('allreduce'))
" || true
exit $rc
