#!/usr/bin/env bash
# Round 6: the fused-kernel micro (H = 2 / 4, with and without the fold), the standalone fold, the N = 1 harness.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
OUT=gpurun_out/${OUT_TAG:-r6_micro}
mkdir -p $OUT
for H in 2 4; do
  for F in "" "--fold"; do
    timeout -k 10 120 python benchmarks/qkv_fused_micro.py --H $H --B 2048 --grid 256 --train 0 --iters 300 --nolse $F --only img \
      >> $OUT/micro.jsonl 2>> $OUT/micro.err || exit $?
  done
done
timeout -k 10 120 python -c "
import torch, time
from collective_communication_mpi_amd import _native
d=_native.device(); st=torch.cuda.current_stream().cuda_stream
wq=torch.randn(768,768,device='cuda'); we=torch.randn(768,72,device='cuda'); o=torch.empty(768,72,device='cuda').bfloat16()
for _ in range(10): d.fold_emb_qkv(wq.data_ptr(),768,we.data_ptr(),72,o.data_ptr(),72,768,768,72,st)
torch.cuda.synchronize(); s=torch.cuda.Event(enable_timing=True); e=torch.cuda.Event(enable_timing=True)
s.record()
for _ in range(200): d.fold_emb_qkv(wq.data_ptr(),768,we.data_ptr(),72,o.data_ptr(),72,768,768,72,st)
e.record(); torch.cuda.synchronize(); print('fold_us', s.elapsed_time(e)*1e3/200)
" >> $OUT/micro.err 2>&1 || exit $?
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 --mlp-tokens 0 --host-ranks 0 > $OUT/bench.json 2> $OUT/bench.err || exit $?
echo done
