#!/usr/bin/env bash
# Token fc_o TP pipeline at 2 shared ranks: side-stream priority -1 vs 0, alone and
# inside the torchrun bench process (which also holds DP-overlap / comm streams).
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/tpprio
mkdir -p $OUT
export CCMPI_TIMEOUT=300 CCMPI_DEVICE_TIMEOUT_S=10 TMPDIR=/tmp
for pr in -1 0; do
  CCMPI_TP_STREAM_PRIORITY=$pr timeout -k 10 200 scripts/mpirun -n 2 --timeout 190 python -u benchmarks/tp_overlap.py --chunks 1,4 --steps 30 > $OUT/tp_prio$pr.json 2> $OUT/tp_prio$pr.err
  rc=$?; echo "prio=$pr rc=$rc"; cat $OUT/tp_prio$pr.json; [ $rc -ne 0 ] && { tail $OUT/tp_prio$pr.err; exit $rc; }
done
for pr in 0; do
  CCMPI_TP_STREAM_PRIORITY=$pr timeout -k 10 420 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29502 bench.py --gpus 2 --steps 5 --warmup 2 --dp-layers 4 > $OUT/bench_prio$pr.json 2> $OUT/bench_prio$pr.err
  rc=$?; echo "bench prio=$pr rc=$rc"; python -c "import json,sys; d=json.load(open('$OUT/bench_prio$pr.json')); print(d['config']['harness']['token_fc_o'])"; [ $rc -ne 0 ] && exit $rc
done
exit 0
