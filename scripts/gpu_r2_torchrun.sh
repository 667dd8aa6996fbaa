#!/usr/bin/env bash
# Rehearse the driver's N>=2 command (torch.distributed.run + bench.py) with ranks
# sharing this one GPU, after the quick device matrix (incl. the I* façade).
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/tr
mkdir -p $OUT
export CCMPI_TIMEOUT=300 CCMPI_DEVICE_TIMEOUT_S=10 TMPDIR=/tmp
timeout -k 10 200 scripts/mpirun -n 2 --timeout 190 python -u tests/workers/device_worker.py --matrix quick > $OUT/q2.log 2>&1
rc=$?; echo "quick p=2 rc=$rc"; grep -E "device checks|FAIL|Error" $OUT/q2.log | head; [ $rc -ne 0 ] && exit $rc
for n in ${NS:-2}; do
  timeout -k 10 420 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port $((29500 + n)) bench.py --gpus $n --steps 5 --warmup 2 --dp-layers ${DPL:-4} --verbose \
    > $OUT/bench_tr$n.json 2> $OUT/bench_tr$n.err
  rc=$?; echo "torchrun n=$n rc=$rc"; tail -c 1500 $OUT/bench_tr$n.json; [ $rc -ne 0 ] && { tail -20 $OUT/bench_tr$n.err; exit $rc; }
done
exit 0
