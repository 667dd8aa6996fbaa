#!/usr/bin/env bash
# Round-2 collective sweep: RCCL same-GPU probe, then bytes/time sweeps of the
# hand-written collectives at 2/4/8 ranks sharing the GPU, then one rocprofv3
# kernel trace to cross-check the event timing.  Each step time-limited, chained.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r2
export CCMPI_TIMEOUT=300 CCMPI_DEVICE_TIMEOUT_S=10 TMPDIR=/tmp
OUT=gpurun_out/r2
ALGOS=${ALGOS:-oneshot,twoshot,push,reduce_bcast}
timeout -k 10 150 scripts/mpirun -n 2 --timeout 140 python benchmarks/rccl_shared_probe.py --out $OUT/rccl_probe2.json > $OUT/rccl_probe2.log 2>&1
echo "rccl probe rc=$? (recorded, not fatal)"
for n in 2 4 8; do
  timeout -k 10 400 scripts/mpirun -n $n --timeout 390 python benchmarks/coll_sweep.py --ops allreduce --algos $ALGOS \
      --blocks ${BLOCKS:-0} --max-mb 256 --out $OUT/ar_p$n.jsonl > $OUT/ar_p$n.log 2>&1
  rc=$?; echo "sweep allreduce p=$n rc=$rc"; tail -2 $OUT/ar_p$n.log; [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 400 scripts/mpirun -n 4 --timeout 390 python benchmarks/coll_sweep.py --ops allgather,reduce_scatter,alltoall,lastaxis \
    --algos ${OALGOS:-direct} --max-mb 256 --out $OUT/other_p4.jsonl > $OUT/other_p4.log 2>&1
rc=$?; echo "sweep other p=4 rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 scripts/mpirun -n 4 --timeout 290 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_p4 -o rank%pid% -- \
    python benchmarks/coll_sweep.py --ops allreduce --algos twoshot,push --min-bytes 67108864 --max-mb 64 --iters 10 > $OUT/prof_p4.log 2>&1
echo "prof p4 rc=$?"
