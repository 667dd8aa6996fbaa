#!/usr/bin/env bash
# Round-2 collective sweep at the 512-CTA budget: every hand-written algorithm
# at 2/4/8 ranks sharing the GPU, CTA-granularity and HW-queue experiments for
# small messages, and a rocprofv3 kernel trace.  Each step time-limited, chained.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/r2s
mkdir -p $OUT
export CCMPI_TIMEOUT=400 CCMPI_DEVICE_TIMEOUT_S=10 TMPDIR=/tmp
for n in 2 4 8; do
  timeout -k 10 400 scripts/mpirun -n $n --timeout 390 python benchmarks/coll_sweep.py --ops all --max-mb 256 \
      --algos oneshot,twoshot,push,reduce_bcast,ring,rhd,direct,gather,rscatter --out $OUT/all_p$n.jsonl > $OUT/all_p$n.log 2>&1
  rc=$?; echo "sweep p=$n rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
CCMPI_CTA_BYTES=16384 timeout -k 10 300 scripts/mpirun -n 8 --timeout 290 python benchmarks/coll_sweep.py --ops allreduce \
    --algos oneshot,twoshot,ring --max-mb 16 --out $OUT/cta16k_p8.jsonl > $OUT/cta16k_p8.log 2>&1
rc=$?; echo "cta16k rc=$rc"; [ $rc -ne 0 ] && exit $rc
GPU_MAX_HW_QUEUES=1 timeout -k 10 300 scripts/mpirun -n 8 --timeout 290 python benchmarks/coll_sweep.py --ops allreduce \
    --algos oneshot,twoshot --max-mb 1 --out $OUT/hwq1_p8.jsonl > $OUT/hwq1_p8.log 2>&1
rc=$?; echo "hwq1 rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 scripts/mpirun -n 8 --timeout 290 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_p8 -o rank%pid% -- \
    python benchmarks/coll_sweep.py --ops allreduce,alltoall --algos twoshot,push,ring,rhd,direct --min-bytes 67108864 --max-mb 64 --iters 10 > $OUT/prof_p8.log 2>&1
echo "prof p8 rc=$?"
