#!/usr/bin/env bash
# Full collective sweep with every current algorithm (ll, fanout, fanout_lds,
# push all-gather, ...) at 2/4/8 ranks sharing the GPU, plus a rocprofv3 kernel
# trace of the 8-rank 64 MiB points.  Each step time-limited, chained.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/r2s3
mkdir -p $OUT
export CCMPI_TIMEOUT=400 CCMPI_DEVICE_TIMEOUT_S=10 TMPDIR=/tmp
for n in 2 4 8; do
  timeout -k 10 400 scripts/mpirun -n $n --timeout 390 python benchmarks/coll_sweep.py --ops all --max-mb 256 \
      --out $OUT/all_p$n.jsonl > $OUT/all_p$n.log 2>&1
  rc=$?; echo "sweep p=$n rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 300 scripts/mpirun -n 8 --timeout 290 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_p8 -o rank%pid% -- \
    python benchmarks/coll_sweep.py --ops allreduce,allgather --algos twoshot,fanout,direct,push --min-bytes 67108864 --max-mb 64 --iters 10 > $OUT/prof_p8.log 2>&1
echo "prof p8 rc=$?"
