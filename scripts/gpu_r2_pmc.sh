#!/usr/bin/env bash
# HBM bytes of the collective kernels from TCC counters (one counter group per pass),
# and the MoE-shaped all-to-all at 4 and 8 ranks sharing the GPU.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/r2pmc
mkdir -p $OUT
export CCMPI_TIMEOUT=120 CCMPI_DEVICE_TIMEOUT_S=5 TMPDIR=/tmp
for n in 4 8; do
  timeout -k 10 200 scripts/mpirun -n $n --timeout 190 python benchmarks/alltoall_moe.py --mb 256 > $OUT/moe$n.json 2> $OUT/moe$n.err
  rc=$?; echo "moe p=$n rc=$rc: $(cat $OUT/moe$n.json)"; [ $rc -ne 0 ] && exit $rc
done
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 100 scripts/mpirun -n 2 --timeout 90 rocprofv3 --pmc $ctr --output-format csv -d $OUT/pmc_$ctr -o rank%pid% -- \
      python benchmarks/coll_sweep.py --ops allreduce,alltoall --algos twoshot,push,ring,rhd,direct --min-bytes 67108864 --max-mb 64 --iters 3 > $OUT/pmc_$ctr.log 2>&1
  rc=$?; echo "pmc $ctr rc=$rc"; [ $rc -ne 0 ] && { tail -5 $OUT/pmc_$ctr.log; exit $rc; }
done
ls -R $OUT | head -30
