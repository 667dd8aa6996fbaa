#!/usr/bin/env bash
# Write-back stores: correctness (collective matrix, big, skew), TCC bytes, sweep.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/r2wb
mkdir -p $OUT
export CCMPI_TIMEOUT=600 CCMPI_DEVICE_TIMEOUT_S=10 TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_distributed.py -k "multi_rank or big or skew or watchdog" -x -v --timeout 600 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASSED|FAILED" $OUT/pytest.log | sed 's/.*:://' | tr '\n' ' '; echo; [ $rc -ne 0 ] && { tail -30 $OUT/pytest.log; exit $rc; }
export CCMPI_TIMEOUT=120 CCMPI_DEVICE_TIMEOUT_S=5
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 100 scripts/mpirun -n 2 --timeout 90 rocprofv3 --pmc $ctr --output-format csv -d $OUT/pmc_$ctr -o rank%pid% -- \
      python benchmarks/coll_sweep.py --ops allreduce,alltoall --algos twoshot,push,ring,rhd,direct --min-bytes 67108864 --max-mb 64 --iters 3 > $OUT/pmc_$ctr.log 2>&1
  rc=$?; echo "pmc $ctr rc=$rc"; [ $rc -ne 0 ] && { tail -5 $OUT/pmc_$ctr.log; exit $rc; }
done
python scripts/pmc_bytes.py $OUT/pmc_FETCH_SIZE $OUT/pmc_WRITE_SIZE
export CCMPI_TIMEOUT=400 CCMPI_DEVICE_TIMEOUT_S=10
for n in 2 8; do
  timeout -k 10 300 scripts/mpirun -n $n --timeout 290 python benchmarks/coll_sweep.py --ops all --min-bytes 1048576 --max-mb 256 \
      --algos oneshot,twoshot,push,reduce_bcast,ring,rhd,direct,gather,rscatter --out $OUT/all_p$n.jsonl > $OUT/all_p$n.log 2>&1
  rc=$?; echo "sweep p=$n rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
