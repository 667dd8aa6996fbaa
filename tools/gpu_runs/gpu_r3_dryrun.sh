#!/usr/bin/env bash
# where the 8-rank shared-GPU DP4xTP2 forward time goes.
# Three timings with the default hardware queues, three with GPU_MAX_HW_QUEUES=1,
# then one rocprofv3 kernel trace of each (per-rank timelines, queue ids).
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/r3_dryrun
mkdir -p $OUT
export CCMPI_DEVICE_TIMEOUT_S=20 TMPDIR=/tmp
L="python -m collective_communication_mpi_amd.launch -n ${N:-8} --timeout 200"
for q in default 1; do
  for i in 1 2 3; do
    if [ $q = default ]; then E=""; else E="GPU_MAX_HW_QUEUES=$q"; fi
    timeout -k 10 240 env $E $L python benchmarks/harness_dryrun.py ${ARGS:-} >> $OUT/times_q$q.jsonl 2>> $OUT/err.log
    rc=$?; [ $rc -ne 0 ] && { echo "dry run q=$q rc=$rc"; tail -20 $OUT/err.log; exit $rc; }
  done
  tail -3 $OUT/times_q$q.jsonl
done
[ -n "$NOPROF" ] && exit 0
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace_qdefault -o out -- \
  python -m collective_communication_mpi_amd.launch -n ${N:-8} --timeout 200 python benchmarks/harness_dryrun.py --steps 10 \
  > $OUT/trace_qdefault.log 2>&1 || { echo "trace failed"; tail $OUT/trace_qdefault.log; exit 1; }
echo dryrun done
