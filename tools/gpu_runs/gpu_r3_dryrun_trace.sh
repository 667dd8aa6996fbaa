#!/usr/bin/env bash
# kernel traces of the 8-rank shared-GPU DP4xTP2 forward (default
# hardware queues and GPU_MAX_HW_QUEUES=1), plus three timings of each setting.
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/r3_dryrun2
mkdir -p $OUT
export CCMPI_DEVICE_TIMEOUT_S=20 TMPDIR=/tmp
L="python -m collective_communication_mpi_amd.launch -n 8 --timeout 200"
for i in 1 2 3; do
  timeout -k 10 240 $L python benchmarks/harness_dryrun.py >> $OUT/times_qdefault.jsonl 2>> $OUT/err.log || { echo "dry run rc=$?"; tail -20 $OUT/err.log; exit 1; }
  timeout -k 10 240 env GPU_MAX_HW_QUEUES=1 $L python benchmarks/harness_dryrun.py >> $OUT/times_q1.jsonl 2>> $OUT/err.log || { echo "dry run q1 rc=$?"; tail -20 $OUT/err.log; exit 1; }
done
cat $OUT/times_qdefault.jsonl $OUT/times_q1.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace_qdefault -o out -- \
  python -m collective_communication_mpi_amd.launch -n 8 --timeout 200 python benchmarks/harness_dryrun.py --steps 10 \
  > $OUT/trace_qdefault.log 2>&1 || { echo "trace failed"; tail $OUT/trace_qdefault.log; exit 1; }
GPU_MAX_HW_QUEUES=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace_q1 -o out -- \
  python -m collective_communication_mpi_amd.launch -n 8 --timeout 200 python benchmarks/harness_dryrun.py --steps 10 \
  > $OUT/trace_q1.log 2>&1 || { echo "trace q1 failed"; tail $OUT/trace_q1.log; exit 1; }
echo dryrun done
