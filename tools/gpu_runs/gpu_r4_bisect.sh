#!/usr/bin/env bash
# Round-3 HIP-graph replay segfault: which preceding phase of the old one-process bench it
# needs.  8 ranks on the one GPU, one hardware queue each, the harness forward (HIP graph)
# after growing prefixes of the collective phase; stops at the first failing prefix (the
# native crash reporter's backtrace is in its .err).
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/${OUT_TAG:-r4_bisect}
mkdir -p $OUT
export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=${Q:-1}
export CCMPI_DEVICE_TIMEOUT_S=20 CCMPI_HARNESS_VERBOSE=1
# variant = prefix:train (train 0 = the round-3 harness_dryrun.py forward-only run)
for v in ${VARIANTS:-none:0 none:1 ar:1 ar,bf16,a2a,free:1}; do
  pre=${v%%:*}; train=${v##*:}
  p=$pre; [ "$p" = none ] && p=""
  timeout -k 10 300 python -m collective_communication_mpi_amd.launch -n 8 --timeout 280 \
    python benchmarks/graph_replay_repro.py --prefix "$p" --train $train > $OUT/${pre}_t$train.out 2> $OUT/${pre}_t$train.err
  rc=$?; echo "prefix '$pre' train $train rc=$rc"; tail -2 $OUT/${pre}_t$train.out
  if [ $rc -ne 0 ]; then
    grep -m1 -A60 "ccmpi crash" $OUT/${pre}_t$train.err || tail -40 $OUT/${pre}_t$train.err
    exit $rc
  fi
done
echo "bisect: every prefix replayed"
