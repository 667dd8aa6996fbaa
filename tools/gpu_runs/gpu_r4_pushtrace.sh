#!/usr/bin/env bash
# Kernel traces of the TP = 2 Llama MLP block (2 ranks on one GPU, ring GEMMs on) in the plain
# and push row modes: the down GEMM with and without the push epilogue, and the two-shot
# all-reduce against the inbox-to-local kernel.
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/r4_pushtrace
mkdir -p $OUT
export TMPDIR=/tmp CCMPI_SHARED_RING=1 CCMPI_DEVICE_TIMEOUT_S=60
for mode in plain push; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/$mode -o run -- \
    python -m collective_communication_mpi_amd.launch -n 2 --timeout 280 python benchmarks/tp_mlp.py --mode $mode \
    --iters 5 --warmup 2 > $OUT/$mode.json 2> $OUT/$mode.err || { echo "$mode rc=$?"; tail -20 $OUT/$mode.err; exit 1; }
  echo "== $mode"; tail -c 600 $OUT/$mode.json
  python3 scripts/kernel_durations.py $OUT/$mode --match k_ > $OUT/$mode.durations.md 2>&1
  cat $OUT/$mode.durations.md | head -30
done
