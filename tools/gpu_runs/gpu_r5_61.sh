#!/usr/bin/env bash
# Round 5: dW_emb on the matrix cores in the wgrad kernel -- micro-timings, then kernel +
# harness tests and the train-step probe (tools/gpu_runs/gpu_r5_48.sh).
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/${OUT_TAG:-r5_61}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 python3 benchmarks/train_kernels_micro.py wgrad > $OUT/micro.jsonl 2> $OUT/micro.err
rc=$?; cat $OUT/micro.jsonl; [ $rc -ne 0 ] && { tail -20 $OUT/micro.err; exit $rc; }
CCMPI_WGRAD_GE=atomic timeout -k 10 200 python3 benchmarks/train_kernels_micro.py wgrad > $OUT/micro_atomic.jsonl 2> $OUT/micro_atomic.err
rc=$?; cat $OUT/micro_atomic.jsonl; [ $rc -ne 0 ] && { tail -20 $OUT/micro_atomic.err; exit $rc; }
OUT_TAG=${OUT_TAG:-r5_61}_t bash tools/gpu_runs/gpu_r5_48.sh
