#!/usr/bin/env bash
# Round 6: is the fused attention kernel's ~8 k-clock prologue the kernel-argument fetch?  The same
# micro with the kernarg segment in device memory (HIP_FORCE_DEV_KERNARG=1) vs the default.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
OUT=gpurun_out/${OUT_TAG:-r6_kernarg}
mkdir -p $OUT
for K in 0 1; do
  HIP_FORCE_DEV_KERNARG=$K timeout -k 10 120 python benchmarks/qkv_fused_micro.py --H 2 --B 2048 --grid 256 --train 0 \
    --iters 300 --nolse --trace > $OUT/trace_k$K.jsonl 2>&1 || exit $?
done
echo done
