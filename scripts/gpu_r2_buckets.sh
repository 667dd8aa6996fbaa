#!/usr/bin/env bash
# DP gradient all-reduce overlapped with the wgrad GEMMs: bucket-size sweep
# (2 ranks sharing the GPU, 4 Llama-3-8B layers, bf16 grads, auto = fan-out).
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/r2bk
mkdir -p $OUT
export CCMPI_TIMEOUT=400 CCMPI_DEVICE_TIMEOUT_S=10 TMPDIR=/tmp
for b in 0 256 64 16 4; do
  for blk in 64 128; do
    timeout -k 10 200 scripts/mpirun -n 2 --timeout 190 python benchmarks/dp_grad_overlap.py --layers 4 --tokens 4096 \
        --bucket-mb $b --blocks $blk > $OUT/dp2_b${b}_c$blk.json 2> $OUT/dp2_b${b}_c$blk.err
    rc=$?; echo "bucket ${b} MiB, $blk CTAs rc=$rc: $(cat $OUT/dp2_b${b}_c$blk.json)"; [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
