#!/usr/bin/env bash
# Per-rank GEMM shapes of the Llama MLP block at TP = 2 and TP = 8 (the 8-GPU bench's mlp
# phase): the pair ring (plain and persistent) and the 4-slot ring vs hipBLASLt.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
mkdir -p gpurun_out/r4_tpshapes
timeout -k 10 300 python benchmarks/gemm_ps_ab.py --scheds 8,16392,16393 \
  --shapes 4096x14336x4096,4096x4096x7168,4096x3584x4096,4096x4096x1792 > gpurun_out/r4_tpshapes/ps_ab.jsonl 2> gpurun_out/r4_tpshapes/ps_ab.err
rc=$?; echo "rc=$rc"; cat gpurun_out/r4_tpshapes/ps_ab.jsonl; exit $rc
