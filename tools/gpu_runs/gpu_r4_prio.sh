#!/usr/bin/env bash
# Pair ring: static wave priority (s_setprio 1) for odd waves / waves 2-3 / waves 0-1 vs none.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
mkdir -p gpurun_out/r4_prio
timeout -k 10 400 python benchmarks/gemm_ps_ab.py --scheds 16392,147464,278536,409608 \
  --shapes 4096x4096x14336,4096x28672x4096,4096x14336x4096 > gpurun_out/r4_prio/ps_ab.jsonl 2> gpurun_out/r4_prio/ps_ab.err
rc=$?; echo "rc=$rc"; cat gpurun_out/r4_prio/ps_ab.jsonl; exit $rc
