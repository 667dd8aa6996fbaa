#!/usr/bin/env bash
# Experiment: L2 prefetch of the pair 2 (bit 16) or 4 (bit 17) phases before its LDS-DMA, in
# the pair-slot ring, against the default pair ring and hipBLASLt (interleaved rounds).
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
OUT=gpurun_out/r4_pf
mkdir -p $OUT
timeout -k 10 400 python benchmarks/gemm_ps_ab.py --scheds 16392,81928,147464 --rounds 7 > $OUT/ab.jsonl 2> $OUT/ab.err
rc=$?; echo "ab rc=$rc"; cat $OUT/ab.jsonl; exit $rc
