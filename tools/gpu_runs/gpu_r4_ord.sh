#!/usr/bin/env bash
# Experiment: the pair ring's odd-phase fragment reads front-loaded into the first four MFMA
# groups (sched bit 16), so the last read has 32 MFMAs of cover before the barrier, against the
# default pair ring and hipBLASLt (interleaved rounds).
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
OUT=gpurun_out/r4_ord
mkdir -p $OUT
timeout -k 10 400 python benchmarks/gemm_ps_ab.py --scheds 16392,81928 --rounds 9 > $OUT/ab.jsonl 2> $OUT/ab.err
rc=$?; echo "ab rc=$rc"; cat $OUT/ab.jsonl; exit $rc
