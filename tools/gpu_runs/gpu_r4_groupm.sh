#!/usr/bin/env bash
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
mkdir -p gpurun_out/r4_groupm
timeout -k 10 400 python benchmarks/gemm_groupm.py > gpurun_out/r4_groupm/groupm.jsonl 2> gpurun_out/r4_groupm/groupm.err
rc=$?; echo "rc=$rc"; cat gpurun_out/r4_groupm/groupm.jsonl; exit $rc
