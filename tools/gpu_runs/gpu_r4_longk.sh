#!/usr/bin/env bash
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
mkdir -p gpurun_out/r4_longk
timeout -k 10 300 python benchmarks/gemm_longk_split.py > gpurun_out/r4_longk/split.json 2> gpurun_out/r4_longk/split.err
rc=$?; echo "rc=$rc: $(cat gpurun_out/r4_longk/split.json)"; [ $rc -ne 0 ] && tail -5 gpurun_out/r4_longk/split.err; exit $rc
