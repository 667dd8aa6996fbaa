#!/usr/bin/env bash
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
mkdir -p gpurun_out/r4_probe
timeout -k 10 300 python benchmarks/mlp_fwd_probe.py > gpurun_out/r4_probe/mlp_fwd.json 2> gpurun_out/r4_probe/mlp_fwd.err
rc=$?; echo "probe rc=$rc: $(cat gpurun_out/r4_probe/mlp_fwd.json)"; [ $rc -ne 0 ] && tail -5 gpurun_out/r4_probe/mlp_fwd.err; exit $rc
