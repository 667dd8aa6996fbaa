#!/usr/bin/env bash
# Kernel statistics of the harness forward and train step at TP=1 (bench N=1 config).
set -o pipefail
cd "$(dirname "$0")/.."
rm -rf gpurun_out/hprof; mkdir -p gpurun_out/hprof
export TMPDIR=/tmp
for m in fwd train; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/hprof/$m -o out -- python3 benchmarks/harness_steps.py --mode $m --steps 20 > gpurun_out/hprof/$m.log 2>&1 || { echo "$m failed"; exit 1; }
done
echo ok
