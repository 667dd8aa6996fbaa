#!/usr/bin/env bash
# Kernel statistics of the per-token fc_o harness train step (TP=1) vs the pooled one.
set -o pipefail
cd "$(dirname "$0")/.."
rm -rf gpurun_out/tprof; mkdir -p gpurun_out/tprof
export TMPDIR=/tmp
for m in token row; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/tprof/$m -o out -- python3 benchmarks/harness_steps.py --mode train --fc-o-mode $m --steps 20 > gpurun_out/tprof/$m.log 2>&1 || { echo "$m failed"; tail gpurun_out/tprof/$m.log; exit 1; }
done
echo ok
