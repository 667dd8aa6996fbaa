#!/usr/bin/env bash
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/r2tp
mkdir -p $OUT
export CCMPI_TIMEOUT=100 CCMPI_DEVICE_TIMEOUT_S=5 TMPDIR=/tmp CCMPI_HARNESS_VERBOSE=1
for v in "eager_c2:CCMPI_NO_GRAPH=1:--chunks 2" "graph_c1:X=1:--chunks 1" "graph_c2:X=1:--chunks 2"; do
  IFS=: read name envv a <<< "$v"
  env $envv timeout -k 10 80 scripts/mpirun -n 2 --timeout 70 python benchmarks/tp_overlap.py --steps 5 $a > $OUT/$name.json 2> $OUT/$name.err
  echo "$name rc=$?: $(cat $OUT/$name.json) | $(grep -E 'harness|watchdog|Error' $OUT/$name.err | tr '\n' ' ' | cut -c1-600)"
done
exit 0
