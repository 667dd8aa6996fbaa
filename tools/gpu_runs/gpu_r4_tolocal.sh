#!/usr/bin/env bash
# allreduce_to_local: two-shot pull (default) vs fan-out into heap scratch + local copy.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
OUT=gpurun_out/r4_tolocal
mkdir -p $OUT
for n in 2 8; do
  timeout -k 10 200 python -m collective_communication_mpi_amd.launch -n $n --timeout 180 python benchmarks/host_overhead.py > $OUT/host_p$n.json 2> $OUT/host_p$n.err || exit 1
  CCMPI_TO_LOCAL=fanout timeout -k 10 200 python -m collective_communication_mpi_amd.launch -n $n --timeout 180 python benchmarks/host_overhead.py > $OUT/host_fanout_p$n.json 2> $OUT/host_fanout_p$n.err || exit 1
  echo "p=$n: $(cat $OUT/host_p$n.json | cut -c1-400)"; echo "   fanout: $(cat $OUT/host_fanout_p$n.json)"
done
L="python -m collective_communication_mpi_amd.launch -n 2 --timeout 280"
for v in default fanout default fanout; do
  if [ $v = fanout ]; then export CCMPI_TO_LOCAL=fanout; else unset CCMPI_TO_LOCAL; fi
  CCMPI_SHARED_RING=1 timeout -k 10 300 $L python benchmarks/tp_mlp.py > $OUT/tp2_$v.json 2> $OUT/tp2_$v.err || exit 1
  echo "tp2 $v: $(cut -c1-330 $OUT/tp2_$v.json)"
done
