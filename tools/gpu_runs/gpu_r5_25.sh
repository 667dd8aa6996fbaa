#!/usr/bin/env bash
# Round 5: the TP = 2 harness forward (2 ranks sharing the GPU), plain vs push-to-logits,
# timed and under a kernel trace -- the per-rank kernels of the N = 8 DP4xTP2 forward.
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/r5_25
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -m collective_communication_mpi_amd.launch -n 2 --timeout 280 python benchmarks/fc_o_forms.py \
  > $OUT/forms2.json 2> $OUT/forms2.err
rc=$?; echo "forms2 rc=$rc"; cat $OUT/forms2.json; [ $rc -ne 0 ] && { tail -20 $OUT/forms2.err; exit $rc; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run_%pid% -- \
  python -m collective_communication_mpi_amd.launch -n 2 --timeout 280 python benchmarks/fc_o_forms.py --steps 10 \
  > $OUT/forms2_prof.json 2> $OUT/forms2_prof.err
rc=$?; echo "prof rc=$rc"; exit $rc
