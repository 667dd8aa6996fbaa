#!/usr/bin/env bash
# Round-3 validation: full GPU suite, smoke, 1-GPU bench (incl. the 8-rank shared dry run),
# then the DP-overlap rehearsal at 2 shared ranks (4 layers, then the full Llama-3-8B size).
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/r3_final
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest_gpu.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error" $OUT/pytest_gpu.log | head; exit $rc; }
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 $OUT/smoke.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 500 python bench.py --verbose > $OUT/bench1.json 2> $OUT/bench1.err
rc=$?; echo "bench rc=$rc"; cut -c1-600 $OUT/bench1.json; [ $rc -ne 0 ] && exit $rc
export CCMPI_DEVICE_TIMEOUT_S=60
L="python -m collective_communication_mpi_amd.launch -n 2 --timeout 280"
timeout -k 10 300 $L python benchmarks/dp_grad_overlap.py --verbose --layers 4 > $OUT/dp2_l4.json 2>> $OUT/dp2_progress.log
rc=$?; echo "dp l4 rc=$rc"; cat $OUT/dp2_l4.json; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 $L python benchmarks/dp_grad_overlap.py --verbose > $OUT/dp2_full.json 2>> $OUT/dp2_progress.log
rc=$?; echo "dp full rc=$rc"; cat $OUT/dp2_full.json
exit $rc
