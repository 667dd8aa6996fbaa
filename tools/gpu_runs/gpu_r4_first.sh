#!/usr/bin/env bash
# Round 4, first GPU pass: allocation-identity probe, the TP / registration GPU tests touched
# this round, the restructured 1-GPU bench (supervised phases + 8-rank dry run), and the TP
# MLP row-parallel modes at TP = 2 on the shared GPU.
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/${OUT_TAG:-r4_first}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  "tests/test_gpu_distributed.py::test_bench_harness_crash_keeps_headline" > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -8 $OUT/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py --verbose > $OUT/bench1.json 2> $OUT/bench1.err
rc=$?; echo "bench rc=$rc"; cut -c1-600 $OUT/bench1.json; [ $rc -ne 0 ] && { tail -30 $OUT/bench1.err; exit $rc; }
timeout -k 10 300 python -m collective_communication_mpi_amd.launch -n 2 --timeout 280 \
  python benchmarks/tp_mlp.py --variants > $OUT/tp2_variants.json 2> $OUT/tp2_variants.err
rc=$?; echo "tp2 rc=$rc"; cat $OUT/tp2_variants.json
[ $rc -ne 0 ] && exit $rc
bash tools/gpu_runs/gpu_r4_gemm.sh
