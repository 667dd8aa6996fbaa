#!/usr/bin/env bash
# TP token-mode harness tests + TP overlap timing + kernel trace (2 ranks sharing the GPU).
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/r2ov
mkdir -p $OUT
export CCMPI_TIMEOUT=300 CCMPI_DEVICE_TIMEOUT_S=10 TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_distributed.py -k "harness_matches and token" -x -v --timeout 300 --timeout-method thread > $OUT/pytest_token.log 2>&1
rc=$?; echo "token tests rc=$rc"; grep -E "PASSED|FAILED" $OUT/pytest_token.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 scripts/mpirun -n 2 --timeout 190 python benchmarks/tp_overlap.py > $OUT/tp2.json 2> $OUT/tp2.err
rc=$?; echo "tp overlap rc=$rc"; cat $OUT/tp2.json; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 scripts/mpirun -n 2 --timeout 190 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof_tp2 -o rank%pid% -- \
    python benchmarks/tp_overlap.py --steps 10 --chunks 4 > $OUT/prof_tp2.log 2>&1
rc=$?; echo "prof tp rc=$rc"
python scripts/overlap_from_trace.py $OUT/prof_tp2 --compute gemm,attn > $OUT/tp2_trace_overlap.md; cat $OUT/tp2_trace_overlap.md
exit $rc
