#!/usr/bin/env bash
# After pruning the ring GEMM variants: full GPU suite + smoke, GEMM A/B, N=1 bench.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
OUT=gpurun_out/r4_twelve
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 $OUT/smoke.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python benchmarks/gemm_ps_ab.py --scheds 8,16392,16393 > $OUT/ps_ab.jsonl 2> $OUT/ps_ab.err
rc=$?; echo "ps_ab rc=$rc"; cat $OUT/ps_ab.jsonl; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py > $OUT/bench1.json 2> $OUT/bench1.err
rc=$?; echo "bench rc=$rc"; python3 -c "import json;d=json.load(open('$OUT/bench1.json'));print(d['value'], d['config']['tp_fwd_step_ms'], d['config']['tp_mlp']['fwd_ms'], d['config']['tp_mlp']['fwd_bwd_ms'])"; exit $rc
