#!/usr/bin/env bash
# Round 6, second lease: (1) GPU tests of the round's changed paths (DDP schedules, llama DP
# record, MLP row-mode agreement, the 4-rank bench path), (2) the host fresh-array trace
# with marks inside isend, (3) the fused attention kernel's fixed vs
# per-iteration cost (batch sweep at the DP4xTP2 per-rank shape).
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
OUT=gpurun_out/${OUT_TAG:-r6_second}
mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests/test_gpu_distributed.py -x -v --timeout 300 --timeout-method thread \
  -k "ddp or llama or bench_multi_rank or swiglu_mlp_gpu" > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 $OUT/pytest.log
[ $rc -eq 0 ] || exit $rc
CCMPI_P2P_TRACE=2 HT_MODES=reuse,fresh,pool,fresh,reuse,fresh_touch_d,fresh_nofree,fresh timeout -k 10 300 \
  python -m collective_communication_mpi_amd.launch -n 8 python benchmarks/host_trace.py > $OUT/host_trace.jsonl 2> $OUT/host_trace.err || exit $?
for H in 2 4; do
  for B in 256 512 1024 2048 4096; do
    timeout -k 10 120 python benchmarks/qkv_fused_micro.py --H $H --B $B --grid 512 --only img --train 0 --iters 300 \
      >> $OUT/qkv_bsweep.jsonl 2>> $OUT/qkv_bsweep.err || exit $?
  done
done
echo done
