#!/usr/bin/env bash
# Pair-slot ring: even vs front-loaded DMA placement, long K on the ring (bit 15), and the
# TP=1 Llama MLP block with each ring schedule as the auto default (CCMPI_RING_SCHED).
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
OUT=gpurun_out/r4_pair2
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_kernels.py \
  -k "pair" > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python benchmarks/gemm_ps_ab.py --scheds 8,16392,65544,49160,98312 > $OUT/ps_ab.jsonl 2> $OUT/ps_ab.err
rc=$?; echo "ps_ab rc=$rc"; cat $OUT/ps_ab.jsonl; [ $rc -ne 0 ] && { tail -20 $OUT/ps_ab.err; exit $rc; }
for rs in 8 16392 65544 98312; do
  CCMPI_RING_SCHED=$rs timeout -k 10 200 python benchmarks/tp_mlp.py > $OUT/tp_mlp_$rs.json 2> $OUT/tp_mlp_$rs.err
  rc=$?; echo "tp_mlp sched $rs rc=$rc: $(cut -c1-400 $OUT/tp_mlp_$rs.json)"; [ $rc -ne 0 ] && exit $rc
done
exit 0
