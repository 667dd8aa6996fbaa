#!/usr/bin/env bash
# Round 6: where the TP = 1 Llama-3-8B MLP block's forward + backward time goes (rocprofv3 kernel
# statistics), and the forward / backward GEMM shapes against hipBLASLt (interleaved A/B).
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
OUT=gpurun_out/${OUT_TAG:-r6_gemm}
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o mlp_%pid% -- \
  python3 benchmarks/tp_mlp.py --iters 10 > $OUT/tp_mlp.json 2> $OUT/tp_mlp.err
rc=$?; echo "mlp prof rc=$rc"; cat $OUT/tp_mlp.json | cut -c1-300; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 benchmarks/tp_mlp.py --iters 10 > $OUT/tp_mlp_noprof.json 2>&1 || exit $?
timeout -k 10 300 python3 benchmarks/gemm_bench.py --rounds 5 --shapes 4096x28672x4096,4096x4096x14336,4096x14336x4096 \
  > $OUT/gemm_fwd.jsonl 2>&1 || exit $?
timeout -k 10 300 python3 benchmarks/gemm_ring_bench.py --iters 20 > $OUT/gemm_bwd.jsonl 2>&1 || exit $?
echo done
