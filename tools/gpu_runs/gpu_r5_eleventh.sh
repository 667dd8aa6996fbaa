#!/usr/bin/env bash
# Round 5, eleventh GPU pass: fused patchify + in-kernel token mean in the fused QKV kernel,
# the fp32-MFMA weight fold, hardware bf16 conversion -- the kernels' numerics tests, the
# harness tests, then the fused-on/off harness profile.
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/r5_eleventh
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_kernels.py -k "attn_qkv_fused or attn_token_fc_o or fold_emb" > $OUT/tests_k.log 2>&1
rc=$?; tail -3 $OUT/tests_k.log; [ $rc -ne 0 ] && { grep -E "FAILED|^E " $OUT/tests_k.log | head -30; exit $rc; }
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_distributed.py -k "harness" > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -ne 0 ] && { grep -E "FAILED|^E " $OUT/tests.log | head -20; exit $rc; }
OUT_TAG=r5_eleventh bash tools/gpu_runs/gpu_r5_ninth.sh
