#!/usr/bin/env bash
# Round 5, tenth GPU pass: the register-resident fused QKV kernel -- its numerics tests and the
# harness tests that run it, then the ninth pass's fused-on/off harness profile.
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/r5_tenth
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_kernels.py -k "attn_qkv_fused or attn_token_fc_o" > $OUT/tests_k.log 2>&1
rc=$?; tail -3 $OUT/tests_k.log; [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
CCMPI_FUSE_QKV=${FUSE:-1} timeout -k 10 600 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_distributed.py -k "harness" > $OUT/tests.log 2>&1
rc=$?; tail -5 $OUT/tests.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error|error" $OUT/tests.log | head -20; exit $rc; }
[ -n "$NOPROF" ] && exit 0
OUT_TAG=r5_tenth bash tools/gpu_runs/gpu_r5_ninth.sh
