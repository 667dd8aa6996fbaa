#!/usr/bin/env bash
# Round 5, second GPU pass: the new kernel / harness / DDP / scratch tests first, then the
# whole GPU suite, then the 1-GPU bench with its 8-rank shared dry run.
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/${OUT_TAG:-r5_second}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  "tests/test_gpu_kernels.py::test_attn_token_fc_o" \
  "tests/test_gpu_distributed.py::test_harness_fc_o_push_equals_plain" \
  "tests/test_gpu_distributed.py::test_harness_token_push_matches_single_rank" \
  "tests/test_gpu_distributed.py::test_tp_scratch_reused_across_token_counts" \
  "tests/test_gpu_distributed.py::test_llama_ddp_gradient_sinks_gpu" > $OUT/pytest_new.log 2>&1
rc=$?; echo "new tests rc=$rc"; tail -12 $OUT/pytest_new.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "suite rc=$rc"; tail -3 $OUT/pytest_gpu.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error" $OUT/pytest_gpu.log | head; exit $rc; }
exit 0
