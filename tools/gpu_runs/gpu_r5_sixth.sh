#!/usr/bin/env bash
# Round 5, sixth GPU pass: token fc_o kernel with 16-B write-through pushes (no per-workgroup
# release), its tests, plain vs push harness forwards at 2 and 8 shared ranks, and the pair
# ring's sync ablations.
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/${OUT_TAG:-r5_sixth}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  "tests/test_gpu_kernels.py::test_attn_token_fc_o" "tests/test_gpu_distributed.py::test_harness_fc_o_push_equals_plain" \
  > $OUT/pytest.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $OUT/pytest.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error" $OUT/pytest.log | head; exit $rc; }
timeout -k 10 200 python -m collective_communication_mpi_amd.launch -n 2 --timeout 190 python benchmarks/fc_o_forms.py \
  > $OUT/forms2.json 2> $OUT/forms2.err
rc=$?; echo "forms2 rc=$rc"; cat $OUT/forms2.json; [ $rc -ne 0 ] && { tail -20 $OUT/forms2.err; exit $rc; }
GPU_MAX_HW_QUEUES=1 timeout -k 10 300 python -m collective_communication_mpi_amd.launch -n 8 --timeout 290 \
  python benchmarks/fc_o_forms.py > $OUT/forms8.json 2> $OUT/forms8.err
rc=$?; echo "forms8 rc=$rc"; cat $OUT/forms8.json; [ $rc -ne 0 ] && { tail -20 $OUT/forms8.err; exit $rc; }
timeout -k 10 300 python benchmarks/gemm_nobar_ab.py > $OUT/nobar.jsonl 2> $OUT/nobar.err
rc=$?; echo "nobar rc=$rc"; cat $OUT/nobar.jsonl; [ $rc -ne 0 ] && { tail -20 $OUT/nobar.err; exit $rc; }
exit 0
