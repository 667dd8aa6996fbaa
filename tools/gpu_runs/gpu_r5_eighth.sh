#!/usr/bin/env bash
# Round 5, eighth GPU pass: the fused QKV + attention + token fc_o kernel -- numerics, the
# harness runs against the single-rank reference (token mode, plain and push), push == plain,
# then the harness forward timings (N = 1 bench harness phase and the 2/8-rank forms).
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/${OUT_TAG:-r5_eighth}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  "tests/test_gpu_kernels.py::test_attn_qkv_fused" "tests/test_gpu_kernels.py::test_attn_token_fc_o" \
  "tests/test_gpu_distributed.py::test_harness_fc_o_push_equals_plain" \
  "tests/test_gpu_distributed.py::test_harness_token_push_matches_single_rank" \
  "tests/test_gpu_distributed.py::test_harness_matches_single_rank" \
  "tests/test_gpu_distributed.py::test_harness_checkpoint_resume" > $OUT/pytest.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $OUT/pytest.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" $OUT/pytest.log | head -20; exit $rc; }
timeout -k 10 300 python bench.py --no-secondary --shared-dry-run 0 --host-ranks 0 > $OUT/bench1.json 2> $OUT/bench1.err
rc=$?; echo "bench rc=$rc"; python3 -c "
import json; d=json.loads(open('$OUT/bench1.json').read().strip().splitlines()[-1]); c=d['config']
print('tp_fwd', c.get('tp_fwd_step_ms'), 'train', c.get('tp_train_step_ms'))"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -m collective_communication_mpi_amd.launch -n 2 --timeout 190 python benchmarks/fc_o_forms.py \
  > $OUT/forms2.json 2> $OUT/forms2.err
rc=$?; echo "forms2 rc=$rc"; cat $OUT/forms2.json; [ $rc -ne 0 ] && { tail -20 $OUT/forms2.err; exit $rc; }
GPU_MAX_HW_QUEUES=1 timeout -k 10 300 python -m collective_communication_mpi_amd.launch -n 8 --timeout 290 \
  python benchmarks/fc_o_forms.py > $OUT/forms8.json 2> $OUT/forms8.err
rc=$?; echo "forms8 rc=$rc"; cat $OUT/forms8.json; [ $rc -ne 0 ] && { tail -20 $OUT/forms8.err; exit $rc; }
exit 0
