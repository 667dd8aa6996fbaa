#!/usr/bin/env bash
# Round 6, last lease: the attention / fold / plan kernel tests and smoke() on the final tree.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
OUT=gpurun_out/${OUT_TAG:-r6_sanity}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_harness_grad.py tests/test_gpu_distributed.py -x -q --timeout 200 --timeout-method thread -k "attn or qkv or fold or plan or harness or patchify" > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 $OUT/smoke.log
exit $rc
