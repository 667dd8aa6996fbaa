set -o pipefail
cd $GRAFT_REPO_ROOT
export CCMPI_TIMEOUT=300 CCMPI_DEVICE_TIMEOUT_S=20 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_harness_grad.py -x -q --timeout 120 --timeout-method thread > gpurun_out/chunks_test.log 2>&1; rc=$?; tail -3 gpurun_out/chunks_test.log; [ $rc -eq 0 ] || exit $rc
for c in 1 2 4 1 2 4; do
  CCMPI_FWD_CHUNKS=$c timeout -k 10 200 python bench.py > gpurun_out/bc$c.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/bc$c.json'));print('chunks $c', d['config']['tp_fwd_step_ms'], d['config']['tp_train_step_ms'])"
done
