#!/usr/bin/env bash
# Per-token fc_o: gradient tests, DP x TP equivalence, train-step kernel stats, bench line.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/token
rm -rf $OUT; mkdir -p $OUT
export TMPDIR=/tmp CCMPI_DEVICE_TIMEOUT_S=20
timeout -k 10 500 python -u -m pytest tests/test_gpu_harness_grad.py "tests/test_gpu_distributed.py::test_harness_matches_single_rank" -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" $OUT/pytest.log | head -20; exit $rc; }
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o out -- python3 benchmarks/harness_steps.py --mode train --fc-o-mode token --steps 20 > $OUT/prof.log 2>&1 || { echo "prof failed"; exit 1; }
timeout -k 10 300 python bench.py --shared-dry-run 0 > $OUT/n1.json 2> $OUT/n1.err && echo n1 ok || exit 1
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29502 bench.py --gpus 2 --steps 10 --warmup 3 --dp-layers 0 > $OUT/n2.json 2> $OUT/n2.err && echo n2 ok
