#!/usr/bin/env bash
# Round 5, fourth GPU pass: the pair ring's K-major A form (TA / TA+TB) numerics, the MLP
# backward routes incl. the no-transpose one, the ring / RHD after the one-launch fix (2 and 8
# shared ranks), then the whole GPU suite.
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/${OUT_TAG:-r5_fourth}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  "tests/test_gpu_kernels.py::test_gemm_ring_layouts" "tests/test_gpu_kernels.py::test_gemm_ring_kmajor_routes" \
  > $OUT/pytest_ring.log 2>&1
rc=$?; echo "ring gemm tests rc=$rc"; tail -4 $OUT/pytest_ring.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error" $OUT/pytest_ring.log | head; exit $rc; }
timeout -k 10 300 python benchmarks/mlp_bwd_routes.py > $OUT/mlp_bwd_routes.jsonl 2> $OUT/mlp_bwd_routes.err
rc=$?; echo "routes rc=$rc"; cat $OUT/mlp_bwd_routes.jsonl; [ $rc -ne 0 ] && { tail -20 $OUT/mlp_bwd_routes.err; exit $rc; }
for n in 2 8; do
  timeout -k 10 300 python -m collective_communication_mpi_amd.launch -n $n --timeout 280 python benchmarks/coll_sweep.py \
    --ops allreduce --algos fanout,ring,rhd --min-bytes 268435456 --max-mb 1024 --iters 5 \
    --out $OUT/ring$n.jsonl > $OUT/ring$n.log 2>&1
  rc=$?; echo "ring$n rc=$rc"; [ $rc -ne 0 ] && { tail -20 $OUT/ring$n.log; exit $rc; }
  python scripts/coll_table.py $OUT/ring$n.jsonl || true
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "suite rc=$rc"; tail -3 $OUT/pytest_gpu.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error" $OUT/pytest_gpu.log | head; exit $rc; }
exit 0
