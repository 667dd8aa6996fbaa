#!/usr/bin/env bash
# Round 5, first GPU pass: the bench's candidate loop under injected failures (fp32 first
# candidate + every bf16 candidate), the 4-rank shared N >= 2 path, then the 1-GPU bench
# (headline, secondaries, sweep, host phase, 8-rank shared dry run).
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/${OUT_TAG:-r5_first}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest -x -v --timeout 400 --timeout-method thread \
  "tests/test_gpu_distributed.py::test_bench_failing_candidates_keep_headline" \
  "tests/test_gpu_distributed.py::test_bench_multi_rank_path_shared_gpu" > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -8 $OUT/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 700 python bench.py --verbose > $OUT/bench1.json 2> $OUT/bench1.err
rc=$?; echo "bench rc=$rc"; cut -c1-600 $OUT/bench1.json; [ $rc -ne 0 ] && { tail -30 $OUT/bench1.err; exit $rc; }
exit 0
