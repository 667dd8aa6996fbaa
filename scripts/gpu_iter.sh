#!/usr/bin/env bash
# Iteration run: selected GPU tests (PYTEST_K), 1-GPU bench, harness kernel stats.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export CCMPI_TIMEOUT=300 CCMPI_DEVICE_TIMEOUT_S=20 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -k "${PYTEST_K:-harness or patchify or distributed}" -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_iter.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -12 gpurun_out/pytest_iter.log; [ $rc -ne 0 ] && exit $rc
[ -n "${SKIP_BENCH:-}" ] && exit 0
timeout -k 10 300 python bench.py --verbose > gpurun_out/bench1.json 2> gpurun_out/bench1.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench1.json; [ $rc -ne 0 ] && exit $rc
rm -rf gpurun_out/hprof; mkdir -p gpurun_out/hprof
for m in fwd train; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/hprof/$m -o out -- python3 benchmarks/harness_steps.py --mode $m --steps 20 > gpurun_out/hprof/$m.log 2>&1 || { echo "$m prof failed"; exit 1; }
done
echo prof ok
