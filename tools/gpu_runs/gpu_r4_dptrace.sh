#!/usr/bin/env bash
# Kernel trace of the config-5 DDP step (4 Llama-3-8B-shaped layers, 2 ranks sharing the GPU,
# ring GEMMs kept on): bucket all-reduce kernels concurrent with the backward GEMMs.
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/r4_dptrace
mkdir -p $OUT
export CCMPI_DEVICE_TIMEOUT_S=60 TMPDIR=/tmp CCMPI_SHARED_RING=1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace -o run -- \
  python -m collective_communication_mpi_amd.launch -n 2 --timeout 280 python benchmarks/llama_ddp.py --layers 4 --blocks 32 \
  > $OUT/trace.json 2> $OUT/progress.log || { echo "trace rc=$?"; tail -20 $OUT/progress.log; exit 1; }
cat $OUT/trace.json
python3 scripts/overlap_from_trace.py $OUT/trace --comm k_allreduce --compute gemm > $OUT/overlap.md 2>&1
cat $OUT/overlap.md | head -30
