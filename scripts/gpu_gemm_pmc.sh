#!/usr/bin/env bash
# PMC counters for the GEMM kernels (counter collection only: no tracing domains).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
rocprofv3 -L > gpurun_out/pmc/avail.txt 2>&1 || true
run() {  # name M N K MODE counters...
  local name=$1; shift; local M=$1 N=$2 K=$3 MODE=$4; shift 4
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --pmc "$@" --output-format csv -d gpurun_out/pmc/$name -o out -- python3 benchmarks/gemm_one.py $M $N $K $MODE 10 > gpurun_out/pmc/$name.log 2>&1
}
C1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"
C2="SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM"
for shp in "k256_4096 4096 4096 4096 2" "k128_4096 4096 4096 4096 1" "blas_4096 4096 4096 4096 -1" "k128_qkv 32768 768 768 1" "blas_qkv 32768 768 768 -1"; do
  set -- $shp
  run ${1}_c1 $2 $3 $4 $5 $C1 && run ${1}_c2 $2 $3 $4 $5 $C2 || { echo "pmc run $1 failed rc=$?"; exit 1; }
done
echo pmc done
