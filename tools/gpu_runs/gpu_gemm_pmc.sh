#!/usr/bin/env bash
# GEMM counters: rocprofv3 PMC passes (one run per pass) of gemm_one.py for each
# MODE in $MODES (-1 = hipBLASLt, 5 = four-wave kernel with CCMPI_W4_SCHED) on $SHAPE.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
OUT=gpurun_out/gemm_pmc${TAG:+_$TAG}
mkdir -p $OUT
read M N K <<< "$(echo ${SHAPE:-4096x28672x4096} | tr x ' ')"
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_SALU SQ_ACTIVE_INST_VALU"
for mode in ${MODES:--1 5}; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_m$mode -o out -- \
    python3 benchmarks/gemm_one.py $M $N $K $mode 20 > $OUT/trace_m$mode.log 2>&1 || { echo "trace $mode failed"; exit 1; }
  for pass in P1 P2; do
    timeout -s KILL 90 rocprofv3 --pmc ${!pass} --output-format csv -d $OUT/pmc_m${mode}_$pass -o out -- \
      python3 benchmarks/gemm_one.py $M $N $K $mode 10 > $OUT/pmc_m${mode}_$pass.log 2>&1 || { echo "pmc $mode $pass failed"; exit 1; }
  done
done
echo gemm pmc done
