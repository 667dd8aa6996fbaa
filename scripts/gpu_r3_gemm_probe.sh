#!/usr/bin/env bash
# Round 3 GEMM probe: hipBLASLt kernel names/times and PMC counters against our
# 256x256 kernel on the four Llama-3-8B MLP shapes (M N K).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/r3_gemm_probe
mkdir -p $OUT
SHAPES=${SHAPES:-"4096,4096,14336 4096,28672,4096 4096,4096,28672 4096,14336,4096"}
for s in $SHAPES; do
  IFS=, read M N K <<< "$s"
  for mode in -1 2; do
    timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_${M}x${N}x${K}_m$mode -o out -- \
      python3 benchmarks/gemm_one.py $M $N $K $mode 20 > $OUT/trace_${M}x${N}x${K}_m$mode.log 2>&1 || { echo "trace $s $mode failed"; exit 1; }
  done
done
C1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"
C2="SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS"
for mode in -1 2; do
  for c in C1 C2; do
    timeout -s KILL 90 rocprofv3 --kernel-trace --stats --pmc ${!c} --output-format csv -d $OUT/pmc_m${mode}_$c -o out -- \
      python3 benchmarks/gemm_one.py 4096 28672 4096 $mode 10 > $OUT/pmc_m${mode}_$c.log 2>&1 || { echo "pmc $mode $c failed"; exit 1; }
  done
done
timeout -k 10 300 python3 benchmarks/gemm_bench.py --rounds 3 --shapes 4096x4096x14336,4096x28672x4096,4096x4096x28672,4096x14336x4096 > $OUT/gemm_bench.txt 2>&1 || echo "gemm_bench failed"
echo probe done
