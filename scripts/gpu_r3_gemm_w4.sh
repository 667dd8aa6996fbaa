#!/usr/bin/env bash
# Four-wave 256x256 GEMM: correctness + A/B against the 8-wave kernel and hipBLASLt,
# then PMC counters (MFMA busy, waits, LDS conflicts) on the gate|up shape.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/r3_gemm_w4${TAG:+_$TAG}
mkdir -p $OUT
timeout -k 10 400 python3 benchmarks/gemm_bench.py --rounds 3 --w4 ${W4:-0:8,1:8,3:8} \
  --shapes ${SHAPES:-4096x4096x14336,4096x28672x4096,4096x4096x28672,4096x14336x4096,8192x8192x8192} \
  > $OUT/gemm_bench.txt 2>&1 || { echo "gemm_bench failed"; tail -20 $OUT/gemm_bench.txt; exit 1; }
cat $OUT/gemm_bench.txt
[ -n "$NOPMC" ] && exit 0
C1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"
C2="SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS"
for c in C1 C2; do
  timeout -s KILL 90 rocprofv3 --kernel-trace --stats --pmc ${!c} --output-format csv -d $OUT/pmc_w4_$c -o out -- \
    python3 benchmarks/gemm_one.py 4096 28672 4096 5 10 > $OUT/pmc_w4_$c.log 2>&1 || { echo "pmc $c failed"; exit 1; }
done
echo w4 done
