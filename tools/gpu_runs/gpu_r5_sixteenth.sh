#!/usr/bin/env bash
# Round 5, sixteenth GPU pass: PMC counters of the fused QKV kernel (rows mode, inference,
# z rows, grid 512), one counter group per run.
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/r5_sixteenth
mkdir -p $OUT
export TMPDIR=/tmp
i=0
for pmc in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
           "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM SQ_LDS_BANK_CONFLICT SQ_INSTS_MFMA" \
           "SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_FLAT SQ_INSTS_BRANCH SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SMEM"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $pmc --output-format csv -d $OUT/pmc$i -o run -- \
    python3 benchmarks/qkv_fused_micro.py --iters 20 --only rows --grid 512 --train 0 > $OUT/pmc$i.log 2>&1
  rc=$?; echo "pmc$i rc=$rc"; [ $rc -ne 0 ] && { tail -5 $OUT/pmc$i.log; exit 0; }
done
exit 0
