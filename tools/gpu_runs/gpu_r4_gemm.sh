#!/usr/bin/env bash
# Round 4 GEMM pass: LDS-ring NT phase placements vs hipBLASLt on the Llama MLP shapes, then
# rocprofv3 PMC passes (own ring kernel, default and PS 1 placement, and hipBLASLt) on
# 4096x28672x4096.
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/${OUT_TAG:-r4_gemm}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python benchmarks/gemm_ps_ab.py --scheds ${SCHEDS:-8,9,1032,1033} > $OUT/ps_ab.jsonl 2> $OUT/ps_ab.err
rc=$?; echo "ps_ab rc=$rc"; cat $OUT/ps_ab.jsonl; [ $rc -ne 0 ] && { tail -20 $OUT/ps_ab.err; exit $rc; }
[ "${PMC:-1}" = 0 ] && exit 0
read M N K <<< "$(echo ${SHAPE:-4096x28672x4096} | tr x ' ')"
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_SALU SQ_ACTIVE_INST_VALU"
for v in ${PMC_VARIANTS:-"-1:0" "0:8" "0:1032"}; do
  mode=${v%%:*}; rs=${v##*:}; tag=m${mode}_s${rs}
  for pass in P1 P2; do
    CCMPI_RING_SCHED=$rs timeout -s KILL 90 rocprofv3 --pmc ${!pass} --output-format csv -d $OUT/pmc_${tag}_$pass -o out -- \
      python3 benchmarks/gemm_one.py $M $N $K $mode 10 > $OUT/pmc_${tag}_$pass.log 2>&1 || { echo "pmc $tag $pass failed"; tail -5 $OUT/pmc_${tag}_$pass.log; exit 1; }
    echo "pmc $tag $pass ok"
  done
done
dirs=""
for v in ${PMC_VARIANTS:-"-1:0" "0:8" "0:1032"}; do dirs="$dirs $OUT/pmc_m${v%%:*}_s${v##*:}_P1 $OUT/pmc_m${v%%:*}_s${v##*:}_P2"; done
python3 scripts/pmc_table.py $dirs > $OUT/pmc_table.md 2>&1
cat $OUT/pmc_table.md
