#!/usr/bin/env bash
# Round 5, thirteenth GPU pass: the fused QKV kernel in isolation (modes x persistent grid,
# TP = 1 and TP = 2 head counts), then PMC counter passes on the image-mode kernel.
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/r5_thirteenth
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 python3 benchmarks/qkv_fused_micro.py --H 4 > $OUT/micro_h4.jsonl 2> $OUT/micro_h4.err
rc=$?; echo "micro h4 rc=$rc"; [ $rc -ne 0 ] && { tail -20 $OUT/micro_h4.err; exit $rc; }
timeout -k 10 200 python3 benchmarks/qkv_fused_micro.py --H 2 > $OUT/micro_h2.jsonl 2> $OUT/micro_h2.err
rc=$?; echo "micro h2 rc=$rc"; [ $rc -ne 0 ] && { tail -20 $OUT/micro_h2.err; exit $rc; }
i=0
for pmc in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
           "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM SQ_LDS_BANK_CONFLICT SQ_INSTS_MFMA"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $pmc --output-format csv -d $OUT/pmc$i -o run -- \
    python3 benchmarks/qkv_fused_micro.py --iters 20 --only img > $OUT/pmc$i.log 2>&1
  rc=$?; echo "pmc$i rc=$rc"; [ $rc -ne 0 ] && { tail -5 $OUT/pmc$i.log; exit 0; }
done
exit 0
