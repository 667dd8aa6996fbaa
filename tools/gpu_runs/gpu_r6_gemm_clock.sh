#!/usr/bin/env bash
# Round 6: shader clock during the pair-ring GEMM and hipBLASLt on the same forward shape
# (GRBM_GUI_ACTIVE cycles over the kernel's duration), plus MFMA busy and LDS instruction counts
# -- one rocprofv3 --pmc pass each, kernel trace only.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
OUT=gpurun_out/${OUT_TAG:-r6_gemm_clock}
mkdir -p $OUT
for MODE in 0 -1; do
  timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES \
    --output-format csv -d $OUT/m$MODE -o pmc -- python3 benchmarks/gemm_one.py 4096 28672 4096 $MODE 20 > $OUT/m$MODE.log 2>&1 || exit $?
done
echo done
