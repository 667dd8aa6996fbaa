#!/usr/bin/env bash
# Round 6: instruction / scalar cache counters of the fused attention kernel after the lean instantiations (one rocprofv3 --pmc
# pass of SQ counters, kernel trace only, over the micro at H = 2 / 4).
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
OUT=gpurun_out/${OUT_TAG:-r6_icache_lean}
mkdir -p $OUT
for H in 2 4; do
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_IFETCH SQC_ICACHE_MISSES SQC_ICACHE_HITS SQC_DCACHE_MISSES SQC_DCACHE_HITS \
    --kernel-include-regex qkv_attn16 --output-format csv -d $OUT/h$H -o pmc -- \
    python3 benchmarks/qkv_fused_micro.py --H $H --B 2048 --grid 256 --train 0 --iters 20 --nolse --only img > $OUT/h$H.log 2>&1 || exit $?
done
echo done
