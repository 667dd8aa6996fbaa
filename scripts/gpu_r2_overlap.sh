#!/usr/bin/env bash
# DP and TP overlap measurements + rocprofv3 kernel traces (2 ranks sharing the GPU).
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/r2ov
mkdir -p $OUT
export CCMPI_TIMEOUT=400 CCMPI_DEVICE_TIMEOUT_S=10 TMPDIR=/tmp
for v in "prio-1_b64:--comm-priority -1" "prio0_b64:--comm-priority 0" "prio-1_b16:--comm-priority -1 --blocks 16"; do
  name=${v%%:*}; a=${v#*:}
  timeout -k 10 200 scripts/mpirun -n 2 --timeout 190 python benchmarks/dp_grad_overlap.py --layers 4 --tokens 4096 --verbose $a > $OUT/dp2_$name.json 2> $OUT/dp2_$name.err
  rc=$?; echo "dp overlap $name rc=$rc: $(cat $OUT/dp2_$name.json)"; [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 300 scripts/mpirun -n 2 --timeout 290 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof_dp2 -o rank%pid% -- \
    python benchmarks/dp_grad_overlap.py --layers 4 --tokens 4096 --iters 2 > $OUT/prof_dp2.log 2>&1
rc=$?; echo "prof dp rc=$rc"; [ $rc -ne 0 ] && exit $rc
python scripts/overlap_from_trace.py $OUT/prof_dp2 --compute gemm > $OUT/dp2_trace_overlap.md; cat $OUT/dp2_trace_overlap.md
timeout -k 10 300 scripts/mpirun -n 2 --timeout 290 python benchmarks/tp_overlap.py > $OUT/tp2.json 2> $OUT/tp2.err
rc=$?; echo "tp overlap rc=$rc"; cat $OUT/tp2.json; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 scripts/mpirun -n 2 --timeout 290 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof_tp2 -o rank%pid% -- \
    python benchmarks/tp_overlap.py --steps 10 --chunks 4 > $OUT/prof_tp2.log 2>&1
rc=$?; echo "prof tp rc=$rc"
python scripts/overlap_from_trace.py $OUT/prof_tp2 --compute gemm,attn > $OUT/tp2_trace_overlap.md; cat $OUT/tp2_trace_overlap.md
exit $rc
