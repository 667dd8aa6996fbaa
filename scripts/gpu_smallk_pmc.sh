#!/usr/bin/env bash
# PMC counters for the small-K (patch embedding) GEMM and the QKV GEMM (counter passes only).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/pmc2
export TMPDIR=/tmp
run() {  # name M N K MODE counters...
  local name=$1; shift; local M=$1 N=$2 K=$3 MODE=$4; shift 4
  timeout -s KILL 60 rocprofv3 --pmc "$@" --output-format csv -d gpurun_out/pmc2/$name -o out -- python3 benchmarks/gemm_one.py $M $N $K $MODE 10 > gpurun_out/pmc2/$name.log 2>&1
}
C1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD"
C2="SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE"
C3="TCC_HIT_sum TCC_MISS_sum TCC_EA0_WRREQ_sum TCC_EA0_RDREQ_sum"
for shp in "sk 32768 768 72 0" "qkv 32768 768 768 1"; do
  set -- $shp
  run ${1}_c1 $2 $3 $4 $5 $C1 && run ${1}_c2 $2 $3 $4 $5 $C2 && run ${1}_c3 $2 $3 $4 $5 $C3 || { echo "pmc run $1 failed rc=$?"; exit 1; }
done
python3 - <<'PY'
import csv, glob, os
for f in sorted(glob.glob("gpurun_out/pmc2/*/out_counter_collection.csv")):
    rows = list(csv.DictReader(open(f)))
    agg = {}
    for r in rows:
        if "gemm" not in r.get("Kernel_Name", ""):
            continue
        agg.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    print(os.path.basename(os.path.dirname(f)), {k: round(sum(v) / len(v)) for k, v in agg.items()})
PY
echo pmc done
