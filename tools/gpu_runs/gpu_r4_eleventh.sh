#!/usr/bin/env bash
# TP=2 Llama MLP on the shared GPU with the ring GEMMs kept on (CCMPI_SHARED_RING=1: every
# collective within half the CUs): row-parallel modes side by side; then config 5 (2 layers
# and the full model) on the new backward path.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp CCMPI_DEVICE_TIMEOUT_S=60
OUT=gpurun_out/r4_eleven
mkdir -p $OUT
L="python -m collective_communication_mpi_amd.launch -n 2 --timeout 280"
for c in 1 0; do
  CCMPI_TP_BWD_CONCURRENT=$c timeout -k 10 200 python benchmarks/tp_mlp.py > $OUT/tp1_conc$c.json 2> $OUT/tp1_conc$c.err
  rc=$?; echo "tp1 concurrent=$c rc=$rc: $(cut -c1-330 $OUT/tp1_conc$c.json)"; [ $rc -ne 0 ] && exit $rc
done
CCMPI_SHARED_RING=1 timeout -k 10 300 $L python benchmarks/tp_mlp.py --variants > $OUT/tp2_ring.json 2> $OUT/tp2_ring.err
rc=$?; echo "tp2 shared-ring rc=$rc: $(cut -c1-600 $OUT/tp2_ring.json)"; [ $rc -ne 0 ] && { tail -5 $OUT/tp2_ring.err; exit $rc; }
timeout -k 10 300 $L python benchmarks/tp_mlp.py --variants > $OUT/tp2_noring.json 2> $OUT/tp2_noring.err
rc=$?; echo "tp2 rc=$rc: $(cut -c1-600 $OUT/tp2_noring.json)"; [ $rc -ne 0 ] && { tail -5 $OUT/tp2_noring.err; exit $rc; }
CCMPI_SHARED_RING=1 timeout -k 10 560 $L python benchmarks/llama_ddp.py --verbose --blocks 32,64 > $OUT/dp_full.json 2> $OUT/dp_full.err
rc=$?; echo "dp full rc=$rc: $(cut -c1-700 $OUT/dp_full.json)"; exit $rc
