#!/usr/bin/env bash
# Why does the DP-overlap measurement time out with ranks sharing the GPU?  Small variants, short limits.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/r2ovx
mkdir -p $OUT
export CCMPI_TIMEOUT=100 CCMPI_DEVICE_TIMEOUT_S=5 TMPDIR=/tmp
run() {  # name, env, args
  local name=$1; shift
  env "$@" timeout -k 10 90 scripts/mpirun -n 2 --timeout 80 python benchmarks/dp_grad_overlap.py --verbose --iters 2 $DPARGS > $OUT/$name.json 2> $OUT/$name.err
  echo "$name rc=$?: $(cat $OUT/$name.json) | $(grep -v amdgpu.ids $OUT/$name.err | grep -E 'dp_overlap|watchdog' | head -4 | tr '\n' ' ')"
}
DPARGS="--layers 1 --tokens 1024" run a_l1_t1024 X=1
DPARGS="--layers 4 --tokens 1024" run b_l4_t1024 X=1
DPARGS="--layers 1 --tokens 4096" run c_l1_t4096 X=1
DPARGS="--layers 4 --tokens 4096 --comm-priority 0" run d_l4_prio0 X=1
DPARGS="--layers 4 --tokens 4096" run e_l4_hwq2 GPU_MAX_HW_QUEUES=2
DPARGS="--layers 4 --tokens 4096" run f_l4_blocks64 CCMPI_MAX_BLOCKS=64
DPARGS="--layers 4 --tokens 4096 --algo ring" run g_l4_ring X=1
exit 0
