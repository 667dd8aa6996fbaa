#!/usr/bin/env bash
# Round 6, first lease: sysfs placement prediction vs the runtime's device (placement_probe),
# the N = 1 bench with the GPU-local binding, and the shared-GPU dry run A/B over
# CCMPI_DRYRUN_BIND = gpu | l3 | none (316.6 -> 305.5 GB/s).
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
OUT=gpurun_out/${OUT_TAG:-r6_first}
mkdir -p $OUT
timeout -k 10 180 python benchmarks/placement_probe.py > $OUT/probe.json 2> $OUT/probe.err &&
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_gpu.json 2> $OUT/bench_gpu.err &&
for b in l3 none gpu; do
  CCMPI_DRYRUN_BIND=$b timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --mlp-tokens 0 \
    --host-ranks 0 > $OUT/bench_dry_$b.json 2> $OUT/bench_dry_$b.err || exit $?
done
python3 - <<PY || true
import json
for f in ["bench_gpu", "bench_dry_l3", "bench_dry_none", "bench_dry_gpu"]:
    d = json.loads(open("$OUT/%s.json" % f).read().strip().splitlines()[-1]); c = d["config"]; s = c.get("shared_gpu_dry_run", {})
    print(f, d["value"], c.get("tp_fwd_step_ms"), "dry:", s.get("binding"), s.get("value"), s.get("tp_fwd_step_ms"),
          s.get("tp_train_step_ms"), (s.get("harness") or {}).get("fc_o_variants", {}).get("token_push_fwd_timed"))
PY
