#!/usr/bin/env bash
# Round 5: new tests, MLP backward routes + ring sweep, then the whole GPU suite.
set -o pipefail
cd "$(dirname "$0")/../.."
export OUT_TAG_BASE=${OUT_TAG_BASE:-r5}
OUT_TAG=${OUT_TAG_BASE}_third bash tools/gpu_runs/gpu_r5_third.sh || exit $?
OUT_TAG=${OUT_TAG_BASE}_second bash tools/gpu_runs/gpu_r5_second.sh
