#!/bin/bash
# Property-test soak on the GPU box: the hypothesis tests of every kernel
# against the C oracle, in ROUNDS separate runs of EXAMPLES examples each
# (fresh random draws per run; each run is its own time-limited step, so a
# hang ends early and the log grows as the soak goes).
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${TAG:-soak}"
mkdir -p "$OUT"
cd "$ROOT"
LOG="$OUT/soak.log"
: > "$LOG"
for i in $(seq 1 "${ROUNDS:-6}"); do
  echo "round $i $(date)" >> "$LOG"
  AMPH_HYPOTHESIS_EXAMPLES="${EXAMPLES:-300}" timeout -k 10 170 python -m pytest tests/test_hip_props.py \
    -q -p no:cacheprovider >> "$LOG" 2>&1 || { echo "round $i FAILED rc=$?" >> "$LOG"; exit 1; }
done
echo "soak ok" >> "$LOG"
