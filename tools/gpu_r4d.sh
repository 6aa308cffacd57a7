#!/bin/bash
# Round-4 GPU pass D: does the field layout in HBM move K_MASK / K_RV at C4?
# (rows 2^26 words apart vs padded rows); each run under its own limit.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${TAG:-r4d}"
mkdir -p "$OUT"
cd "$ROOT"
for rep in 1 2; do
  for pad in 0 4099 65557 1048583; do
    timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 200 --warmup 20 --pad-words $pad >> "$OUT/pad.jsonl" 2>> "$OUT/pad.err" || exit 1
  done
done
