#!/bin/bash
# Run the wire-kernel occupancy sweep (tools/build_wire_occ.sh) on the GPU:
# every variant under its own time limit, the first failure ends the call.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${TAG:-wocc}"
mkdir -p "$OUT"
: > "$OUT/sweep.jsonl"
for rep in 1 2; do
  for b in "$ROOT"/tools/ubench/wocc/u_g*; do
    timeout -k 10 120 "$b" 4194304 20 >> "$OUT/sweep.jsonl" 2>> "$OUT/sweep.err" || { echo "fail $b" >> "$OUT/sweep.err"; exit 1; }
  done
  timeout -k 10 120 "$ROOT/tools/ubench/wocc/u_g5p0" 4194304 20 reg >> "$OUT/sweep.jsonl" 2>> "$OUT/sweep.err" || exit 1
done
echo done >> "$OUT/sweep.err"
