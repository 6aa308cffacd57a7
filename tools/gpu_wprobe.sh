#!/bin/bash
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$ROOT/gpurun_out/wprobe"; mkdir -p "$OUT"
B="$ROOT/tools/ubench/wocc/u_g5p0"
for i in 1 2 3; do
  timeout -k 10 120 "$B" 4194304 20 probe >> "$OUT/p.jsonl" 2>>"$OUT/p.err" || exit 1
  timeout -k 10 120 "$B" 4194304 20 >> "$OUT/p.jsonl" 2>>"$OUT/p.err" || exit 1
done
