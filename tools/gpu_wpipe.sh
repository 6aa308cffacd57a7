#!/bin/bash
# The persistent pipelined K_MASK-from-text (k_mask_b64_pipe) against the
# one-tile-per-workgroup kernel, same binary, same box (tools/ubench/ubench_wire_occ.hip).
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$ROOT/gpurun_out/${TAG:-wpipe}"; mkdir -p "$OUT"
for rep in 1 2; do
  for b in u_g5p0 u_g3p0; do
    B="$ROOT/tools/ubench/wocc/$b"
    timeout -k 10 120 "$B" 4194304 20 >> "$OUT/p.jsonl" 2>>"$OUT/p.err" || exit 1
    for w in 2 3 4; do
      timeout -k 10 120 "$B" 4194304 20 pipe $w >> "$OUT/p.jsonl" 2>>"$OUT/p.err" || exit 1
    done
  done
  timeout -k 10 120 "$ROOT/tools/ubench/wocc/u_g5p0" 4194304 20 probe >> "$OUT/p.jsonl" 2>>"$OUT/p.err" || exit 1
done
