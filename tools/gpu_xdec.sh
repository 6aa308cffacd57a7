#!/bin/bash
# GPU side of the exchange-decode A/B (variants from tools/build_xdec_variants.sh):
# each variant's end-to-end decode time (the harness's own events) on 8 Mi
# FactorPairs, full-length and mixed-length text, then a rocprofv3 kernel-trace
# summary of the same run for the per-kernel split.  Every step has its own limit.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${TAG:-xdec}"
mkdir -p "$OUT"
D="$ROOT/tools/ubench/xv"
cd /tmp && export TMPDIR=/tmp
for rep in 1 2; do
  for v in ${VARIANTS:-base noparse noconv}; do
    for full in 1 0; do
      echo "== $v full=$full rep=$rep" >> "$OUT/times.txt"
      timeout -k 10 60 "$D/ubench_xdec2_$v" 20 $full >> "$OUT/times.txt" 2>&1 || { echo "FAIL $v" >> "$OUT/times.txt"; exit 1; }
    done
  done
done
for v in ${VARIANTS:-base noparse noconv}; do
  timeout -k 10 90 rocprofv3 --kernel-trace --stats -T -d "$OUT/prof_$v" -o kt --output-format csv -- "$D/ubench_xdec2_$v" 20 1 > "$OUT/prof_$v.log" 2>&1 || exit 1
done
echo done >> "$OUT/times.txt"
