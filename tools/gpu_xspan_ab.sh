#!/bin/bash
# GPU: span-form decode A/B (tools/ubench/xv/ubench_xdec_spans_dma{0,1}, built
# with -DAMPH_XDEC_SPAN_DMA=0/1 at commit 2 after c420ec8 (the DMA variant was then removed):
# per-span workgroups vs the persistent LDS-DMA
# double-buffered pass), full-length and mixed texts, alternated; rocprofv3
# kernel traces of both; then the party-session tests and the pipelines.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${TAG:-xspan}"
mkdir -p "$OUT"
cd "$ROOT"
D=tools/ubench/xv
for rep in 1 2; do
  for v in 0 1; do
    for full in 1 0; do
      echo "== dma$v full=$full rep=$rep" >> "$OUT/ab.txt"
      timeout -k 10 60 $D/ubench_xdec_spans_dma$v 20 $full >> "$OUT/ab.txt" 2>&1 || exit 1
    done
  done
done
for v in 0 1; do
  (cd /tmp && TMPDIR=/tmp timeout -k 10 90 rocprofv3 --kernel-trace --stats -T -d "$OUT/prof_dma$v" -o kt --output-format csv -- "$ROOT/$D/ubench_xdec_spans_dma$v" 20 1 > "$OUT/prof_dma$v.log" 2>&1) || exit 1
done
[ -n "$SKIP_PIPE" ] || SKIP_XDEC=1 PYTEST_PATHS="${PYTEST_PATHS:-tests/test_party_session.py}" TAG=${TAG:-xspan}/r3d bash tools/gpu_r3d.sh || exit 1
echo done >> "$OUT/ab.txt"
