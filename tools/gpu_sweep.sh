#!/bin/bash
# Block-size sweep of the product kernels through bench.py (device-resident).
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${TAG:-sweep}"
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 900 python -m pytest tests -m gpu -x -q > "$OUT/pytest_gpu.log" 2>&1 || exit 1
for cfg in "--words 1048576 --parties 2" "--words 16777216 --parties 3"; do
  for b in 128 256 512 1024; do
    echo "== AMPH_BLOCK=$b $cfg" >> "$OUT/sweep.txt"
    AMPH_BLOCK=$b timeout -k 10 300 python bench.py --no-cpu-baseline --steps 100 $cfg >> "$OUT/sweep.txt" 2>> "$OUT/sweep.err" || exit 1
  done
done
