#!/bin/bash
# GPU tests + host-memory (PCIe-inclusive) rate measurements.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${TAG:-host}"
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 900 python -m pytest tests -m gpu -x -q > "$OUT/pytest_gpu.log" 2>&1 || exit 1
echo tests ok > "$OUT/status.txt"
run() { echo "== $*" >> "$OUT/host.txt"; timeout -k 10 600 python bench.py --mode host "$@" >> "$OUT/host.txt" 2>> "$OUT/host.err"; }
run --words 1048576 --parties 2 --steps 10 --warmup 2 && \
run --words 1048576 --parties 2 --steps 10 --warmup 2 --pin && \
run --words 33554432 --parties 3 --steps 3 --warmup 1 && \
run --words 33554432 --parties 3 --steps 3 --warmup 1 --pin && \
run --words 33554432 --parties 3 --steps 3 --warmup 1 --pin --batch-words 8388608
echo "end rc=$?" >> "$OUT/status.txt"
