#!/bin/bash
# GPU: host-memory wire-to-wire pipelines (tools/bench_pipeline_host.py) at
# 4 Mi words x 3 parties, pageable and page-locked, and 1 Mi x 2.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${TAG:-pipeh}"
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 400 python tools/bench_pipeline_host.py --words 4194304 --parties 3 > "$OUT/host_4Mi_3.json" 2> "$OUT/err.txt" || exit 1
timeout -k 10 400 python tools/bench_pipeline_host.py --words 4194304 --parties 3 --pinned > "$OUT/host_4Mi_3_pinned.json" 2>> "$OUT/err.txt" || exit 1
timeout -k 10 300 python tools/bench_pipeline_host.py --words 1048576 --parties 2 > "$OUT/host_1Mi_2.json" 2>> "$OUT/err.txt" || exit 1
echo done > "$OUT/status.txt"
