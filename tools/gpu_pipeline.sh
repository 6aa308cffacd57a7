#!/bin/bash
# GPU: wire-to-wire pipelines (tools/bench_pipeline.py) at 4 Mi words, N = 3 and 2,
# then a rocprofv3 kernel trace of the N = 3 run for the per-kernel split.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${TAG:-pipe}"
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 300 python tools/bench_pipeline.py --words 4194304 --parties 3 > "$OUT/pipe_4Mi_3.json" 2> "$OUT/pipe.err" || exit 1
timeout -k 10 300 python tools/bench_pipeline.py --words 4194304 --parties 2 > "$OUT/pipe_4Mi_2.json" 2>> "$OUT/pipe.err" || exit 1
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d "$OUT/prof" -o kt --output-format csv -- python3 tools/bench_pipeline.py --words 4194304 --parties 3 --reps 5 > "$OUT/prof.log" 2>&1 || exit 1
echo done > "$OUT/status.txt"
