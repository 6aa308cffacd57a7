#!/bin/bash
# GPU: full GPU tests, then the host-path probes (batch sizes, pipelines incl. the party session)
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${TAG:-hostpath}"
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { echo "pytest failed" > "$OUT/status.txt"; exit 1; }
timeout -k 10 400 python tools/host_rate_probe.py > "$OUT/probe.jsonl" 2> "$OUT/err.txt" || exit 1
timeout -k 10 400 python tools/bench_pipeline_host.py --words 4194304 --parties 3 > "$OUT/host_4Mi_3.json" 2>> "$OUT/err.txt" || exit 1
timeout -k 10 400 python tools/bench_pipeline_host.py --words 4194304 --parties 3 --pinned > "$OUT/host_4Mi_3_pinned.json" 2>> "$OUT/err.txt" || exit 1
timeout -k 10 300 python bench.py --mode host --steps 5 --warmup 1 > "$OUT/bench_host.json" 2>> "$OUT/err.txt" || exit 1
echo done > "$OUT/status.txt"
