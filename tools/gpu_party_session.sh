#!/bin/bash
# GPU: the party-session tests, then the host pipelines (incl. the session) at 4 Mi x 3.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${TAG:-sess}"
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 600 python -u -m pytest tests/test_party_session.py tests/test_jni_core.py tests/test_abi.py -x -v --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { echo "pytest failed" > "$OUT/status.txt"; exit 1; }
timeout -k 10 400 python tools/bench_pipeline_host.py --words 4194304 --parties 3 > "$OUT/host_4Mi_3.json" 2> "$OUT/err.txt" || exit 1
timeout -k 10 400 python tools/bench_pipeline_host.py --words 4194304 --parties 3 --pinned > "$OUT/host_4Mi_3_pinned.json" 2>> "$OUT/err.txt" || exit 1
echo done > "$OUT/status.txt"
