#!/bin/bash
# GPU tests + party-kernel bench at 16 Mi and 1 Mi words, N = 2 and 3.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${TAG:-party}"
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > "$OUT/pytest_gpu.log" 2>&1 && echo "pytest ok" >> "$OUT/status.txt" || exit 1
for cfg in "--words 16777216 --parties 2" "--words 16777216 --parties 3" "--words 1048576 --parties 2"; do
  timeout -k 10 300 python tools/bench_party.py $cfg >> "$OUT/party.jsonl" 2>> "$OUT/party.err" || exit 1
done
echo "party ok" >> "$OUT/status.txt"
