#!/bin/bash
# Full GPU pass: smoke, GPU tests, bench (C2), rocprofv3 stats, PMC passes.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${TAG:-all}"
mkdir -p "$OUT"
cd "$ROOT"
echo "start $(date)" > "$OUT/status.txt"
timeout -k 10 600 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 && echo "smoke ok" >> "$OUT/status.txt" && \
timeout -k 10 1200 python -m pytest tests -m gpu -x -q > "$OUT/pytest_gpu.log" 2>&1 && echo "pytest ok" >> "$OUT/status.txt" && \
TAG="${TAG:-all}" bash tools/gpu_prof.sh
rc=$?
echo "end rc=$rc $(date)" >> "$OUT/status.txt"
exit $rc
