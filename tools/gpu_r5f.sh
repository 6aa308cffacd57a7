#!/bin/bash
# Round-5 closing evidence: smoke, then tools/gpu_prof.sh (the default bench
# line, rocprofv3 --kernel-trace --stats of the same command (full template
# names: the host phase's 3-party batch launches are listed apart), FETCH_SIZE and
# WRITE_SIZE passes).
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${TAG:-r5f}"
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1 || exit $?
TAG="${TAG:-r5f}" bash tools/gpu_prof.sh
