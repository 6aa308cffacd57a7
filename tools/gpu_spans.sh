#!/bin/bash
# GPU: the exchange decode into span form (k_xdec_span) -- harness timing and
# check (tools/ubench/ubench_xdec2, 8 Mi FactorPairs full-length and mixed),
# the party-session and wire GPU tests, and a rocprofv3 kernel trace of the
# harness.  Each step has its own limit; the first failure ends the call.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${TAG:-spans}"
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 120 ./tools/ubench/xv/ubench_xdec_spans 20 1 > "$OUT/xdec_full.txt" 2>&1 || exit 1
timeout -k 10 120 ./tools/ubench/xv/ubench_xdec_spans 20 0 > "$OUT/xdec_mixed.txt" 2>&1 || exit 1
timeout -k 10 600 python3 -u -m pytest tests/test_party_session.py tests/test_wire.py ${PYTEST_EXTRA:-} -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.txt" 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -T -d "$OUT/prof" -o kt --output-format csv -- "$ROOT/tools/ubench/xv/ubench_xdec_spans" 20 1 > "$OUT/prof.log" 2>&1 || exit 1
echo done > "$OUT/status.txt"
