#!/bin/bash
# GPU: pair-order decode A/B -- count pass + compact pass (via0) vs the span
# pass + gather (via1, AMPH_XDEC_VIA_SPANS), full-length and mixed texts,
# alternated, rocprofv3 traces of both; then the exchange / session tests.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${TAG:-via}"
mkdir -p "$OUT"
cd "$ROOT"
D=tools/ubench/xv
for rep in 1 2; do
  for v in 0 1; do
    for full in 1 0; do
      echo "== via$v full=$full rep=$rep" >> "$OUT/ab.txt"
      timeout -k 10 60 $D/ubench_xdec_via$v 20 $full >> "$OUT/ab.txt" 2>&1 || exit 1
    done
  done
done
for v in 0 1; do
  (cd /tmp && TMPDIR=/tmp timeout -k 10 90 rocprofv3 --kernel-trace --stats -T -d "$OUT/prof_via$v" -o kt --output-format csv -- "$ROOT/$D/ubench_xdec_via$v" 20 1 > "$OUT/prof_via$v.log" 2>&1) || exit 1
done
timeout -k 10 600 python3 -u -m pytest ${PYTEST_PATHS:-tests/test_party_session.py tests/test_wire.py} -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.txt" 2>&1 || exit 1
echo done >> "$OUT/ab.txt"
