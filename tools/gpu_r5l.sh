#!/bin/bash
# Round-5 LDS-table wire decode on the product library: the wire / codec GPU
# tests, then tools/wire_kernels.py (4 Mi words x 3 parties, 30 reps) under
# rocprofv3 --kernel-trace --stats (sustained averages over 31 launches).
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${TAG:-r5l}"
mkdir -p "$OUT"
cd "$ROOT"
echo "start $(date)" > "$OUT/status.txt"
timeout -k 10 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu ${TESTS:-tests/test_wire.py tests/test_wire_fused.py} > "$OUT/tests.log" 2>&1
rc=$?; echo "tests rc=$rc $(date +%T)" >> "$OUT/status.txt"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 tools/wire_kernels.py --reps 30 > "$OUT/wire.json" 2> "$OUT/wire.err"
rc=$?; echo "wire rc=$rc $(date +%T)" >> "$OUT/status.txt"
[ $rc -ne 0 ] && exit $rc
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/ktrace" -o k --output-format csv -- python3 "$ROOT/tools/wire_kernels.py" --reps 30) > "$OUT/ktrace.log" 2>&1
rc=$?; echo "ktrace rc=$rc $(date +%T)" >> "$OUT/status.txt"
echo "end rc=$rc $(date)" >> "$OUT/status.txt"
exit $rc
