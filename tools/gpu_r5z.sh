#!/bin/bash
# Round-5 final check on the committed build: smoke, the full -m gpu suite,
# the driver's default bench command.  Each step under its own limit; the
# first failure ends the call.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${TAG:-r5z}"
mkdir -p "$OUT"
cd "$ROOT"
echo "start $(date)" > "$OUT/status.txt"
step() {
  local name=$1 lim=$2
  shift 2
  timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?; echo "$name rc=$rc $(date +%T)" >> "$OUT/status.txt"; return $rc
}
step smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" &&
step tests 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests &&
step bench 400 python -u bench.py --steps 20 --warmup 5
rc=$?
echo "end rc=$rc $(date)" >> "$OUT/status.txt"
exit $rc
