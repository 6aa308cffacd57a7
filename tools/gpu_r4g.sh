#!/bin/bash
# Round-4 GPU pass G: smoke, the full GPU suite, the driver's bench line and
# the fused wire kernels' rocprofv3 kernel-trace on the current library.
# Each GPU step has its own time limit; the first failure ends the call.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${TAG:-r4g}"
mkdir -p "$OUT"
cd "$ROOT"
echo "start $(date)" > "$OUT/status.txt"
step() {  # step NAME SECONDS CMD...
  local name=$1 secs=$2
  shift 2
  timeout -k 10 "$secs" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?
  echo "$name rc=$rc $(date +%T)" >> "$OUT/status.txt"
  return $rc
}
run_all() {
  [ -n "$SKIP_SMOKE" ] || step smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()" || return
  [ -n "$SKIP_TESTS" ] || step pytest 900 python3 -u -m pytest ${PYTEST_FILES:-tests} -m gpu -x -v --timeout 300 --timeout-method thread || return
  [ -n "$SKIP_BENCH" ] || step bench_driver 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 || return
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/wire_ktrace" -o k --output-format csv -- python3 "$ROOT/tools/wire_kernels.py") > "$OUT/wire_ktrace.log" 2>&1
  local rc=$?; echo "wire_ktrace rc=$rc $(date +%T)" >> "$OUT/status.txt"; return $rc
}
run_all
rc=$?
echo "end rc=$rc $(date)" >> "$OUT/status.txt"
exit $rc
