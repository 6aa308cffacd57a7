#!/bin/bash
# Round-3 session-2 GPU pass: the full GPU suite, the decode harness (span form
# vs pair order), the wire-to-wire pipelines (per-call and device-mode session)
# and a rocprofv3 kernel trace of the N = 3 pipeline.  Every step has its own
# limit; the first failure ends the call.  Logs in gpurun_out/$TAG.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${TAG:-r3d}"
mkdir -p "$OUT"
cd "$ROOT"
step() {  # step NAME SECONDS CMD...
  local name=$1 secs=$2
  shift 2
  timeout -k 10 "$secs" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?
  echo "$name rc=$rc $(date +%T)" >> "$OUT/status.txt"
  return $rc
}
run_all() {
  [ -n "$SKIP_TESTS" ] || step pytest 900 python3 -u -m pytest ${PYTEST_PATHS:-tests} -m gpu -x -q --timeout 300 --timeout-method thread || return
  [ -n "$SKIP_XDEC" ] || step xdec_full 120 ./tools/ubench/xv/ubench_xdec_spans 20 1 || return
  step pipe3 300 python3 tools/bench_pipeline.py --words 4194304 --parties 3 || return
  step pipe2 300 python3 tools/bench_pipeline.py --words 4194304 --parties 2 || return
  [ -n "$SKIP_PROF" ] || (cd /tmp && TMPDIR=/tmp timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d "$OUT/prof" -o kt --output-format csv -- python3 "$ROOT/tools/bench_pipeline.py" --words 4194304 --parties 3 --reps 5 > "$OUT/prof.log" 2>&1) || return
}
run_all
rc=$?
echo "end rc=$rc" >> "$OUT/status.txt"
exit $rc
