#!/bin/bash
# Round-4 GPU pass (first call): the driver's default bench line (C4 at N=1,
# --steps 20 --warmup 5 as the driver runs it, then the 1000-step default),
# and the self-spawned 2-rank C4 rehearsal (gloo, both ranks on cuda:0) with
# the grouped root scatter/gather and the CPU baseline.  Every GPU step has
# its own time limit; steps are chained with && so the first failure ends
# the call.  Logs land in gpurun_out/$TAG (merged back).
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${TAG:-r4}"
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
  [ -n "$SKIP_TESTS" ] || step pytest 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} || return
  step bench_driver 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 || return
  [ -n "$SKIP_LONG" ] || step bench_default 300 python3 bench.py --no-cpu-baseline || return
  step bench_c4_gloo2 600 python3 bench.py --gpus 2 --backend gloo --same-device --steps 200 --warmup 20 --sg-steps 2 || return
  [ -z "$EXTRA" ] || step extra 600 bash -c "$EXTRA" || return
}
run_all
rc=$?
echo "end rc=$rc $(date)" >> "$OUT/status.txt"
exit $rc
