#!/bin/bash
# Round-3 GPU pass: smoke, GPU parity tests, the C2 headline, C4 on one GPU,
# and the self-spawned 2-rank C4 rehearsal (gloo, both ranks on cuda:0).
# Every GPU step has its own time limit; steps are chained with && so the
# first failure ends the call.  Logs land in gpurun_out/$TAG (merged back).
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${TAG:-r3}"
mkdir -p "$OUT"
cd "$ROOT"
echo "start $(date)" > "$OUT/status.txt"
{ nproc; cat /sys/fs/cgroup/cpu.max; python3 -c "import os; print(len(os.sched_getaffinity(0)))"; } > "$OUT/cpus.txt" 2>&1 || true
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
  step bench_c2 300 python3 bench.py || return
  step bench_c4_n1 300 python3 bench.py --workload c4 --no-cpu-baseline || return
  step bench_c4_gloo2 300 python3 bench.py --gpus 2 --backend gloo --same-device || return
  step c1_own 120 ./tools/c1_native 1024 30 own || return
  step c1_shared 120 ./tools/c1_native 1024 30 shared || return
  step c1_own_fresh 120 ./tools/c1_native 1024 30 own 2 fresh || return
  step c1_own_3p 120 ./tools/c1_native 1024 30 own 3 || return
  step c1_own_4k 120 ./tools/c1_native 4096 20 own || return
  step c1_own_64k 120 ./tools/c1_native 65536 10 own || return
}
run_all
rc=$?
echo "end rc=$rc $(date)" >> "$OUT/status.txt"
exit $rc
