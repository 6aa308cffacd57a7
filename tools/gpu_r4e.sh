#!/bin/bash
# Round-4 GPU pass E: the 6-bit decode (b64.hpp dec4_values6) in the fused
# wire kernels -- old/new ubench A/B (both checked against the previous
# library, build/prev/r4old), the wire/codec GPU tests on the new library,
# the new kernels' VALU-count PMC pass.  First failure ends the call.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${TAG:-r4e}"
mkdir -p "$OUT"
cd "$ROOT"
echo "start $(date)" > "$OUT/status.txt"
step() {  # step NAME SECONDS CMD...
  local name=$1 secs=$2
  shift 2
  timeout -k 10 "$secs" "$@" >> "$OUT/$name.out" 2>> "$OUT/$name.err"
  local rc=$?
  echo "$name rc=$rc $(date +%T)" >> "$OUT/status.txt"
  return $rc
}
run_all() {
  for rep in 1 2 3; do
    for v in ${VARIANTS:-old new new4}; do
      LD_LIBRARY_PATH="$ROOT/build/prev/r4old" step ab_$v 120 "$ROOT/tools/ubench/wocc/u_g5p0_$v" 4194304 20 || return
    done
  done
  step pytest 600 python3 -u -m pytest ${PYTEST_FILES:-tests/test_wire_fused.py tests/test_wire.py} -m gpu -x -v --timeout 300 --timeout-method thread || return
  step wire_new 300 python3 tools/wire_kernels.py || return
  (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 150 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_BUSY_CYCLES -T -d "$OUT/pmc_valu" -o pmc --output-format csv -- python3 "$ROOT/tools/wire_kernels.py" --reps 3) > "$OUT/pmc_valu.log" 2>&1
  local rc=$?; echo "pmc_valu rc=$rc" >> "$OUT/status.txt"; return $rc
}
run_all
rc=$?
echo "end rc=$rc $(date)" >> "$OUT/status.txt"
exit $rc
