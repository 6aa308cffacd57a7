#!/bin/bash
# Round-4 GPU pass B: JNI region-mode tests, the HIP-API trace of the
# multi-device per-call latency tool (no per-call hipSetDevice thread setup),
# the fused wire kernels' kernel-trace and PMC passes.
# Every GPU step has its own time limit; the first failure ends the call.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${TAG:-r4b}"
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
pmc() {  # pmc NAME COUNTERS... -- CMD...
  local name=$1
  shift
  local ctr=()
  while [ "$1" != "--" ]; do ctr+=("$1"); shift; done
  shift
  (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 150 rocprofv3 --kernel-trace --pmc "${ctr[@]}" -T -d "$OUT/$name" -o pmc --output-format csv -- "$@") > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc $(date +%T)" >> "$OUT/status.txt"
  return $rc
}
run_all() {
  [ -n "$SKIP_TESTS" ] || step pytest 600 python3 -u -m pytest ${PYTEST_FILES:-tests/test_wire_fused.py tests/test_wire.py tests/test_jni_core.py} -m gpu -x -v --timeout 300 --timeout-method thread || return
  [ -n "$SKIP_TRACE" ] || { (cd /tmp && export TMPDIR=/tmp && timeout -k 10 120 rocprofv3 --hip-trace --stats -d "$OUT/hiptrace_new" -o t --output-format csv -- "$ROOT/tools/multi_latency" "$ROOT/amphora_amd/libamphora_hip.so" 1024 100 0,0,0) > "$OUT/hiptrace_new.log" 2>&1 && echo "hiptrace_new ok" >> "$OUT/status.txt" || return; }
  [ -n "$SKIP_TRACE" ] || { (cd /tmp && export TMPDIR=/tmp && timeout -k 10 120 rocprofv3 --hip-trace --stats -d "$OUT/hiptrace_old" -o t --output-format csv -- "$ROOT/tools/multi_latency" "$ROOT/build/prev/libamphora_hip_r3.so" 1024 100 0,0,0) > "$OUT/hiptrace_old.log" 2>&1 && echo "hiptrace_old ok" >> "$OUT/status.txt" || return; }
  for form in reg lds; do
    ( export AMPH_WIRE_FORM=$form; step wire_$form 300 python3 tools/wire_kernels.py ) || return
  done
  ( export AMPH_WIRE_FORM=reg; step wire_reg2 300 python3 tools/wire_kernels.py ) || return
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/wire_ktrace" -o k --output-format csv -- python3 "$ROOT/tools/wire_kernels.py") > "$OUT/wire_ktrace.log" 2>&1 && echo "wire_ktrace ok" >> "$OUT/status.txt" || return
  [ -n "$SKIP_PMC" ] && return 0
  for form in lds reg; do
    ( export AMPH_WIRE_FORM=$form
      pmc pmc0_$form SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_WAVES -- python3 "$ROOT/tools/wire_kernels.py" --reps 3 &&
      pmc pmc1_$form FETCH_SIZE -- python3 "$ROOT/tools/wire_kernels.py" --reps 3 &&
      pmc pmc2_$form WRITE_SIZE -- python3 "$ROOT/tools/wire_kernels.py" --reps 3 ) || return
  done
  (timeout -k 10 60 rocprofv3 -L > "$OUT/counters.txt" 2>&1; true)
  for form in lds reg; do
    ( export AMPH_WIRE_FORM=$form
      pmc pmc3_$form SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR -- python3 "$ROOT/tools/wire_kernels.py" --reps 3 ) || return
  done
}
run_all
rc=$?
echo "end rc=$rc $(date)" >> "$OUT/status.txt"
exit $rc
