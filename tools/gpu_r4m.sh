#!/bin/bash
# Round-4 GPU pass M: counter passes over the final fused wire kernels at
# 4 Mi words x 3 parties (tools/wire_kernels.py on the product library):
# SQ issue / wait / LDS counters, FETCH_SIZE and WRITE_SIZE, each pass its own
# run with --kernel-trace only.  The first failure ends the call.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${TAG:-r4m}"
mkdir -p "$OUT"
cd "$ROOT"
echo "start $(date)" > "$OUT/status.txt"
pmc() {  # pmc NAME COUNTERS...
  local name=$1
  shift
  (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 150 rocprofv3 --kernel-trace --pmc "$@" -T -d "$OUT/$name" -o pmc --output-format csv -- python3 "$ROOT/tools/wire_kernels.py" --reps 3) > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc $(date +%T)" >> "$OUT/status.txt"
  return $rc
}
pmc pmc0 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_WAVES &&
pmc pmc1 FETCH_SIZE &&
pmc pmc2 WRITE_SIZE &&
pmc pmc3 SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR
rc=$?
echo "end rc=$rc $(date)" >> "$OUT/status.txt"
exit $rc
