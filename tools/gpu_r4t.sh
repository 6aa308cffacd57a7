#!/bin/bash
# Round-4 GPU pass T: counter passes over the exchange codec kernels (for the
# next round's plan): ubench_xdec2 (8 Mi FactorPairs, full-length) under
# rocprofv3 --pmc, SQ issue / wait / LDS counters, FETCH_SIZE, WRITE_SIZE.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${TAG:-r4t}"
mkdir -p "$OUT"
echo "start $(date)" > "$OUT/status.txt"
B="$ROOT/tools/ubench/xv/ubench_xdec2_base"
pmc() {
  local name=$1
  shift
  (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --kernel-trace --pmc "$@" -T -d "$OUT/$name" -o pmc --output-format csv -- "$B" 3 1) > "$OUT/$name.log" 2>&1
  local rc=$?; echo "$name rc=$rc $(date +%T)" >> "$OUT/status.txt"; return $rc
}
pmc pmc0 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_WAVES &&
pmc pmc1 FETCH_SIZE &&
pmc pmc2 WRITE_SIZE &&
pmc pmc3 SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR
rc=$?
echo "end rc=$rc $(date)" >> "$OUT/status.txt"
exit $rc
