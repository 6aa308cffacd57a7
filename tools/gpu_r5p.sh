#!/bin/bash
# Round-5 counter passes over the exchange codec ubench (8 Mi FactorPairs,
# full-length): for each variant binary, two --pmc passes (SQ issue / wait /
# LDS counters), kernel-trace only, each under its own time limit.
#   VARIANTS="r4 mac"   binaries tools/ubench/xv/ubench_xdec2_<v>
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${TAG:-r5p}"
mkdir -p "$OUT"
echo "start $(date)" > "$OUT/status.txt"
cd /tmp && export TMPDIR=/tmp
pmc() {
  local v=$1 name=$2
  shift 2
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc "$@" -T -d "$OUT/${v}_$name" -o pmc --output-format csv -- "$ROOT/tools/ubench/xv/ubench_xdec2_$v" 3 1 > "$OUT/${v}_$name.log" 2>&1
  local rc=$?; echo "$v $name rc=$rc $(date +%T)" >> "$OUT/status.txt"; return $rc
}
rc=0
for v in ${VARIANTS:-r4 mac}; do
  pmc $v p0 SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT &&
  pmc $v p1 SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD
  rc=$?
  [ $rc -ne 0 ] && break
done
echo "end rc=$rc $(date)" >> "$OUT/status.txt"
exit $rc
