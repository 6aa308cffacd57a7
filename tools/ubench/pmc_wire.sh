#!/bin/bash
# (A/B helper: the binaries are built into ab/ at the repo root, which travels
# with gpurun -- tools/ubench/ does not; copy this script there to run it)
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${TAG:-pmcw}"
mkdir -p "$OUT"
cd "$ROOT/ab"
export TMPDIR=/tmp
i=0
for g in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_WAVES" \
         "SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL SQ_LDS_ADDR_CONFLICT SQ_THREAD_CYCLES_VALU" \
         "SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_VMEM SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_LEVEL_WAVES SQ_CYCLES"; do
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $g -d "$OUT/p$i" -o pmc --output-format csv -- ./wire_wave 3 4 > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed" >> "$OUT/status.txt"; exit 1; }
  echo "pass $i ok" >> "$OUT/status.txt"
  i=$((i+1))
done
