#!/bin/bash
# C1 through the C++ mirror under rocprofv3: kernel and HIP-runtime traces with
# per-call statistics (where a 1 k-word upload / download spends its time),
# then a PMC pass over the exchange decode (LDS bank conflicts, VALU, waits).
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${TAG:-c1prof}"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 "$ROOT/tools/c1_native" 1024 30 own > "$OUT/c1_plain.json" 2>&1 || exit 1
timeout -k 10 180 rocprofv3 --kernel-trace --hip-runtime-trace --stats -T -d "$OUT/c1" -o c1 --output-format csv -- "$ROOT/tools/c1_native" 1024 30 own > "$OUT/c1_prof.log" 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_WAVES -T -d "$OUT/pmc" -o pmc --output-format csv -- "$ROOT/tools/ubench/xv/ubench_xdec2_base" 3 1 > "$OUT/pmc.log" 2>&1 || exit 1
echo done > "$OUT/status.txt"
