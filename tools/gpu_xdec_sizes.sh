#!/bin/bash
# GPU: the base exchange-decode harness at several text sizes (Mi FactorPairs),
# full-length values, rocprofv3 kernel trace each (does the second read of the
# text hit the 256 MiB Infinity Cache when the text fits?).
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${TAG:-xsz}"
mkdir -p "$OUT"
D="$ROOT/tools/ubench/xv"
cd /tmp && export TMPDIR=/tmp
for m in ${SIZES:-1 2 4 8 16}; do
  timeout -k 10 90 rocprofv3 --kernel-trace --stats -T -d "$OUT/prof_$m" -o kt --output-format csv -- "$D/ubench_xdec2_${V:-base}" 20 1 $m > "$OUT/run_$m.log" 2>&1 || exit 1
done
echo done > "$OUT/status.txt"
