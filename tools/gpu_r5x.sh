#!/bin/bash
# Round-5 exchange-codec A/B: ubench_xdec2 (8 Mi FactorPairs, full-length
# diffs, 752 MB of text) built against the round-4 exchange.hip and each
# variant, run in turn (A B A B ...) under rocprofv3 --kernel-trace --stats.
#   VARIANTS="r4 mac ..."   binaries tools/ubench/xv/ubench_xdec2_<v>
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${TAG:-r5x}"
mkdir -p "$OUT"
echo "start $(date)" > "$OUT/status.txt"
cd /tmp && export TMPDIR=/tmp
rc=0
for pass in 1 2; do
  for v in ${VARIANTS:-r4 mac}; do
    B="$ROOT/tools/ubench/xv/ubench_xdec2_$v"
    timeout -k 10 120 rocprofv3 --kernel-trace --stats -T -d "$OUT/${v}_$pass" -o kt --output-format csv -- "$B" 20 1 > "$OUT/${v}_$pass.log" 2>&1
    rc=$?; echo "$v pass $pass rc=$rc $(date +%T)" >> "$OUT/status.txt"
    [ $rc -ne 0 ] && break 2
  done
done
echo "end rc=$rc $(date)" >> "$OUT/status.txt"
exit $rc
