#!/bin/bash
# Round-5 pipelined pair-order exchange decode A/B: ubench_xdec2 (8 Mi
# FactorPairs, full-length, 752 MB) on one stream vs the two-stream pipeline
# (argv 4 = pipe), passes A B A B: plain runs (HIP-event medians of the whole
# call, which is what overlap changes), then one rocprofv3 --kernel-trace each.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${TAG:-r5d}"
mkdir -p "$OUT"
echo "start $(date)" > "$OUT/status.txt"
B="$ROOT/tools/ubench/xv/ubench_xdec2_${BIN:-prod2}"
rc=0
for pass in 1 2; do
  for m in one pipe; do
    timeout -k 10 120 "$B" 20 1 8 $m > "$OUT/${m}_$pass.log" 2>&1
    rc=$?; echo "$m pass $pass rc=$rc $(date +%T)" >> "$OUT/status.txt"
    [ $rc -ne 0 ] && exit $rc
  done
done
cd /tmp && export TMPDIR=/tmp
for m in one pipe; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$m" -o kt --output-format csv -- "$B" 20 1 8 $m > "$OUT/prof_$m.log" 2>&1
  rc=$?; echo "prof $m rc=$rc $(date +%T)" >> "$OUT/status.txt"
  [ $rc -ne 0 ] && exit $rc
done
echo "end rc=$rc $(date)" >> "$OUT/status.txt"
exit $rc
