#!/bin/bash
# Round-5 wire-kernel A/B: tools/ubench/ubench_wire_ab.hip built against
# csrc copies (tools/ubench/xv/csrc_<v>), 4 Mi words x 3 parties, 30
# back-to-back launches of k_mask_b64 then k_rv_b64 per run, passes A B C A B C
# under rocprofv3 --kernel-trace --stats (the sustained averages).
#   VARIANTS="base lutA lutB"
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${TAG:-r5w}"
mkdir -p "$OUT"
echo "start $(date)" > "$OUT/status.txt"
cd /tmp && export TMPDIR=/tmp
rc=0
for pass in 1 2; do
  for v in ${VARIANTS:-base lutA lutB}; do
    timeout -k 10 120 rocprofv3 --kernel-trace --stats -T -d "$OUT/${v}_$pass" -o kt --output-format csv -- "$ROOT/tools/ubench/xv/ubench_wire_ab_$v" 30 4 > "$OUT/${v}_$pass.json" 2> "$OUT/${v}_$pass.err"
    rc=$?; echo "$v pass $pass rc=$rc $(date +%T)" >> "$OUT/status.txt"
    [ $rc -ne 0 ] && break 2
  done
done
echo "end rc=$rc $(date)" >> "$OUT/status.txt"
exit $rc
