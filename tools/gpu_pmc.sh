#!/bin/bash
# PMC passes over one program: each counter group in its own rocprofv3 run
# (--kernel-trace only beside --pmc), each under its own time limit; the
# first failing pass ends the call.  Usage:
#   TAG=name tools/gpu_pmc.sh "<group1>" "<group2>" ... -- <program> [args]
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${TAG:-pmc}"
mkdir -p "$OUT"
groups=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do groups+=("$1"); shift; done
shift
cd /tmp && export TMPDIR=/tmp
i=0
for g in "${groups[@]}"; do
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $g -T -d "$OUT/p$i" -o pmc --output-format csv -- "$@" > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed: $g" >> "$OUT/status.txt"; exit 1; }
  echo "pass $i ok: $g" >> "$OUT/status.txt"
  i=$((i+1))
done
