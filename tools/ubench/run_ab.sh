#!/bin/bash
# (A/B helper: the binaries are built into ab/ at the repo root, which travels
# with gpurun -- tools/ubench/ does not; copy this script there to run it)
# interleaved A/B of two ubench binaries + one rocprofv3 --stats pass each
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${TAG:-ab}"
mkdir -p "$OUT"
cd "$ROOT/ab"
export TMPDIR=/tmp
A=${A:-xdec_base}; B=${B:-xdec_new}; ARGS=${ARGS:-"30 1 8"}
for i in 1 2 3; do
  for v in $A $B; do
    echo "== $v pass $i" >> "$OUT/ab.txt"
    timeout -k 10 120 ./$v $ARGS >> "$OUT/ab.txt" 2>&1 || exit 1
  done
done
for v in $A $B; do
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$v" -o kt --output-format csv -- ./$v $ARGS > "$OUT/prof_$v.log" 2>&1 || exit 1
done
echo done >> "$OUT/ab.txt"
