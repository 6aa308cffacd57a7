#!/bin/bash
# Round-5 GPU pass A: the default bench line with its new host_memory phase
# (driver command shape), a world-2 gloo rehearsal on the one GPU (per-rank
# records, host_memory over two ranks, scatter/gather), and the same world-2
# rehearsal with an injected stuck gather (the line must still print, with
# scatter_gather.skipped).
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${TAG:-r5a}"
mkdir -p "$OUT"
cd "$ROOT"
echo "start $(date)" > "$OUT/status.txt"
step() {
  local name=$1 lim=$2
  shift 2
  timeout -k 10 "$lim" "$@" > "$OUT/$name.json" 2> "$OUT/$name.err"
  local rc=$?; echo "$name rc=$rc $(date +%T)" >> "$OUT/status.txt"; return $rc
}
step bench_default 300 python -u bench.py --steps 20 --warmup 5 &&
step bench_gloo2 400 python -u bench.py --gpus 2 --backend gloo --same-device --steps 20 --warmup 5 &&
step bench_gloo2_hang 400 python -u bench.py --gpus 2 --backend gloo --same-device --steps 20 --warmup 5 \
  --inject-sg-fault hang --sg-timeout 15 --no-cpu-baseline
rc=$?
echo "end rc=$rc $(date)" >> "$OUT/status.txt"
exit $rc
