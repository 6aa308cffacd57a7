#!/bin/bash
# Round-4 GPU pass C: the full GPU suite and smoke on the current library, the
# driver's bench line, its rocprofv3 kernel-trace summary and FETCH / WRITE
# PMC passes (profiles/traffic.json for the C4 roofline), the JNI
# pinned-vs-region benchmark.  Each GPU step has its own time limit; the
# first failure ends the call.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${TAG:-r4c}"
mkdir -p "$OUT"
cd "$ROOT"
echo "start $(date)" > "$OUT/status.txt"
step() {  # step NAME SECONDS CMD...
  local name=$1 secs=$2
  shift 2
  timeout -k 10 "$secs" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?
  echo "$name rc=$rc $(date +%T)" >> "$OUT/status.txt"
  return $rc
}
prof() {  # prof NAME SECONDS ROCPROF-ARGS... -- CMD...
  local name=$1 secs=$2
  shift 2
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 "$secs" rocprofv3 "$@") > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc $(date +%T)" >> "$OUT/status.txt"
  return $rc
}
run_all() {
  [ -n "$SKIP_SMOKE" ] || step smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()" || return
  [ -n "$SKIP_TESTS" ] || step pytest 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread || return
  step bench_driver 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 || return
  prof bench_ktrace 300 --kernel-trace --stats -d "$OUT/bench_ktrace" -o k --output-format csv -- python3 "$ROOT/bench.py" --steps 20 --warmup 5 --no-cpu-baseline || return
  prof bench_fetch 300 --kernel-trace --pmc FETCH_SIZE -d "$OUT/bench_fetch" -o pmc --output-format csv -- python3 "$ROOT/bench.py" --steps 10 --warmup 2 --no-cpu-baseline || return
  prof bench_write 300 --kernel-trace --pmc WRITE_SIZE -d "$OUT/bench_write" -o pmc --output-format csv -- python3 "$ROOT/bench.py" --steps 10 --warmup 2 --no-cpu-baseline || return
  step jni_regions 300 python3 tools/bench_jni_regions.py || return
  step wire 300 python3 tools/wire_kernels.py || return
  step valu_rate 120 ./tools/ubench/ubench_valu_rate || return
  timeout -k 10 120 ./tools/ubench/wocc/u_g5p0 4194304 20 probe >> "$OUT/wire_probe.jsonl" 2>> "$OUT/wire_probe.err" || return
  timeout -k 10 200 ./tools/ubench/wocc/u_g5p0 16777216 5 probe >> "$OUT/wire_probe.jsonl" 2>> "$OUT/wire_probe.err" || return
  for blk in 256 512 1024 256 512 1024; do
    ( export AMPH_BLOCK=$blk; step bench_blk${blk}_$RANDOM 300 python3 bench.py --no-cpu-baseline --steps 200 --warmup 20 ) || return
  done
}
run_all
rc=$?
echo "end rc=$rc $(date)" >> "$OUT/status.txt"
exit $rc
