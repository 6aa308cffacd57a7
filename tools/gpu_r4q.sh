#!/bin/bash
# Round-4 GPU pass Q: the exchange encode's digit images + wide literal stores
# -- ubench_xdec2 (base = previous exchange.hip, new = current) kernel traces,
# tools/bench_codec.py with the previous and the new library in turn, then the
# exchange / party-session GPU tests on the new library.  First failure ends it.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${TAG:-r4q}"
mkdir -p "$OUT"
cd "$ROOT"
echo "start $(date)" > "$OUT/status.txt"
LIB="$ROOT/amphora_amd/libamphora_hip.so"
run_all() {
  for v in base new; do
    (cd /tmp && export TMPDIR=/tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$v" -o kt --output-format csv -- "$ROOT/tools/ubench/xv/ubench_xdec2_$v" 20 1) > "$OUT/prof_$v.log" 2>&1
    local rc=$?; echo "prof_$v rc=$rc $(date +%T)" >> "$OUT/status.txt"; [ $rc -eq 0 ] || return $rc
  done
  for rep in 1 2; do
    for v in old new; do
      cp "$ROOT/build/ab/$v.so" "$LIB" || return
      timeout -k 10 300 python3 tools/bench_codec.py >> "$OUT/codec_$v.jsonl" 2>> "$OUT/codec_$v.err"
      local rc=$?; echo "codec_$v rc=$rc $(date +%T)" >> "$OUT/status.txt"; [ $rc -eq 0 ] || return $rc
    done
  done
  cp "$ROOT/build/ab/new.so" "$LIB" || return
  timeout -k 10 600 python3 -u -m pytest tests/test_wire.py tests/test_party_session.py tests/test_abi.py tests/test_host_ordering.py tests/test_hip_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.out" 2>&1
  local rc=$?; echo "pytest rc=$rc $(date +%T)" >> "$OUT/status.txt"; return $rc
}
run_all
rc=$?
echo "end rc=$rc $(date)" >> "$OUT/status.txt"
exit $rc
