#!/bin/bash
# Round-4 GPU pass R: base64 block kernels with the tail as their last
# workgroup (one launch per call) -- codec / wire / party GPU tests on the new
# library, tools/bench_codec.py old / new in turn, the 4 Mi x 3 pipelines.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${TAG:-r4r}"
mkdir -p "$OUT"
cd "$ROOT"
echo "start $(date)" > "$OUT/status.txt"
LIB="$ROOT/amphora_amd/libamphora_hip.so"
run_all() {
  cp "$ROOT/build/ab/new.so" "$LIB" || return
  timeout -k 10 600 python3 -u -m pytest tests/test_wire.py tests/test_wire_fused.py tests/test_party_session.py tests/test_abi.py tests/test_host_ordering.py tests/test_hip_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.out" 2>&1
  local rc=$?; echo "pytest rc=$rc $(date +%T)" >> "$OUT/status.txt"; [ $rc -eq 0 ] || return $rc
  for rep in 1 2; do
    for v in old new; do
      cp "$ROOT/build/ab/$v.so" "$LIB" || return
      timeout -k 10 300 python3 tools/bench_pipeline.py --words 4194304 --parties 3 --reps 10 >> "$OUT/pipe_$v.jsonl" 2>> "$OUT/pipe_$v.err"
      rc=$?; echo "pipe_$v rc=$rc $(date +%T)" >> "$OUT/status.txt"; [ $rc -eq 0 ] || return $rc
    done
  done
  cp "$ROOT/build/ab/new.so" "$LIB"
}
run_all
rc=$?
echo "end rc=$rc $(date)" >> "$OUT/status.txt"
exit $rc
