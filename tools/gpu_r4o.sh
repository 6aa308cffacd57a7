#!/bin/bash
# Round-4 GPU pass N/O: the base64 codec kernels (decode, then encode) --
# tools/bench_codec.py with the previous library and the new one in turn
# (build/ab/{old,new}.so copied over the in-tree library, twice each), then
# the codec / wire GPU tests on the new library.  First failure ends the call.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${TAG:-r4o}"
mkdir -p "$OUT"
cd "$ROOT"
echo "start $(date)" > "$OUT/status.txt"
LIB="$ROOT/amphora_amd/libamphora_hip.so"
run_all() {
  for rep in 1 2; do
    for v in old new; do
      cp "$ROOT/build/ab/$v.so" "$LIB" || return
      timeout -k 10 300 python3 tools/bench_codec.py >> "$OUT/codec_$v.jsonl" 2>> "$OUT/codec_$v.err"
      local rc=$?; echo "codec_$v rc=$rc $(date +%T)" >> "$OUT/status.txt"; [ $rc -eq 0 ] || return $rc
    done
  done
  cp "$ROOT/build/ab/new.so" "$LIB" || return
  for rep in 1 2 3; do  # the fused K_MASK's records encode: previous / new wire kernels (ubench)
    for v in new8 enc; do
      LD_LIBRARY_PATH="$ROOT/build/ab/oldlib" timeout -k 10 120 "$ROOT/tools/ubench/wocc/u_g5p0_$v" 4194304 20 >> "$OUT/wire_$v.jsonl" 2>> "$OUT/wire_$v.err" || return
    done
  done
  echo "wire ab done $(date +%T)" >> "$OUT/status.txt"
  timeout -k 10 600 python3 -u -m pytest tests/test_wire.py tests/test_wire_fused.py tests/test_hip_parity.py tests/test_abi.py tests/test_host_ordering.py tests/test_party_session.py -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.out" 2>&1
  local rc=$?; echo "pytest rc=$rc $(date +%T)" >> "$OUT/status.txt"; return $rc
}
run_all
rc=$?
echo "end rc=$rc $(date)" >> "$OUT/status.txt"
exit $rc
