#!/bin/bash
# CPU side: exchange-decode variants for an A/B on the GPU (tools/gpu_xdec.sh).
# Each variant is exchange.hip with one sed edit, compiled into the
# ubench_xdec2 harness (tools/ubench/ubench_xdec2.hip includes XDEC_SRC).
# Output: tools/ubench/xv/ (git-ignored; travels to the GPU box).
set -e
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
X="$ROOT/amphora_amd/csrc/exchange.hip"
D="$ROOT/tools/ubench/xv"
mkdir -p "$D"
variant() {  # name [-Dflags] sed-expression...
  local name=$1 defs=""
  shift
  while [ "${1#-D}" != "$1" ]; do defs="$defs $1"; shift; done
  cp "$X" "$D/exchange_$name.hip"
  for e in "$@"; do sed -i "$e" "$D/exchange_$name.hip"; done
  cmp -s "$X" "$D/exchange_$name.hip" && [ "$name" != base ] && [ -z "$defs" ] && { echo "variant $name: sed changed nothing" >&2; exit 1; }
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -I"$ROOT/include" -I"$ROOT/amphora_amd/csrc" \
    $defs -DXDEC_SRC="\"$D/exchange_$name.hip\"" "$ROOT/tools/ubench/ubench_xdec2.hip" -o "$D/ubench_xdec2_$name" &
}
variant base
# the single-read decode (published counts instead of the count pass)
variant fused -DAMPH_XDEC_FUSED=1
# the general pass's grid (its early exit vs its own speed)
variant g1k -DAMPH_XDEC_SLOW_GRID=1024
variant g16k -DAMPH_XDEC_SLOW_GRID=16384
for v in "$@"; do :; done
wait
ls -la "$D"
