#!/bin/bash
# Build the LDS-form wire-kernel occupancy variants (tools/ubench/ubench_wire_occ.hip)
# into tools/ubench/wocc/u_g<G>p<PD> against the in-tree libamphora_hip.so.
set -e
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
mkdir -p "$ROOT/tools/ubench/wocc"
for G in ${GS:-1 2 3 5}; do for PD in ${PDS:-0 1 2 3}; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -Wno-pass-failed -DAMPH_WIRE_G=$G -DAMPH_WIRE_PD=$PD \
    -I"$ROOT/include" "$ROOT/tools/ubench/ubench_wire_occ.hip" -L"$ROOT/amphora_amd" -lamphora_hip \
    -Wl,-rpath,'$ORIGIN/../../../amphora_amd' -o "$ROOT/tools/ubench/wocc/u_g${G}p${PD}" &
done; done
wait
ls "$ROOT/tools/ubench/wocc"
