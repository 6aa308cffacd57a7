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
# k_xdec_fast diagnostics (outputs wrong; read its rocprofv3 time):
#   store  - every value stored whatever its checks say (the reference for the two below)
#   noconf - as store, each lane parsing bytes at a lane-staggered LDS offset (13-dword
#            stride: conflict-free ds_read_b32 banks) instead of its value's
variant store 's/if (g < nvals \&\& fast_segment(l32, at + 1 + kWinPad, g, nvals, b0 + at + 1 - text.mis, len, fn)) {/if (g < nvals \&\& (fast_segment(l32, at + 1 + kWinPad, g, nvals, b0 + at + 1 - text.mis, len, fn) || true)) {/'
variant noconf 's/if (g < nvals \&\& fast_segment(l32, at + 1 + kWinPad, g, nvals, b0 + at + 1 - text.mis, len, fn)) {/if (g < nvals \&\& (fast_segment(l32, (threadIdx.x * 52u + 300u) % 7900u + 16u, g, nvals, b0 + at + 1 - text.mis, len, fn) || true)) {/'
# digit run + segment checks, no base-10^8 conversion
variant noconv 's/^  const uint32_t full = nd >> 3, rem = nd \& 7u;$/  r.v[0] = nd; r.v[1] = r.v[2] = r.v[3] = 0; return true;\n  const uint32_t full = nd >> 3, rem = nd \& 7u;/'
# k_xenc_write diagnostics (text wrong; read its rocprofv3 time):
#   enost  - the run staged in LDS as usual, the 16-byte global stores skipped
#   enconv - no base-10^9 split (chunks from the raw limbs, 38-39 digits)
#   enfmt  - conversion as usual, no digit formatting into LDS
variant enost 's/      xst16(reinterpret_cast<uint4\*>(dal) + u, bufv\[u\]);/      if (bufv[u].x == 0x01020304u) xst16(reinterpret_cast<uint4*>(dal) + u, bufv[u]);/'
variant enconv 's/^    nd = to_chunks(d, cd);$/    nd = 38 + (d.x \& 1); cd[0] = d.x \& 0x1FFFFFFFu; cd[1] = d.y \& 0x1FFFFFFFu; cd[2] = d.z \& 0x1FFFFFFFu; cd[3] = d.w \& 0x1FFFFFFFu; cd[4] = 99u + (d.x \& 1) * 900u;/' 's/^    ne = to_chunks(e, ce);$/    ne = 38 + (e.x \& 1); ce[0] = e.x \& 0x1FFFFFFFu; ce[1] = e.y \& 0x1FFFFFFFu; ce[2] = e.z \& 0x1FFFFFFFu; ce[3] = e.w \& 0x1FFFFFFFu; ce[4] = 99u + (e.x \& 1) * 900u;/'
variant enfmt 's/^    o = put_digits(o, cd, nd);$/    o += nd + (cd[0] == 7u);/' 's/^    o = put_digits(o, ce, ne);$/    o += ne + (ce[0] == 7u);/'
# k_xenc_write formatting diagnostics (text wrong):
#   enal8  - each whole chunk's 8 digit bytes stored at an 8-aligned LDS address (does the
#            unaligned ds_write_b64 cost?)
#   enpart - the leading partial chunk's predicated byte stores skipped
variant enal8 's/      __builtin_memcpy(o + base + 1, \&w0, 4);/      char* oa = o + base + 1 - ((uintptr_t)(o + base + 1) \& 7); __builtin_memcpy(oa, \&w0, 4);/' 's/      __builtin_memcpy(o + base + 5, \&w1, 4);/      __builtin_memcpy(oa + 4, \&w1, 4);/'
variant enpart 's/      if (base + j >= 0) o\[base + j\] = (char)dig\[j\];/      if (base + j >= 0 \&\& j > 99) o[base + j] = (char)dig[j];/'
# (the persistent compact-pass variants p1536/p2048/p4096 need exchange.hip at commit dc51c3d)
for v in "$@"; do :; done
wait
ls -la "$D"
