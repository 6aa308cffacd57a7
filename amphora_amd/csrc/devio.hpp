// Device-side helpers shared by the kernel translation units (kernels.hip,
// wire.hip): the launch macro, 16-byte streaming loads / stores with their
// cache policy, the wave-level first-fail report and the party-count dispatch.
#pragma once
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include "kernels.hpp"

namespace amph {

// Every launch goes through hipExtLaunchKernelGGL: with the config's timing
// events set (amph_time_next_launch) the events are stamped by the kernel's
// own dispatch, i.e. they measure the kernel, not the queue gap before it.
#define AMPH_LAUNCH(K, G, B, C, ...) \
  hipExtLaunchKernelGGL(K, G, B, 0, (C).stream, (C).ev_start, (C).ev_stop, 0, __VA_ARGS__)

#define AMPH_DISPATCH_NP(n, BIG, LAUNCH) \
  switch (n) {                           \
    case 1: LAUNCH(1, BIG); break;       \
    case 2: LAUNCH(2, BIG); break;       \
    case 3: LAUNCH(3, BIG); break;       \
    case 4: LAUNCH(4, BIG); break;       \
    default: LAUNCH(0, BIG); break;      \
  }

namespace {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// Streamed-once inputs: nontemporal 16-byte loads (global_load_dwordx4 nt;
// AMPH_LD_NT=0 for A/B: plain loads measured 8-10 % slower at C2 with the
// nontemporal stores in place).
#ifndef AMPH_LD_NT
#define AMPH_LD_NT 1
#endif
__device__ __forceinline__ uint4 ld(const uint4* p) {
  if constexpr (AMPH_LD_NT) {
    const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
    return make_uint4(v.x, v.y, v.z, v.w);
  } else {
    return *p;
  }
}
__device__ __forceinline__ void st(uint4* p, const W4& v) { *p = u4(v); }
// Result words (K_RV / K_MASK and their wire forms, the open, the products):
// nontemporal 16-byte stores.  Measured in bench.py on one box, alternating
// builds 3x: C2 14.6-15.0 -> 15.6-15.8 G words/s, C3 10.7-10.8 -> 11.0-11.2;
// k_open / k_open_post -7 % at 16 Mi words (profiles/r02_ab_store_policy.txt).
// Plain stores left each kernel's output dirty in the caches for the next
// launch to drain.  (Round 1's ubench_store had preferred plain stores at
// 16 Mi words.)  Intermediates read again at once (K_ODO_PRE's diffs) keep
// plain stores.
#ifndef AMPH_ST_NT
#define AMPH_ST_NT 1
#endif
__device__ __forceinline__ void st_out(uint4* p, const W4& v) {
  if constexpr (AMPH_ST_NT) {
    const uint4 x = u4(v);
    __builtin_nontemporal_store(u32x4{x.x, x.y, x.z, x.w}, reinterpret_cast<u32x4*>(p));
  } else {
    *p = u4(v);
  }
}

// Party-side outputs that the next stage reads at once (K_CONV's share
// words, K_ODO_PRE's raw copies and diffs): nontemporal as well.  Alternated
// A/B, 3x on one box: K_CONV and K_ODO_PRE -4 % at 16 Mi words, the exchange
// encode that reads the diffs -8 %, party Output Delivery 4 Mi x 3
// 1.81 -> 1.79 ms (profiles/r02_ab_store_policy.txt).  AMPH_PARTY_NT=0 for
// plain stores.
#ifndef AMPH_PARTY_NT
#define AMPH_PARTY_NT 1
#endif
__device__ __forceinline__ void st_party(uint4* p, const uint4& x) {
  if constexpr (AMPH_PARTY_NT) __builtin_nontemporal_store(u32x4{x.x, x.y, x.z, x.w}, reinterpret_cast<u32x4*>(p));
  else *p = x;
}

// Wave-level reduction of the failing indices to one atomic per wave: the
// lowest set lane holds the smallest index of this iteration.
__device__ __forceinline__ void report_fail(bool bad, size_t i, unsigned long long* ff) {
  const unsigned long long m = __ballot(bad);
  if (m != 0ULL) {
    const int lane = __lane_id();
    if (lane == __ffsll((long long)m) - 1) atomicMin(ff, (unsigned long long)i);
  }
}

}  // namespace
}  // namespace amph
