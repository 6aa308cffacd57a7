// Memory-pattern A/B for K_MASK's access pattern (tool): 10 ODO arrays + the
// secrets read (11 x 16 B per word at 2 parties), one 16-B word written, an
// XOR in place of the field arithmetic.  Which load structure moves these
// bytes fastest on MI355X?
//   A  probe: one word per lane, full grid of 1024-lane workgroups, all 11
//      loads issued up front (= k_stream_probe, what K_MASK does)
//   B  the same bytes as ONE contiguous read stream (+ the same writes):
//      the rate of a plain sweep, for calibration
//   D  A with the loads as LDS-DMA (global_load_lds_dwordx4, nt): each wave's
//      11 KiB land in its LDS slice, no VGPR destinations
//   E  persistent workgroups over contiguous word ranges (G workgroups),
//      registers double-buffered: tile t+1's loads issued before tile t's
//      XOR and store
//   C  persistent waves over contiguous ranges with an LDS-DMA ring: each
//      wave keeps R tiles (64 words x 11 arrays = 11 KiB each) in flight,
//      retiring one per step with a counted vmcnt
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 ubench_stream.hip -o ubench_stream
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
constexpr int NA = 11;  // read arrays (10 ODO fields at 2 parties + secrets)

struct Arrs {
  const uint4* a[NA];
};

__device__ __forceinline__ uint4 ld(const uint4* p) {
  const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
  return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void xr(uint4& x, const uint4& v) {
  x.x ^= v.x; x.y ^= v.y; x.z ^= v.z; x.w ^= v.w;
}

__global__ __launch_bounds__(1024) void kA(Arrs in, size_t W, uint4* out) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= W) return;
  uint4 v[NA];
#pragma unroll
  for (int k = 0; k < NA; ++k) v[k] = ld(in.a[k] + i);
  uint4 x = v[0];
#pragma unroll
  for (int k = 1; k < NA; ++k) xr(x, v[k]);
  out[i] = x;
}

// one contiguous stream of NA*W words: word j of "lane" i is at NA*i + j
__global__ __launch_bounds__(1024) void kB(const uint4* one, size_t W, uint4* out) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= W) return;
  const size_t blk = (size_t)blockIdx.x * blockDim.x * NA;
  uint4 v[NA];
#pragma unroll
  for (int k = 0; k < NA; ++k) v[k] = ld(one + blk + (size_t)k * blockDim.x + threadIdx.x);
  uint4 x = v[0];
#pragma unroll
  for (int k = 1; k < NA; ++k) xr(x, v[k]);
  out[i] = x;
}

__global__ __launch_bounds__(256) void kD(Arrs in, size_t W, uint4* out) {
  __shared__ uint4 buf[4][NA][64];  // per wave: NA x 1 KiB (44 KiB per workgroup: 3 per CU)
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t ic = i < W ? i : W - 1;
#pragma unroll
  for (int k = 0; k < NA; ++k)
    __builtin_amdgcn_global_load_lds((const void*)(in.a[k] + ic), (__attribute__((address_space(3))) void*)&buf[wave][k][0], 16, 0, 2);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  uint4 x = buf[wave][0][lane];
#pragma unroll
  for (int k = 1; k < NA; ++k) xr(x, buf[wave][k][lane]);
  if (i < W) out[i] = x;
}

// E: workgroup b owns words [b*per, min(W,(b+1)*per)), tiles of blockDim words
template <int BS>
__global__ __launch_bounds__(BS) void kE(Arrs in, size_t W, size_t per, uint4* out) {
  const size_t s0 = (size_t)blockIdx.x * per, e0 = min(W, s0 + per);
  if (s0 >= e0) return;
  uint4 cur[NA], nxt[NA];
  size_t i = s0 + threadIdx.x;
  {
    const size_t ic = i < e0 ? i : e0 - 1;
#pragma unroll
    for (int k = 0; k < NA; ++k) nxt[k] = ld(in.a[k] + ic);
  }
  for (; i < e0; i += BS) {
#pragma unroll
    for (int k = 0; k < NA; ++k) cur[k] = nxt[k];
    const size_t n = i + BS, nc = n < e0 ? n : e0 - 1;
#pragma unroll
    for (int k = 0; k < NA; ++k) nxt[k] = ld(in.a[k] + nc);
    uint4 x = cur[0];
#pragma unroll
    for (int k = 1; k < NA; ++k) xr(x, cur[k]);
    out[i] = x;
  }
}

// C: wave-persistent LDS-DMA ring.  Wave w (of all waves) owns words
// [w*per, (w+1)*per) (per a multiple of 64); R ring slots of NA KiB each.
template <int R, int WPB>
__global__ __launch_bounds__(64 * WPB) void kC(Arrs in, size_t W, size_t per, uint4* out) {
  __shared__ uint4 ring[WPB][R][NA][64];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const size_t gw = (size_t)blockIdx.x * WPB + wave;
  const size_t s0 = gw * per;
  if (s0 >= W) return;
  const size_t e0 = min(W, s0 + per);
  const size_t nt = (e0 - s0 + 63) / 64;
  auto issue = [&](size_t t, int slot) {
    size_t i = s0 + t * 64 + lane;
    i = i < e0 ? i : e0 - 1;
#pragma unroll
    for (int k = 0; k < NA; ++k)
      __builtin_amdgcn_global_load_lds((const void*)(in.a[k] + i),
                                       (__attribute__((address_space(3))) void*)&ring[wave][slot][k][0], 16, 0, 2);
  };
  // prologue: R - 1 tiles in flight
#pragma unroll
  for (int t = 0; t < R - 1; ++t)
    if ((size_t)t < nt) issue(t, t);
  for (size_t t = 0; t < nt; ++t) {
    const int slot = (int)(t % R);
    // issue tile t + R - 1 into the slot tile t - 1 used (already consumed)
    if (t + R - 1 < nt) {
      issue(t + R - 1, (int)((t + R - 1) % R));
      // tile t's NA loads retire once at most (R - 1) * NA newer ones remain
      asm volatile("s_waitcnt vmcnt(%0)" :: "n"((R - 1) * NA) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    uint4 x = ring[wave][slot][0][lane];
#pragma unroll
    for (int k = 1; k < NA; ++k) xr(x, ring[wave][slot][k][lane]);
    const size_t i = s0 + t * 64 + lane;
    if (i < e0) out[i] = x;
    __builtin_amdgcn_wave_barrier();
  }
}

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 20;
  for (size_t W : {(size_t)1 << 20, (size_t)1 << 24}) {
    uint4* buf;
    uint4* out;
    CK(hipMalloc(&buf, (size_t)NA * W * 16));
    CK(hipMalloc(&out, W * 16));
    CK(hipMemset(buf, 0x5A, (size_t)NA * W * 16));
    // a second set of inputs, read between timed launches so every launch
    // starts from HBM (not the Infinity Cache), as in the bench's steps
    uint4* flush;
    const size_t fl = (size_t)512 << 20;
    CK(hipMalloc(&flush, fl));
    Arrs in;
    for (int k = 0; k < NA; ++k) in.a[k] = buf + (size_t)k * W;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const double bytes = (double)(NA + 1) * 16 * W;
    auto run = [&](const char* name, auto launch) {
      std::vector<float> ts;
      for (int r = 0; r < reps + 3; ++r) {
        CK(hipMemsetAsync(flush, r, fl, 0));
        CK(hipEventRecord(e0, 0));
        launch();
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (r >= 3) ts.push_back(ms);
      }
      CK(hipGetLastError());
      std::sort(ts.begin(), ts.end());
      const float med = ts[ts.size() / 2];
      printf("  %-34s median %9.2f us  min %9.2f us  %7.1f GB/s\n", name, med * 1e3, ts[0] * 1e3,
             bytes / (med * 1e-3) / 1e9);
    };
    printf("W=%zu words, %d read arrays + 1 write (%.1f MB)\n", W, NA, bytes / 1e6);
    const unsigned gA = (unsigned)((W + 1023) / 1024);
    run("A probe (word/lane, 1024)", [&] { hipLaunchKernelGGL(kA, dim3(gA), dim3(1024), 0, 0, in, W, out); });
    run("B one contiguous stream", [&] { hipLaunchKernelGGL(kB, dim3(gA), dim3(1024), 0, 0, buf, W, out); });
    run("D glds word/lane, 256", [&] { hipLaunchKernelGGL(kD, dim3(4 * gA), dim3(256), 0, 0, in, W, out); });
    for (unsigned G : {256u, 512u, 1024u}) {
      char nm[64];
      const size_t per = ((W + G - 1) / G + 255) / 256 * 256;
      snprintf(nm, sizeof nm, "E persistent regs bs256 G=%u", G);
      run(nm, [&] { hipLaunchKernelGGL(kE<256>, dim3(G), dim3(256), 0, 0, in, W, per, out); });
      const size_t per2 = ((W + G - 1) / G + 511) / 512 * 512;
      snprintf(nm, sizeof nm, "E persistent regs bs512 G=%u", G);
      run(nm, [&] { hipLaunchKernelGGL(kE<512>, dim3(G), dim3(512), 0, 0, in, W, per2, out); });
    }
    for (unsigned waves : {1024u, 2048u, 4096u}) {
      char nm[64];
      const size_t per = ((W + waves - 1) / waves + 63) / 64 * 64;
      snprintf(nm, sizeof nm, "C glds ring R=2 x4 waves=%u", waves);
      run(nm, [&] { hipLaunchKernelGGL((kC<2, 4>), dim3(waves / 4), dim3(256), 0, 0, in, W, per, out); });
      snprintf(nm, sizeof nm, "C glds ring R=3 x4 waves=%u", waves);
      run(nm, [&] { hipLaunchKernelGGL((kC<3, 4>), dim3(waves / 4), dim3(256), 0, 0, in, W, per, out); });
      snprintf(nm, sizeof nm, "C glds ring R=4 x2 waves=%u", waves);
      run(nm, [&] { hipLaunchKernelGGL((kC<4, 2>), dim3(waves / 2), dim3(128), 0, 0, in, W, per, out); });
      snprintf(nm, sizeof nm, "C glds ring R=2 x2 waves=%u", waves);
      run(nm, [&] { hipLaunchKernelGGL((kC<2, 2>), dim3(waves / 2), dim3(128), 0, 0, in, W, per, out); });
    }
    run("A probe (again)", [&] { hipLaunchKernelGGL(kA, dim3(gA), dim3(1024), 0, 0, in, W, out); });
    CK(hipFree(buf));
    CK(hipFree(out));
    CK(hipFree(flush));
  }
  return 0;
}
