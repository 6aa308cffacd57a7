// LDS store cost by width and alignment (tool): each lane stores to its own
// entry of a per-workgroup buffer at stride S bytes (90 ~ an exchange-encode
// entry: misaligned; 96: 16-aligned), K times, as the encode's formatter does.
// Prints ns per wave-instruction per CU for each (form, stride).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

constexpr int kBlock = 256, kK = 256;

template <int FORM>
__global__ __launch_bounds__(kBlock) void k_store(int stride, int shift, uint32_t* sink) {
  __shared__ uint4 buf[(kBlock * 100 + 64) / 16];
  char* b = reinterpret_cast<char*>(buf);
  const uint32_t base = threadIdx.x * stride + shift;
  uint32_t o[8], v[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {  // 9-byte steps inside the entry, as digit chunks
    o[j] = base + 9 * j;
    v[j] = (threadIdx.x + j) * 2654435761u;
  }
  // only the stores in the loop: addresses and data stay in registers
  for (int k = 0; k < kK / 8; ++k) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if constexpr (FORM == 0) {  // one byte
        b[o[j]] = (char)v[j];
      } else if constexpr (FORM == 1) {  // 8 bytes, as the formatter's memcpy (alignment unknown)
        const uint64_t x = ((uint64_t)v[j] << 32) | v[(j + 1) & 7];
        __builtin_memcpy(b + o[j], &x, 8);
      } else if constexpr (FORM == 2) {  // 4 bytes at the dword below (aligned)
        reinterpret_cast<uint32_t*>(b)[o[j] >> 2] = v[j];
      } else if constexpr (FORM == 3) {  // atomic OR of a dword (aligned)
        atomicOr(reinterpret_cast<uint32_t*>(b) + (o[j] >> 2), v[j]);
      } else {  // 8 bytes at the 8-aligned address below
        reinterpret_cast<uint64_t*>(b)[o[j] >> 3] = ((uint64_t)v[j] << 32) | v[(j + 1) & 7];
      }
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  __syncthreads();
  if (threadIdx.x == 0) atomicAdd(sink, reinterpret_cast<uint32_t*>(b)[blockIdx.x & 63]);
}

template <int FORM>
float run(int stride, int shift, uint32_t* sink) {
  hipEvent_t a, z;
  hipEventCreate(&a); hipEventCreate(&z);
  const int grid = 256 * 64;
  for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(k_store<FORM>, dim3(grid), dim3(kBlock), 0, 0, stride, shift, sink);
  hipEventRecord(a, 0);
  const int R = 10;
  for (int r = 0; r < R; ++r) hipLaunchKernelGGL(k_store<FORM>, dim3(grid), dim3(kBlock), 0, 0, stride, shift, sink);
  hipEventRecord(z, 0);
  hipEventSynchronize(z);
  float ms; hipEventElapsedTime(&ms, a, z);
  // wave-instructions of the store per CU: grid/256 CUs * 4 waves * kK
  const double per_cu = (double)grid / 256 * (kBlock / 64) * kK * R;
  return (float)(ms * 1e6 / per_cu);
}

int main() {
  uint32_t* sink;
  CK(hipMalloc(&sink, 4));
  const char* names[] = {"b8", "b64-memcpy", "b32-aligned", "or-b32-aligned", "b64-aligned"};
  const int strides[] = {90, 92, 96};
  for (int s : strides) {
    for (int sh = 0; sh < 2; ++sh) {
      float t[5] = {run<0>(s, sh, sink), run<1>(s, sh, sink), run<2>(s, sh, sink), run<3>(s, sh, sink),
                    run<4>(s, sh, sink)};
      printf("{\"stride\": %d, \"shift\": %d", s, sh);
      for (int f = 0; f < 5; ++f) printf(", \"%s_ns\": %.3f", names[f], t[f]);
      printf("}\n");
    }
  }
  return 0;
}
