// VALU issue rate (tool): wave-instructions per SIMD-cycle for a few 32-bit
// integer instructions the wire decode is made of (v_perm_b32, v_xad /
// v_add_u32, v_and_or, v_dot4_u32_u8) and the field multiply's v_mad_u64_u32
// and v_mul_lo_u32 against v_fma_f32, at 8 waves per SIMD
// with 8 independent chains per lane, so nothing but the pipe limits issue.
// Reports ns per wave-instruction per SIMD and cycles at the measured clock
// (s_memtime ticks = shader clock, MI355X_MICROARCH.md).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

constexpr int kIters = 4096, kChains = 8;

template <int OP>
__global__ __launch_bounds__(256) void k_rate(unsigned* out, unsigned seed, unsigned long long* ticks) {
  unsigned a[kChains];
  unsigned long long m[kChains];
  float f[kChains];
#pragma unroll
  for (int c = 0; c < kChains; ++c) { a[c] = seed ^ (threadIdx.x * 2654435761u + c); f[c] = (float)a[c]; m[c] = a[c]; }
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < kIters; ++i) {
#pragma unroll
    for (int c = 0; c < kChains; ++c) {
      if constexpr (OP == 0) a[c] = __builtin_amdgcn_perm(a[c], seed, 0x05010400u);
      else if constexpr (OP == 1) a[c] = a[c] + (a[c] ^ seed);   // 2 instructions (v_xor + v_add, or v_xad)
      else if constexpr (OP == 2) a[c] = __builtin_amdgcn_udot4(a[c], 0x01400140u, a[c], false);
      else if constexpr (OP == 3) a[c] = __builtin_amdgcn_alignbit(a[c], a[c] ^ seed, 7);  // v_alignbit_b32 (+ v_xor)
      else if constexpr (OP == 5) m[c] = (unsigned long long)(unsigned)m[c] * seed + m[c];  // v_mad_u64_u32
      else if constexpr (OP == 6) a[c] = a[c] * (a[c] | seed);  // v_or + v_mul_lo_u32
      else f[c] = __builtin_fmaf(f[c], 1.0001f, 0.5f);
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  unsigned r = 0;
#pragma unroll
  for (int c = 0; c < kChains; ++c) r ^= a[c] ^ __float_as_uint(f[c]) ^ (unsigned)m[c] ^ (unsigned)(m[c] >> 32);
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
  if (threadIdx.x == 0 && blockIdx.x == 0) ticks[0] = t1 - t0;
}

template <int OP>
void run(const char* name, int instr_per_op, int cus) {  // 0: half an instruction (packed)
  unsigned* out;
  unsigned long long* ticks;
  const int blocks = cus * 8;  // 8 x 256-lane blocks per CU = 8 waves per SIMD
  CK(hipMalloc(&out, (size_t)blocks * 256 * 4));
  CK(hipMalloc(&ticks, 8));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  hipLaunchKernelGGL(k_rate<OP>, dim3(blocks), dim3(256), 0, 0, out, 12345u, ticks);
  CK(hipEventRecord(e0));
  hipLaunchKernelGGL(k_rate<OP>, dim3(blocks), dim3(256), 0, 0, out, 12345u, ticks);
  CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1));
  unsigned long long t; CK(hipMemcpy(&t, ticks, 8, hipMemcpyDeviceToHost));
  const double per = instr_per_op ? (double)instr_per_op : 0.5;
  const double waves_per_simd = 8.0, instr = (double)kIters * kChains * per * waves_per_simd;
  const double ns_per = ms * 1e6 / instr;  // per wave-instruction per SIMD
  const double ghz = (double)t / (ms * 1e6);  // block 0's ticks over the kernel time (approx. clock)
  printf("{\"op\": \"%s\", \"ns_per_wave_instr_per_simd\": %.4f, \"clock_GHz_est\": %.2f, "
         "\"cycles_per_wave_instr\": %.2f}\n", name, ns_per, ghz, ns_per * ghz);
  CK(hipFree(out)); CK(hipFree(ticks));
}

int main() {
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  // instructions per chain step, as the compiler emits them (ISA checked):
  // fma is SLP-packed into v_pk_fma_f32 (half an instruction per step), the
  // xor-add fuses into v_xad_u32, the rotate is v_xor_b32 + v_alignbit_b32
  run<4>("v_pk_fma_f32 (2 fma)", 0, cus);
  run<0>("v_perm_b32", 1, cus);
  run<1>("v_xad_u32", 1, cus);
  run<2>("v_dot4_u32_u8", 1, cus);
  run<3>("v_xor_b32+v_alignbit_b32", 2, cus);
  run<5>("v_mad_u64_u32", 1, cus);
  run<6>("v_or_b32+v_mul_lo_u32", 2, cus);
  return 0;
}
