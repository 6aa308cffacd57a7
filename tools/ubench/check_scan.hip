// Check of the decode's DPP workgroup scan (tool): block_excl_scan32 against
// a host prefix sum at every workgroup size the kernels use.
#include "../../amphora_amd/csrc/exchange.hip"
#include <cstdio>
#include <cstdlib>
#include <vector>

__global__ void kt(const uint32_t* in, uint32_t* out, uint32_t* tot) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t t;
  out[i] = amph::block_excl_scan32(in[i], &t);
  if (threadIdx.x == 0) tot[blockIdx.x] = t;
}

int main() {
  int bad = 0;
  for (int bs : {64, 128, 256, 512, 1024}) {
    const int nb = 97;
    const size_t n = (size_t)nb * bs;
    std::vector<uint32_t> h(n), o(n), t(nb);
    srand(bs);
    for (auto& x : h) x = rand() % 33;
    uint32_t *din, *dout, *dt;
    hipMalloc(&din, n * 4); hipMalloc(&dout, n * 4); hipMalloc(&dt, nb * 4);
    hipMemcpy(din, h.data(), n * 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(kt, dim3(nb), dim3(bs), 0, 0, din, dout, dt);
    hipMemcpy(o.data(), dout, n * 4, hipMemcpyDeviceToHost);
    hipMemcpy(t.data(), dt, nb * 4, hipMemcpyDeviceToHost);
    for (int b = 0; b < nb; ++b) {
      uint32_t acc = 0;
      for (int i = 0; i < bs; ++i) {
        if (o[(size_t)b * bs + i] != acc) ++bad;
        acc += h[(size_t)b * bs + i];
      }
      if (t[b] != acc) ++bad;
    }
    hipFree(din); hipFree(dout); hipFree(dt);
  }
  printf("block_excl_scan32: %s (%d mismatches)\n", bad ? "FAIL" : "ok", bad);
  return bad != 0;
}
