// Exhaustive check of the device reciprocal used by the OBB slab (art_device_fns.hpp rcp_rn):
// for every float bit pattern whose exponent field lies in the fast range [3, 251], rcp_rn(x) must
// equal the IEEE division 1.0f / x bit for bit. Prints the mismatch count and the first few.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off tools/rcp_check.hip -o /tmp/rcp_check && /tmp/rcp_check
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>

__device__ __forceinline__ float rcp_rn(float x) {
  const float r = __builtin_amdgcn_rcpf(x);
  const float e = __builtin_fmaf(-x, r, 1.0f);
  return __builtin_fmaf(e, r, r);
}

__global__ void check(uint32_t hi, unsigned long long* bad, uint32_t* first) {
  const uint32_t bits = (hi << 24) | (blockIdx.x * 256u + threadIdx.x);
  const float x = __builtin_bit_cast(float, bits);
  const uint32_t ex = (bits >> 23) & 0xffu;
  if (ex < 3u || ex > 251u) return;
  const float a = rcp_rn(x);
  const float b = 1.0f / x;
  if (__builtin_bit_cast(uint32_t, a) != __builtin_bit_cast(uint32_t, b)) {
    const unsigned long long k = atomicAdd(bad, 1ull);
    if (k < 8) first[k] = bits;
  }
}

int main() {
  unsigned long long* bad;
  uint32_t* first;
  hipMalloc(&bad, 8);
  hipMalloc(&first, 32);
  hipMemset(bad, 0, 8);
  for (uint32_t hi = 0; hi < 256; ++hi) hipLaunchKernelGGL(check, dim3(1u << 16), dim3(256), 0, 0, hi, bad, first);
  unsigned long long h = 0;
  uint32_t f[8] = {};
  hipMemcpy(&h, bad, 8, hipMemcpyDeviceToHost);
  hipMemcpy(f, first, 32, hipMemcpyDeviceToHost);
  printf("rcp_rn mismatches over exponents [3, 251]: %llu\n", h);
  for (unsigned long long i = 0; i < h && i < 8; ++i) printf("  0x%08x\n", f[i]);
  return h == 0 ? 0 : 1;
}
