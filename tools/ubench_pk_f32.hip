// Microbenchmark: issue rate of packed FP32 (v_pk_mul_f32 / v_pk_add_f32) vs scalar v_mul_f32
// on gfx950. Informs whether the slab test should be written with float2 math.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float float2_t __attribute__((ext_vector_type(2)));

template <int MODE>
__global__ __launch_bounds__(256) void k(float* out, float s, int iters) {
  float a0 = threadIdx.x * 1e-3f, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  float2_t p0 = {a0, a1}, p1 = {a2, a3}, p2 = {a4, a5}, p3 = {a6, a7};
  float2_t ss = {s, s};
  for (int i = 0; i < iters; ++i) {
    if (MODE == 0) {  // 8 independent scalar muls
      a0 *= s; a1 *= s; a2 *= s; a3 *= s; a4 *= s; a5 *= s; a6 *= s; a7 *= s;
    } else if (MODE == 1) {  // 4 packed muls = 8 flops
      p0 *= ss; p1 *= ss; p2 *= ss; p3 *= ss;
    } else {  // 4 packed adds
      p0 += ss; p1 += ss; p2 += ss; p3 += ss;
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + p0.x + p0.y + p1.x + p1.y + p2.x + p2.y + p3.x + p3.y;
}

int main() {
  float* out;
  hipMalloc(&out, 256 * 8192 * 4);
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  const int iters = 20000, blocks = 256 * 8;
  for (int mode = 0; mode < 3; ++mode) {
    for (int rep = 0; rep < 2; ++rep) {
      hipEventRecord(a);
      if (mode == 0) hipLaunchKernelGGL(k<0>, dim3(blocks), dim3(256), 0, 0, out, 0.999f, iters);
      if (mode == 1) hipLaunchKernelGGL(k<1>, dim3(blocks), dim3(256), 0, 0, out, 0.999f, iters);
      if (mode == 2) hipLaunchKernelGGL(k<2>, dim3(blocks), dim3(256), 0, 0, out, 0.999f, iters);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      double lane_flops = 8.0 * iters * blocks * 256;
      if (rep) printf("mode %d (%s): %.3f ms, %.1f T lane-flop/s\n", mode, mode == 0 ? "v_mul_f32 x8" : (mode == 1 ? "v_pk_mul_f32 x4" : "v_pk_add_f32 x4"), ms, lane_flops / ms / 1e9);
    }
  }
  return 0;
}
