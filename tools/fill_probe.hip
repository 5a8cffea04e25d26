// fill_probe.hip — how many independent VALU ops fit in the issue shadow of one
// v_mfma_f32_32x32x2_f32 (one wave per SIMD, one accumulator chain, operands in regs).
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/fill_probe.hip -o tools/fill_probe
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int NV, bool ACCV>
__global__ __launch_bounds__(256) void probe(float* out, int iters, float seed) {
  f32x16 acc;
  for (int g = 0; g < 16; ++g) acc[g] = 0.f;
  float a = seed * (threadIdx.x + 1), b = seed * 0.5f;
  float f[16];
  for (int j = 0; j < 16; ++j) f[j] = seed * j;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      if constexpr (ACCV)
        asm volatile("v_mfma_f32_32x32x2_f32 %0, %1, %2, %0" : "+v"(acc) : "v"(a), "v"(b));
      else
        asm volatile("v_mfma_f32_32x32x2_f32 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
#pragma unroll
      for (int j = 0; j < NV; ++j) asm volatile("v_add_f32 %0, %0, %1" : "+v"(f[j % 16]) : "v"(b));
    }
  }
  float s = 0.f;
  for (int g = 0; g < 16; ++g) s += acc[g] + f[g];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int NV, bool ACCV>
void run(float* out) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const int iters = 400, blocks = 256;
  hipLaunchKernelGGL((probe<NV, ACCV>), dim3(blocks), dim3(256), 0, 0, out, 5, 1.0f);
  (void)hipDeviceSynchronize();
  (void)hipEventRecord(e0, 0);
  hipLaunchKernelGGL((probe<NV, ACCV>), dim3(blocks), dim3(256), 0, 0, out, iters, 1.0f);
  (void)hipEventRecord(e1, 0);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  const double mfmas = (double)iters * 16;
  printf("{\"valu_per_gap\":%d,\"acc_in_vgpr\":%d,\"ns_per_mfma\":%.3f}\n", NV, (int)ACCV, ms * 1e6 / mfmas);
}

int main() {
  float* out;
  (void)hipMalloc(&out, 1024 * 256 * 4);
  run<0, false>(out);
  run<4, false>(out);
  run<8, false>(out);
  run<12, false>(out);
  run<16, false>(out);
  run<24, false>(out);
  run<0, true>(out);
  run<8, true>(out);
  run<12, true>(out);
  run<16, true>(out);
  return 0;
}
