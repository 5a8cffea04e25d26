// mfma_probe.hip — measure v_mfma_f32_32x32x2_f32 / v_mfma_f32_32x32x16_bf16 throughput with
// 1, 2 and 4 independent accumulator chains per wave, operands in registers (no memory in
// the loop).  One workgroup of 4 waves per CU, 256 workgroups.  Prints TFLOP/s per variant.
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/mfma_probe.hip -o tools/mfma_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short bf16x8 __attribute__((ext_vector_type(8)));

template <int NACC, bool BF16>
__global__ __launch_bounds__(256) void probe(float* out, int iters, float seed) {
  f32x16 acc[NACC];
#pragma unroll
  for (int c = 0; c < NACC; ++c)
#pragma unroll
    for (int g = 0; g < 16; ++g) acc[c][g] = 0.f;
  float a = seed * (threadIdx.x + 1), b = seed * 0.5f;
  bf16x8 va, vb;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    va[j] = (short)(threadIdx.x * 7 + j);
    vb[j] = (short)(threadIdx.x * 3 + j);
  }
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int s = 0; s < 16; ++s) {
#pragma unroll
      for (int c = 0; c < NACC; ++c) {
        if constexpr (BF16)
          acc[c] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(va, vb, acc[c], 0, 0, 0);
        else
          acc[c] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[c], 0, 0, 0);
      }
    }
  }
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < NACC; ++c)
#pragma unroll
    for (int g = 0; g < 16; ++g) s += acc[c][g];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int NACC, bool BF16>
void run(float* out, int blocks) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const int iters = 200;
  hipLaunchKernelGGL((probe<NACC, BF16>), dim3(blocks), dim3(256), 0, 0, out, 5, 1.0f);
  (void)hipDeviceSynchronize();
  (void)hipEventRecord(e0, 0);
  hipLaunchKernelGGL((probe<NACC, BF16>), dim3(blocks), dim3(256), 0, 0, out, iters, 1.0f);
  (void)hipEventRecord(e1, 0);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  const double mfmas = (double)blocks * 4 * iters * 16 * NACC;
  const double flop_per = BF16 ? 2.0 * 32 * 32 * 16 : 2.0 * 32 * 32 * 2;
  printf("{\"probe\":\"%s\",\"nacc\":%d,\"blocks\":%d,\"ms\":%.3f,\"tflops\":%.1f,\"cycles_per_mfma_at_2.4GHz\":%.1f}\n",
         BF16 ? "bf16_32x32x16" : "f32_32x32x2", NACC, blocks, ms, mfmas * flop_per / (ms * 1e-3) / 1e12,
         (ms * 1e-3 * 2.4e9) / (mfmas / (blocks * 4.0) / (blocks / 256.0 > 1 ? blocks / 256.0 : 1)));
}

int main() {
  float* out;
  (void)hipMalloc(&out, 1024 * 256 * 4);
  for (int blocks : {256, 512}) {
    run<1, false>(out, blocks);
    run<2, false>(out, blocks);
    run<4, false>(out, blocks);
    run<1, true>(out, blocks);
    run<2, true>(out, blocks);
    run<4, true>(out, blocks);
  }
  return 0;
}
