// mfma_bf16_probe.hip — v_mfma_f32_32x32x16_bf16 issue rate on one wave per SIMD:
// one accumulation chain, srcA VGPR, srcB in AGPR or VGPR, with / without ds_read_b128
// fragment loads (3 per 6 MFMAs, as in scan3) in the stream.
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/mfma_bf16_probe.hip -o tools/mfma_bf16_probe
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

template <int MODE>
__global__ __launch_bounds__(256) void probe(float* out, int iters) {
  __shared__ u32x4 lds[4096];
  const int lane = threadIdx.x & 63;
  for (int i = threadIdx.x; i < 4096; i += 256) lds[i] = u32x4{(unsigned)i, 1u, 2u, 3u};
  __syncthreads();
  f32x16 acc = {};
  u32x4 a0 = lds[lane], a1 = lds[lane + 64], a2 = lds[lane + 128];
  u32x4 b0 = u32x4{1u, 2u, 3u, (unsigned)lane}, b1 = b0 + 1u;
  if constexpr (MODE & 1) {
    asm volatile("" : "+a"(b0));
    asm volatile("" : "+a"(b1));
  }
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      if constexpr (MODE & 2) {
        a0 = lds[(lane + s * 64) & 4095];
        a1 = lds[(lane + s * 64 + 1024) & 4095];
        a2 = lds[(lane + s * 64 + 2048) & 4095];
      }
      if constexpr (MODE & 1) {
        asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(acc) : "v"(a0), "a"(b0));
        asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(acc) : "v"(a1), "a"(b0));
        asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(acc) : "v"(a0), "a"(b1));
        asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(acc) : "v"(a2), "a"(b0));
        asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(acc) : "v"(a0), "a"(b1));
        asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(acc) : "v"(a1), "a"(b1));
      } else {
        asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(acc) : "v"(a0), "v"(b0));
        asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(acc) : "v"(a1), "v"(b0));
        asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(acc) : "v"(a0), "v"(b1));
        asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(acc) : "v"(a2), "v"(b0));
        asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(acc) : "v"(a0), "v"(b1));
        asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(acc) : "v"(a1), "v"(b1));
      }
    }
  }
  asm volatile("s_nop 15\n\ts_nop 15\n\ts_nop 15" : "+v"(acc));
  float s = 0.f;
  for (int g = 0; g < 16; ++g) s += acc[g];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int MODE>
void run(float* out, const char* name) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const int iters = 200;
  hipLaunchKernelGGL((probe<MODE>), dim3(256), dim3(256), 0, 0, out, 5);
  (void)hipDeviceSynchronize();
  (void)hipEventRecord(e0, 0);
  hipLaunchKernelGGL((probe<MODE>), dim3(256), dim3(256), 0, 0, out, iters);
  (void)hipEventRecord(e1, 0);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  const double mfmas = (double)iters * 8 * 6;
  printf("{\"variant\":\"%s\",\"ns_per_mfma\":%.3f,\"tflops\":%.0f}\n", name, ms * 1e6 / mfmas,
         256.0 * 4 * mfmas * 32768 / (ms * 1e-3) / 1e12);
}

int main() {
  float* out;
  (void)hipMalloc(&out, 256 * 256 * 4);
  run<0>(out, "srcB_vgpr");
  run<1>(out, "srcB_agpr");
  run<2>(out, "srcB_vgpr+ds_read");
  run<3>(out, "srcB_agpr+ds_read");
  return 0;
}
