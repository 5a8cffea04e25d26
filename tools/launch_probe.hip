// launch_probe.hip — fixed costs of small kernels on this box: empty kernel, one dependent
// global load per thread (fresh buffer / L2-warm buffer), and a kernel reading data that
// the previous kernel wrote.  Each variant: 200 back-to-back launches timed with hipEvents
// (per-launch average) plus one isolated launch.
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/launch_probe.hip -o tools/launch_probe
#include <hip/hip_runtime.h>

#include <cstdio>

__global__ void k_empty(float* out) {
  if (threadIdx.x == 1023) out[0] = 1.f;
}
__global__ void k_load(const float* in, float* out, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = in[i] * 2.f;
}
__global__ void k_chain(const float* in, float* out, int n, int hops) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  float acc = 0.f;
  int j = i % n;
  for (int h = 0; h < hops; ++h) {
    const float v = in[j];
    acc += v;
    j = (j + 4099 * (1 + (int)v)) % n;
  }
  out[i] = acc;
}
__global__ void k_write(float* buf, int n, float v) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) buf[i] = v + i;
}

template <typename F>
void timeit(const char* name, F launch) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  for (int i = 0; i < 20; ++i) launch();
  (void)hipDeviceSynchronize();
  (void)hipEventRecord(a, 0);
  for (int i = 0; i < 200; ++i) launch();
  (void)hipEventRecord(b, 0);
  (void)hipEventSynchronize(b);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, a, b);
  float one = 0;
  (void)hipEventRecord(a, 0);
  launch();
  (void)hipEventRecord(b, 0);
  (void)hipEventSynchronize(b);
  (void)hipEventElapsedTime(&one, a, b);
  printf("{\"probe\":\"%s\",\"us_per_launch_b2b\":%.3f,\"us_single\":%.3f}\n", name, ms * 1e3 / 200, one * 1e3);
}

int main() {
  const int n = 256 * 384;
  float *in, *out, *big;
  (void)hipMalloc(&in, n * 4);
  (void)hipMalloc(&out, (size_t)64 << 20);
  (void)hipMalloc(&big, (size_t)64 << 20);
  (void)hipMemset(in, 0, n * 4);
  timeit("empty_256wg", [&] { hipLaunchKernelGGL(k_empty, dim3(256), dim3(256), 0, 0, out); });
  timeit("empty_1wg", [&] { hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, 0, out); });
  timeit("load_98K", [&] { hipLaunchKernelGGL(k_load, dim3(n / 256), dim3(256), 0, 0, in, out, n); });
  timeit("chain4_98K", [&] { hipLaunchKernelGGL(k_chain, dim3(n / 256), dim3(256), 0, 0, in, out, n, 4); });
  timeit("chain16_98K", [&] { hipLaunchKernelGGL(k_chain, dim3(n / 256), dim3(256), 0, 0, in, out, n, 16); });
  // write 26 MB then read a slice of it in the next kernel (producer -> consumer)
  const int nb = 26 << 18;
  timeit("write26MB+load", [&] {
    hipLaunchKernelGGL(k_write, dim3(nb / 256), dim3(256), 0, 0, big, nb, 1.f);
    hipLaunchKernelGGL(k_load, dim3(n / 256), dim3(256), 0, 0, big, out, n);
  });
  timeit("write26MB", [&] { hipLaunchKernelGGL(k_write, dim3(nb / 256), dim3(256), 0, 0, big, nb, 1.f); });
  return 0;
}
