// rank_probe.hip — finalize1's rank count in isolation: 1,024 workgroups (one per row), NS
// survivors per row in LDS, every survivor counted against every other (the 16-wide
// ds_read_b128 broadcast loop of finalize_body.h), against variants — how long the count
// itself takes on gfx950, and whether the row's loop or something around it is the cost.
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/rank_probe.hip -o tools/rank_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

template <int NT, int V>
__global__ __launch_bounds__(NT) void rank_kernel(const uint32_t* vals, int ns, int* out) {
  __shared__ __attribute__((aligned(16))) uint32_t sv[512];
  const int q = blockIdx.x, tid = threadIdx.x;
  for (int i = tid; i < ns; i += NT) sv[i] = vals[(size_t)q * 512 + i];
  __syncthreads();
  for (int si = tid; si < ns; si += NT) {
    const uint32_t hh = sv[si];
    int gt = 0, ge = 0, f = 0;
    if constexpr (V == 0) {  // finalize_body.h's loop
      for (; f + 16 <= ns; f += 16) {
        uint32_t kk[16];
#pragma unroll
        for (int j = 0; j < 4; ++j) *(uint4*)(kk + 4 * j) = *(const uint4*)(sv + f + 4 * j);
#pragma unroll
        for (int j = 0; j < 16; ++j) {
          gt += kk[j] > hh;
          ge += kk[j] >= hh;
        }
      }
    } else if constexpr (V == 1) {  // four independent accumulator pairs
      int g1 = 0, g2 = 0, g3 = 0, e1 = 0, e2 = 0, e3 = 0;
      for (; f + 16 <= ns; f += 16) {
        uint32_t kk[16];
#pragma unroll
        for (int j = 0; j < 4; ++j) *(uint4*)(kk + 4 * j) = *(const uint4*)(sv + f + 4 * j);
#pragma unroll
        for (int j = 0; j < 16; j += 4) {
          gt += kk[j] > hh; ge += kk[j] >= hh;
          g1 += kk[j + 1] > hh; e1 += kk[j + 1] >= hh;
          g2 += kk[j + 2] > hh; e2 += kk[j + 2] >= hh;
          g3 += kk[j + 3] > hh; e3 += kk[j + 3] >= hh;
        }
      }
      gt += g1 + g2 + g3;
      ge += e1 + e2 + e3;
    } else {  // gt only (ties found afterwards)
      for (; f + 16 <= ns; f += 16) {
        uint32_t kk[16];
#pragma unroll
        for (int j = 0; j < 4; ++j) *(uint4*)(kk + 4 * j) = *(const uint4*)(sv + f + 4 * j);
#pragma unroll
        for (int j = 0; j < 16; ++j) gt += kk[j] > hh;
      }
      ge = gt + 1;
    }
    for (; f < ns; ++f) {
      gt += sv[f] > hh;
      ge += sv[f] >= hh;
    }
    out[(size_t)q * 512 + si] = gt * 1024 + ge;
  }
}

template <int NT, int V>
float run(const uint32_t* vals, int ns, int* out, hipStream_t s) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  hipLaunchKernelGGL((rank_kernel<NT, V>), dim3(1024), dim3(NT), 0, s, vals, ns, out);
  (void)hipStreamSynchronize(s);
  std::vector<float> t;
  for (int r = 0; r < 20; ++r) {
    (void)hipEventRecord(a, s);
    hipLaunchKernelGGL((rank_kernel<NT, V>), dim3(1024), dim3(NT), 0, s, vals, ns, out);
    (void)hipEventRecord(b, s);
    (void)hipEventSynchronize(b);
    float ms;
    (void)hipEventElapsedTime(&ms, a, b);
    t.push_back(ms * 1e3f);
  }
  std::sort(t.begin(), t.end());
  return t[t.size() / 2];
}

int main() {
  uint32_t* vals;
  int* out;
  (void)hipMalloc(&vals, 1024 * 512 * 4);
  (void)hipMalloc(&out, 1024 * 512 * 4);
  std::vector<uint32_t> h(1024 * 512);
  uint32_t x = 12345;
  for (auto& v : h) { x = x * 1664525u + 1013904223u; v = 0x80000000u | (x >> 1); }
  (void)hipMemcpy(vals, h.data(), h.size() * 4, hipMemcpyHostToDevice);
  hipStream_t s;
  (void)hipStreamCreate(&s);
  for (int ns : {0, 16, 64, 135, 200}) {
    printf("{\"ns\": %d, \"nt128_v0\": %.2f, \"nt128_v1\": %.2f, \"nt128_gt_only\": %.2f, \"nt256_v0\": %.2f, \"nt64_v0\": %.2f}\n", ns,
           run<128, 0>(vals, ns, out, s), run<128, 1>(vals, ns, out, s), run<128, 2>(vals, ns, out, s),
           run<256, 0>(vals, ns, out, s), run<64, 0>(vals, ns, out, s));
    fflush(stdout);
  }
  return 0;
}
