// percu_probe.hip — per-CU operand delivery rate: 256 workgroups (one per CU) each stream a
// private region of X bytes of a buffer that sits in the MALL / L2 (read twice before timing),
// (a) with plain 16-B vector loads into registers, (b) with LDS-DMA (global_load_lds_dwordx4,
// the scans' staging path) into a two-deep 16-KiB ring.  Reports bytes per CU per µs, which
// prices bench.py's operand-delivery floor of the configs[1] scan (2·√(B·N/P)·d·2 B per CU).
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/percu_probe.hip -o tools/percu_probe
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <algorithm>
#include <cstdio>
#include <vector>

__global__ __launch_bounds__(256) void k_vec(const uint4* __restrict__ src, size_t per_wg, uint32_t* out, int share) {
  const uint4* p = src + (size_t)(blockIdx.x / share) * (per_wg / 16);
  const int n = (int)(per_wg / 16);
  uint32_t acc = 0;
  int i = threadIdx.x;
  for (; i + 3 * 256 < n; i += 4 * 256) {
    const uint4 a = p[i], b = p[i + 256], c = p[i + 512], d = p[i + 768];
    acc ^= a.x ^ b.y ^ c.z ^ d.w;
  }
  for (; i < n; i += 256) acc ^= p[i].x;
  if (acc == 0x12345678u) out[0] = acc;
}

__global__ __launch_bounds__(256) void k_lds(const char* __restrict__ src, size_t per_wg, uint32_t* out, int share) {
  __shared__ __attribute__((aligned(16))) char ring[2][4096 * 4];
  const char* p = src + (size_t)(blockIdx.x / share) * per_wg;
  const uint32_t base = (uint32_t)(size_t)((__attribute__((address_space(3))) char*)&ring[0][0]);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int pieces = (int)(per_wg / 16384);  // 16 KiB per step: each wave 4 KiB = four 1-KiB pieces
  for (int s = 0; s < pieces; ++s) {
    const int buf = s & 1;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const char* g = p + (size_t)s * 16384 + (wave * 4 + j) * 1024 + lane * 16;
      const uint32_t dst = __builtin_amdgcn_readfirstlane(base + buf * 16384 + (wave * 4 + j) * 1024);
      asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off" ::"s"(dst), "v"(g) : "memory", "m0");
    }
    if (s >= 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0 && ring[0][5] == 0x7f && ring[1][9] == 0x7e) out[0] = 1;
}

int main() {
  const int wgs = 256;
  const size_t maxb = (size_t)1 << 20;
  char* buf;
  uint32_t* out;
  (void)hipMalloc(&buf, maxb * wgs);
  (void)hipMalloc(&out, 64);
  (void)hipMemset(buf, 1, maxb * wgs);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  // share = consecutive workgroups reading the same region (8: an XCD's eight CUs under the
  // round-robin placement do NOT share; consecutive blockIdx land on different XCDs, so share 8
  // spreads each region over all XCDs' L2s — the MALL serves it once per XCD)
  for (int share : {1, 8, 64})
  for (size_t per : {65536ul, 262144ul, 1048576ul}) {
    for (int variant = 0; variant < 2; ++variant) {
      // kernel-accurate times: the launch carries the events (the dispatch's own begin / end)
      auto runx = [&](hipEvent_t e0, hipEvent_t e1) {
        if (variant == 0) hipExtLaunchKernelGGL(k_vec, dim3(wgs), dim3(256), 0, 0, e0, e1, 0, (const uint4*)buf, per, out, share);
        else hipExtLaunchKernelGGL(k_lds, dim3(wgs), dim3(256), 0, 0, e0, e1, 0, (const char*)buf, per, out, share);
      };
      auto run = [&] { runx(nullptr, nullptr); };
      for (int i = 0; i < 3; ++i) run();
      (void)hipDeviceSynchronize();
      std::vector<float> t;
      for (int r = 0; r < 50; ++r) {
        runx(a, b);
        (void)hipEventSynchronize(b);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, a, b);
        t.push_back(ms * 1e3f);
      }
      std::sort(t.begin(), t.end());
      const float us = t[t.size() / 2];
      printf("{\"variant\":\"%s\",\"share\":%d,\"bytes_per_cu\":%zu,\"us_p50\":%.2f,\"bytes_per_cu_per_us\":%.0f,"
             "\"chip_gbs\":%.0f}\n", variant ? "lds_dma" : "vector_loads", share, per, us, per / us,
             per * wgs / us / 1e3);
    }
  }
  return 0;
}
