// scan4_list_probe.hip — ablations of the configs[2] content list scan (scan4<48, list|f16>:
// 1,024 queries x 25,216 items x 384-d f16, bounded per-lane candidate lists), dense and 2 %
// masks, to find what holds a tile at ~2.4x its MFMA time.  Variants (scan4 ABL bits): full;
// no epilogue (1); no staging after the first tile (2); no per-tile wait + barrier (4);
// MFMA + LDS reads only (7); no query loads (2048).
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 -Iinclude tools/scan4_list_probe.hip -o tools/scan4_list_probe
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#include "../brickbrain-rec-engine_amd/csrc/scan4_kernel.h"

using namespace bb;

__global__ void fill_f16(uint16_t* p, size_t n, uint32_t seed) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u ^ seed;
    h ^= h >> 15;
    h *= 2246822519u;
    h ^= h >> 13;
    const float f = ((float)(h & 0xFFFF) / 65536.0f - 0.5f) * 0.1f;
    p[i] = __builtin_bit_cast(uint16_t, (_Float16)f);
  }
}

template <int KU, int ABL>
void launch(const GemmArgs& a, int nc, int tiles, hipStream_t s, hipEvent_t e0, hipEvent_t e1) {
  hipExtLaunchKernelGGL((scan4_kernel<KU, kScanList | kScanF16 | ABL>), dim3(a.Mpad / 256 * nc), dim3(256), 0, s, e0,
                        e1, 0, a, nc, tiles);
}

// the configs[2] content side (d = 384, KU 48) or, with argument "cf", its CF side (r = 50
// padded to 64, KU 8)
template <int KU>
int run(const char* side) {
  const int M = 1024, N = 25216, D = KU * 8, tiles = (N + 127) / 128 * 4;
  uint16_t *q, *x;
  uint32_t *lists, *ones, *zeros, *mask2;
  float* sh;
  (void)hipMalloc(&q, (size_t)M * D * 2);
  (void)hipMalloc(&x, (size_t)tiles * 32 * D * 2);
  (void)hipMalloc(&lists, (size_t)64 * 8 * (M / 32) * 64 * 16);
  (void)hipMalloc(&ones, tiles * 4 + 64);
  (void)hipMalloc(&zeros, tiles * 4 + 64);
  (void)hipMalloc(&mask2, tiles * 4 + 64);
  (void)hipMalloc(&sh, M * 4);
  hipLaunchKernelGGL(fill_f16, dim3(1024), dim3(256), 0, 0, q, (size_t)M * D, 1u);
  hipLaunchKernelGGL(fill_f16, dim3(4096), dim3(256), 0, 0, x, (size_t)tiles * 32 * D, 2u);
  (void)hipMemset(ones, 0xFF, tiles * 4 + 64);
  (void)hipMemset(zeros, 0, tiles * 4 + 64);
  {
    std::vector<uint32_t> m(tiles + 16, 0u);
    uint32_t r = 12345;
    for (int i = 0; i < tiles * 32; ++i) {
      r = r * 1664525u + 1013904223u;
      if ((r >> 8) % 1000 < 17) m[i >> 5] |= 1u << (i & 31);  // 1.7 % eligible
    }
    (void)hipMemcpy(mask2, m.data(), m.size() * 4, hipMemcpyHostToDevice);
    std::vector<float> h(M, 1e-4f);
    (void)hipMemcpy(sh, h.data(), M * 4, hipMemcpyHostToDevice);
  }
  const int nc = scan4_list_chunks(M, tiles, KU);
  const int tpc = (tiles + nc - 1) / nc;
  GemmArgs a{};
  a.Q = q; a.X = x; a.ldq = a.ldx = D; a.Mpad = M; a.Ncols = tiles * 32; a.Kpad = D;
  a.M_valid = M; a.n_valid = N; a.present = ones; a.excl = zeros; a.excl_ld = 0; a.q_perm = 1;
  a.f16 = 1; a.s_h = sh; a.lists = lists; a.l_period = 8; a.l_np = (tpc + 7) / 8;
  hipStream_t s;
  (void)hipStreamCreate(&s);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  struct V { const char* name; void (*f)(const GemmArgs&, int, int, hipStream_t, hipEvent_t, hipEvent_t); };
  std::vector<V> vs = {{"full", launch<KU, 0>}, {"no_epilogue", launch<KU, 1>}, {"no_staging", launch<KU, 2>},
                       {"no_wait_barrier", launch<KU, 4>}, {"mfma_lds_only", launch<KU, 7>},
                       {"no_query_loads", launch<KU, 2048>}, {"no_epi_no_query_loads", launch<KU, 2048 | 1>},
                       {"mfma_lds_no_query_loads", launch<KU, 2048 | 7>}};
  for (int m = 0; m < 2; ++m) {
    a.mask = m ? mask2 : ones;
    for (auto& v : vs) {
      std::vector<float> t;
      for (int r = 0; r < 12; ++r) {
        v.f(a, nc, tiles, s, e0, e1);
        (void)hipEventSynchronize(e1);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, e0, e1);
        t.push_back(ms * 1e3f);
      }
      if (hipStreamSynchronize(s) != hipSuccess) { printf("{\"error\":\"%s\"}\n", v.name); return 1; }
      std::sort(t.begin(), t.end());
      printf("{\"side\":\"%s\",\"mask\":\"%s\",\"variant\":\"%s\",\"us_p50\":%.2f,\"tflops\":%.0f,\"chunks\":%d}\n", side,
             m ? "1.7%" : "all", v.name, t[6], 2.0 * M * N * D / (t[6] * 1e-6) / 1e12, nc);
      fflush(stdout);
    }
  }
  return 0;
}

int main(int argc, char** argv) {
  if (argc > 1 && argv[1][0] == 'c') return run<8>("cf");
  return run<48>("content");
}
