// scan_probe.hip — ablations of the production scan kernel (C2 shape: 256 queries × 25,344
// items × 384-d f32), interleaved rounds in one process.
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 -Iinclude tools/scan_probe.hip -o tools/scan_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#include "../brickbrain-rec-engine_amd/csrc/scan3_kernel.h"

using namespace bb;

template <int ABL>
void launch(const GemmArgs& a, int n_chunks, int tiles, hipStream_t s) {
  const int n_groups = a.Mpad / 128;
  hipLaunchKernelGGL((scan_kernel<float, 96, ABL>), dim3(n_groups * n_chunks), dim3(256), 0, s, a, n_chunks, tiles);
}

static uint16_t* g_planes = nullptr;
template <int ABL>
void launch3(const GemmArgs& a0, int n_chunks, int tiles, hipStream_t s) {
  GemmArgs a = a0;
  a.X = g_planes;
  a.ldx = 3 * a.Kpad;
  const int n_groups = a.Mpad / 128;
  hipLaunchKernelGGL((scan3_kernel<48, ABL>), dim3(n_groups * n_chunks), dim3(256), 0, s, a, n_chunks, tiles);
}

template <int ABL>
void launch2q(const GemmArgs& a0, int n_chunks, int tiles, hipStream_t s) {
  GemmArgs a = a0;
  a.q_src = a.Q;
  a.q_src_ld = a.ldq;
  a.q_d = a.Kpad;
  a.q_normalize = ABL == 0;
  const int n_groups = a.Mpad / 128;
  hipLaunchKernelGGL((scan2_kernel<float, 96, 0>), dim3(n_groups * n_chunks), dim3(256), 0, s, a, n_chunks, tiles);
}

template <int ABL>
void launch2(const GemmArgs& a, int n_chunks, int tiles, hipStream_t s) {
  const int n_groups = a.Mpad / 128;
  hipLaunchKernelGGL((scan2_kernel<float, 96, ABL>), dim3(n_groups * n_chunks), dim3(256), 0, s, a, n_chunks, tiles);
}

int main() {
  const int N = 25344, D = 384, M = 256;
  float *q, *x, *S;
  uint32_t* tm;
  (void)hipMalloc(&q, (size_t)M * D * 4);
  (void)hipMalloc(&x, (size_t)N * D * 4);
  (void)hipMalloc(&S, (size_t)M * N * 4);
  (void)hipMalloc(&tm, (size_t)M * N / 32 * 4);
  (void)hipMemset(q, 0x3c, (size_t)M * D * 4);
  (void)hipMemset(x, 0x3b, (size_t)N * D * 4);
  GemmArgs a{};
  a.Q = q; a.X = x; a.S = S; a.ldq = a.ldx = D; a.lds = N; a.Mpad = M; a.Ncols = N; a.Kpad = D;
  uint32_t *ones, *zeros, *pm;
  (void)hipMalloc(&ones, N / 8);
  (void)hipMalloc(&zeros, N / 8);
  (void)hipMalloc(&pm, (size_t)M * N / 32 * 4);
  (void)hipMemset(ones, 0xFF, N / 8);
  (void)hipMemset(zeros, 0, N / 8);
  a.M_valid = M; a.n_valid = N; a.tmax = tm; a.pmax = pm; a.ldt = N / 32;
  a.mask = ones; a.present = ones; a.excl = zeros; a.excl_ld = 0;
  hipStream_t s;
  (void)hipStreamCreate(&s);
  (void)hipMalloc(&g_planes, (size_t)N * D * 3 * 2);
  (void)hipMemset(g_planes, 0x3b, (size_t)N * D * 3 * 2);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  struct V { const char* name; void (*f)(const GemmArgs&, int, int, hipStream_t); };
  std::vector<V> vs = {{"full", launch<0>}, {"no_epilogue", launch<1>}, {"no_staging", launch<2>},
                       {"no_barrier", launch<4>}, {"mfma_lds_only", launch<7>},
                       {"v2_full", launch2<0>}, {"v2_no_epilogue", launch2<1>}, {"v2_no_staging", launch2<2>},
                       {"v2_mfma_lds_only", launch2<7>}, {"v2_qsrc_norm", launch2q<0>}, {"v2_qsrc_raw", launch2q<1>},
                       {"v2_no_S", launch2<8>}, {"v2_no_max", launch2<16 | 32>}, {"v2_no_maxstore", launch2<16>},
                       {"v2_only_accread", launch2<8 | 16 | 32>}};
  // (scan3 variants are not run here: its Q-path launches faulted in this harness twice
  //  while tools/scan3_check and the library paths ran clean)
  for (int chunks : {128}) {
    std::vector<std::vector<float>> t(vs.size());
    for (int r = 0; r < 5; ++r)
      for (size_t v = 0; v < vs.size(); ++v) {
        vs[v].f(a, chunks, N / 32, s);
        {
          hipError_t e = hipGetLastError();
          if (e != hipSuccess) printf("{\"variant\":\"%s\",\"launch_error\":\"%s\"}\n", vs[v].name, hipGetErrorString(e));
          e = hipStreamSynchronize(s);
          if (e != hipSuccess) { printf("{\"variant\":\"%s\",\"exec_error\":\"%s\"}\n", vs[v].name, hipGetErrorString(e)); return 1; }
        }
        (void)hipEventRecord(e0, s);
        for (int i = 0; i < 20; ++i) vs[v].f(a, chunks, N / 32, s);
        (void)hipEventRecord(e1, s);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        t[v].push_back(ms * 1e3f / 20);
      }
    for (size_t v = 0; v < vs.size(); ++v) {
      std::sort(t[v].begin(), t[v].end());
      printf("{\"n_chunks\":%d,\"variant\":\"%s\",\"us_med\":%.2f,\"tflops\":%.1f}\n", chunks, vs[v].name,
             t[v][2], 2.0 * M * N * D / (t[v][2] * 1e-6) / 1e12);
    }
  }
  return 0;
}
