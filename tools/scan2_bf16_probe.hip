// scan2_bf16_probe.hip — ablations of scan2_kernel<uint16_t, 48> (the one-product bf16 scan
// of the f32 re-rank path) at the configs[1] shape: M query rows x 25,216 items x 384-d,
// interleaved rounds in one process.  ABL bits (scan2_kernel.h): 1 no epilogue, 2 no
// staging after the first tile, 8 no S stores, 16 no tile-maxima stores, 32 no maxima math.
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 -Iinclude tools/scan2_bf16_probe.hip -o tools/scan2_bf16_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#include "../brickbrain-rec-engine_amd/csrc/scan2_kernel.h"

using namespace bb;

template <int ABL>
void launch2(const GemmArgs& a, int n_chunks, int tiles, hipStream_t s) {
  const int n_groups = a.Mpad / 128;
  hipLaunchKernelGGL((scan2_kernel<uint16_t, 48, ABL>), dim3(n_groups * n_chunks), dim3(256), 0, s, a, n_chunks, tiles);
}

int main() {
  const int N = 25216, D = 384;
  for (int M : {128, 256}) {
    uint16_t *q, *x;
    float* S;
    uint32_t *tm, *pm, *ones, *zeros;
    (void)hipMalloc(&q, (size_t)M * D * 2);
    (void)hipMalloc(&x, (size_t)N * D * 2);
    (void)hipMalloc(&S, (size_t)M * N * 4);
    (void)hipMalloc(&tm, (size_t)M * N / 32 * 4);
    (void)hipMalloc(&pm, (size_t)M * N / 32 * 4);
    (void)hipMalloc(&ones, N / 8);
    (void)hipMalloc(&zeros, N / 8);
    (void)hipMemset(q, 0x3c, (size_t)M * D * 2);
    (void)hipMemset(x, 0x3b, (size_t)N * D * 2);
    (void)hipMemset(ones, 0xFF, N / 8);
    (void)hipMemset(zeros, 0, N / 8);
    GemmArgs a{};
    a.Q = q; a.X = x; a.S = S; a.ldq = a.ldx = D; a.lds = N; a.Mpad = M; a.Ncols = N; a.Kpad = D;
    a.M_valid = M; a.n_valid = N; a.tmax = tm; a.pmax = pm; a.ldt = N / 32;
    a.mask = ones; a.present = ones; a.excl = zeros; a.excl_ld = 0;
    hipStream_t s;
    (void)hipStreamCreate(&s);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    struct V { const char* name; void (*f)(const GemmArgs&, int, int, hipStream_t); };
    std::vector<V> vs = {{"full", launch2<0>}, {"no_S", launch2<8>}, {"no_max_store", launch2<16>},
                         {"no_S_no_max", launch2<8 | 16 | 32>}, {"no_epilogue", launch2<1>},
                         {"no_staging", launch2<2>}, {"mfma_lds_only", launch2<7>}};
    const int tiles = N / 32, chunks = scan_n_chunks(M, tiles);
    std::vector<std::vector<float>> t(vs.size());
    for (int r = 0; r < 7; ++r)
      for (size_t v = 0; v < vs.size(); ++v) {
        vs[v].f(a, chunks, tiles, s);
        hipError_t e = hipGetLastError();
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        if (e != hipSuccess) { printf("{\"variant\":\"%s\",\"error\":\"%s\"}\n", vs[v].name, hipGetErrorString(e)); return 1; }
        (void)hipEventRecord(e0, s);
        for (int i = 0; i < 20; ++i) vs[v].f(a, chunks, tiles, s);
        (void)hipEventRecord(e1, s);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        t[v].push_back(ms * 1e3f / 20);
      }
    for (size_t v = 0; v < vs.size(); ++v) {
      std::sort(t[v].begin(), t[v].end());
      printf("{\"M\":%d,\"n_chunks\":%d,\"variant\":\"%s\",\"us_med\":%.2f,\"tflops\":%.1f}\n", M, chunks, vs[v].name,
             t[v][3], 2.0 * M * N * D / (t[v][3] * 1e-6) / 1e12);
    }
    (void)hipFree(q); (void)hipFree(x); (void)hipFree(S); (void)hipFree(tm); (void)hipFree(pm);
    (void)hipFree(ones); (void)hipFree(zeros);
  }
  return 0;
}
