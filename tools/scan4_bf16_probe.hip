// scan4_bf16_probe.hip — the bf16 scan kernels at the 25,216-item shape without / with their
// score-slab stores (ABL 8 = no S stores, the maxima-only pass of a two-pass bound), for the
// content width (KU 48, 384-d) and the CF width (KU 8, r = 50 padded to 64):
//   scan2 (M = 256) and scan4 (M = 1024, 4096).
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 -Iinclude tools/scan4_bf16_probe.hip -o tools/scan4_bf16_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#include "../brickbrain-rec-engine_amd/csrc/scan4_kernel.h"

using namespace bb;

template <int KU, int ABL>
void l4(const GemmArgs& a, hipStream_t s) {
  const int tiles = a.Ncols / 32, n_chunks = scan4_n_chunks(a.Mpad, tiles);
  hipLaunchKernelGGL((scan4_kernel<KU, ABL>), dim3(a.Mpad / kScan4Queries * n_chunks), dim3(kScanWaves * 64), 0, s, a,
                     n_chunks, tiles);
}
template <int KU, int ABL>
void l2(const GemmArgs& a, hipStream_t s) {
  const int tiles = a.Ncols / 32, n_chunks = scan_n_chunks(a.Mpad, tiles);
  hipLaunchKernelGGL((scan2_kernel<uint16_t, KU, ABL>), dim3(a.Mpad / 128 * n_chunks), dim3(256), 0, s, a, n_chunks,
                     tiles);
}

int main() {
  const int N = 25216;
  struct C { const char* name; int M, D; void (*full)(const GemmArgs&, hipStream_t); void (*noS)(const GemmArgs&, hipStream_t); };
  std::vector<C> cs = {{"scan2_d384", 256, 384, l2<48, 0>, l2<48, 8>},   {"scan2_d64", 256, 64, l2<8, 0>, l2<8, 8>},
                       {"scan4_d384", 1024, 384, l4<48, 0>, l4<48, 8>}, {"scan4_d64", 1024, 64, l4<8, 0>, l4<8, 8>},
                       {"scan4_d384", 4096, 384, l4<48, 0>, l4<48, 8>}};
  for (auto& c : cs) {
    const int M = c.M, D = c.D;
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
    std::vector<float> tf, tn;
    for (int r = 0; r < 7; ++r)
      for (int v = 0; v < 2; ++v) {
        auto f = v ? c.noS : c.full;
        f(a, s);
        hipError_t e = hipGetLastError();
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        if (e != hipSuccess) { printf("{\"case\":\"%s\",\"error\":\"%s\"}\n", c.name, hipGetErrorString(e)); return 1; }
        (void)hipEventRecord(e0, s);
        for (int i = 0; i < 10; ++i) f(a, s);
        (void)hipEventRecord(e1, s);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        (v ? tn : tf).push_back(ms * 1e3f / 10);
      }
    std::sort(tf.begin(), tf.end());
    std::sort(tn.begin(), tn.end());
    printf("{\"case\":\"%s\",\"M\":%d,\"D\":%d,\"full_us\":%.2f,\"no_S_us\":%.2f,\"tflops_noS\":%.1f}\n", c.name, M, D,
           tf[3], tn[3], 2.0 * M * N * D / (tn[3] * 1e-6) / 1e12);
    (void)hipFree(q); (void)hipFree(x); (void)hipFree(S); (void)hipFree(tm); (void)hipFree(pm);
    (void)hipFree(ones); (void)hipFree(zeros);
  }
  return 0;
}
