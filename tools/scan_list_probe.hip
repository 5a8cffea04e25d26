// scan_list_probe.hip — where the time of the configs[2] scans goes: scan4 at 1,024 queries ×
// 25,216 items, the content width (d = 384, KU 48) and the CF width (r = 50 padded to 64,
// KU 8), with the bounded-list epilogue (kScanList) on a 10 %-dense mask and on an all-ones
// mask, the int16 score image (kScanS16), no epilogue (ABL 1) and MFMA + LDS reads only
// (ABL 7).  Random bf16 operands; medians of 3 rounds of 5 launches.
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 -Iinclude tools/scan_list_probe.hip -o tools/scan_list_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#include "../brickbrain-rec-engine_amd/csrc/scan4_kernel.h"

using namespace bb;

__global__ void fill_bf16(uint16_t* p, size_t n, uint32_t seed) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u ^ seed;
    h ^= h >> 15;
    h *= 2246822519u;
    h ^= h >> 13;
    const float f = ((float)(h & 0xFFFF) / 65536.0f - 0.5f) * 0.1f;
    p[i] = (uint16_t)(__float_as_uint(f) >> 16);
  }
}
__global__ void fill_bits(uint32_t* p, size_t n, uint32_t seed, uint32_t thresh) {  // P(bit) = thresh / 2^16
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint32_t w = 0;
    for (int b = 0; b < 32; ++b) {
      uint32_t h = (uint32_t)(i * 32 + b) * 2654435761u ^ seed;
      h ^= h >> 15;
      h *= 2246822519u;
      h ^= h >> 13;
      w |= ((h & 0xFFFF) < thresh ? 1u : 0u) << b;
    }
    p[i] = w;
  }
}

template <int KU, int ABL>
void l4(const GemmArgs& a, hipStream_t s) {
  const int tiles = a.Ncols / 32;
  const int nc = scan4_n_chunks(a.Mpad, tiles);
  hipLaunchKernelGGL((scan4_kernel<KU, ABL>), dim3(a.Mpad / 256 * nc), dim3(256), 0, s, a, nc, tiles);
}

int main() {
  const int M = 1024;
  for (int cfg = 0; cfg < 3; ++cfg) {
    const int D = cfg == 1 ? 64 : 384, N = cfg == 2 ? 2 * 25216 : 25216, tiles = N / 32;
    uint16_t *q, *x;
    float* S;
    uint32_t *tm, *pm, *ones, *zeros, *mask10, *lists;
    float* sh;
    (void)hipMalloc(&q, (size_t)M * D * 2);
    (void)hipMalloc(&x, (size_t)N * D * 2);
    (void)hipMalloc(&S, (size_t)M * N * 2);
    (void)hipMalloc(&tm, (size_t)M * tiles * 4);
    (void)hipMalloc(&pm, (size_t)M * tiles * 4);
    (void)hipMalloc(&ones, N / 8);
    (void)hipMalloc(&zeros, N / 8);
    (void)hipMalloc(&mask10, N / 8);
    (void)hipMalloc(&sh, M * 4);
    const int nc = scan4_n_chunks(M, tiles), tpc = (tiles + nc - 1) / nc;
    int np = (tpc + kListMaxPeriod - 1) / kListMaxPeriod;
    while (2 * nc * np < 3 * 101 && np < tpc) ++np;
    const int G = (tpc + np - 1) / np;
    np = (tpc + G - 1) / G;
    (void)hipMalloc(&lists, (size_t)nc * np * (M / 32) * 64 * 16);
    hipLaunchKernelGGL(fill_bf16, dim3(4096), dim3(256), 0, 0, q, (size_t)M * D, 1u);
    hipLaunchKernelGGL(fill_bf16, dim3(4096), dim3(256), 0, 0, x, (size_t)N * D, 2u);
    hipLaunchKernelGGL(fill_bits, dim3(64), dim3(256), 0, 0, mask10, (size_t)N / 32, 3u, 6554u);
    (void)hipMemset(ones, 0xFF, N / 8);
    (void)hipMemset(zeros, 0, N / 8);
    {
      std::vector<float> h(M, 1e-4f);
      (void)hipMemcpy(sh, h.data(), M * 4, hipMemcpyHostToDevice);
    }
    GemmArgs a{};
    a.Q = q; a.X = x; a.S = S; a.ldq = a.ldx = D; a.lds = N; a.Mpad = M; a.Ncols = N; a.Kpad = D;
    a.M_valid = M; a.n_valid = N; a.tmax = tm; a.pmax = pm; a.ldt = tiles;
    a.mask = ones; a.present = ones; a.excl = zeros; a.excl_ld = 0; a.s_h = sh;
    a.lists = lists; a.l_period = G; a.l_np = np;
    hipStream_t s;
    (void)hipStreamCreate(&s);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    struct V { const char* name; void (*f)(const GemmArgs&, hipStream_t); bool masked; bool perm = false; };
    std::vector<V> vs;
    if (cfg == 2)
      vs = {{"list_mask10", l4<48, kScanList>, true}, {"no_epi", l4<48, 1>, false},
            {"mfma_lds_only", l4<48, 7>, false}, {"mfma_lds_only_noq", l4<48, 7 | 2048>, false}};
    else if (D == 384)
      vs = {{"list_mask10", l4<48, kScanList>, true}, {"list_ones", l4<48, kScanList>, false},
            {"s16_mask10", l4<48, kScanS16>, true}, {"no_epi", l4<48, 1>, false}, {"mfma_lds_only", l4<48, 7>, false},
            {"mfma_lds_only_noq", l4<48, 7 | 2048>, false}, {"list_noq", l4<48, kScanList | 2048>, true},
            {"mfma_lds_only_qperm", l4<48, 7>, false, true}, {"list_mask10_qperm", l4<48, kScanList>, true, true},
            {"no_epi_qperm", l4<48, 1>, false, true}};
    else
      vs = {{"list_mask10", l4<8, kScanList>, true}, {"list_ones", l4<8, kScanList>, false},
            {"s16_mask10", l4<8, kScanS16>, true}, {"no_epi", l4<8, 1>, false}, {"mfma_lds_only", l4<8, 7>, false}};
    std::vector<std::vector<float>> t(vs.size());
    for (int r = 0; r < 3; ++r)
      for (size_t v = 0; v < vs.size(); ++v) {
        GemmArgs av = a;
        av.mask = vs[v].masked ? mask10 : ones;
        av.q_perm = vs[v].perm ? 1 : 0;  // (operand values differ in layout only: timing probe)
        vs[v].f(av, s);
        hipError_t e = hipStreamSynchronize(s);
        if (e != hipSuccess) {
          printf("{\"variant\":\"%s\",\"exec_error\":\"%s\"}\n", vs[v].name, hipGetErrorString(e));
          return 1;
        }
        (void)hipEventRecord(e0, s);
        for (int i = 0; i < 5; ++i) vs[v].f(av, s);
        (void)hipEventRecord(e1, s);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        t[v].push_back(ms * 1e3f / 5);
      }
    for (size_t v = 0; v < vs.size(); ++v) {
      std::sort(t[v].begin(), t[v].end());
      printf("{\"M\":%d,\"n\":%d,\"d\":%d,\"chunks\":%d,\"periods\":%d,\"G\":%d,\"variant\":\"%s\",\"us_med\":%.1f,"
             "\"tflops\":%.1f}\n", M, N, D, nc, np, G, vs[v].name, t[v][1], 2.0 * M * N * D / (t[v][1] * 1e-6) / 1e12);
      fflush(stdout);
    }
    (void)hipFree(q); (void)hipFree(x); (void)hipFree(S); (void)hipFree(tm); (void)hipFree(pm);
    (void)hipFree(ones); (void)hipFree(zeros); (void)hipFree(mask10); (void)hipFree(sh); (void)hipFree(lists);
  }
  return 0;
}
