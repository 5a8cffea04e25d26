// scan4_probe.hip — ablations of the bf16 scans (scan2: 32 queries per wave, scan4: 64) on a
// configs[3]-like slab: 4096 queries × 131,072 items × {768, 384}-d bf16, random operands
// (the clock a bf16 MFMA loop holds depends on the data), interleaved rounds in one process.
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 -Iinclude tools/scan4_probe.hip -o tools/scan4_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
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

static int g_chunks = 0;
template <int KU, int ABL>
void l4(const GemmArgs& a, hipStream_t s) {
  const int tiles = a.Ncols / 32;
  const int nc = g_chunks ? g_chunks : scan4_n_chunks(a.Mpad, tiles);
  hipLaunchKernelGGL((scan4_kernel<KU, ABL>), dim3(a.Mpad / 256 * nc), dim3(256), 0, s, a, nc, tiles);
}
static uint64_t *g_thr_none, *g_thr_real;
template <int KU, int REAL, int ABL = 0>
void l4s(const GemmArgs& a0, hipStream_t s) {
  GemmArgs a = a0;
  a.thr_keys = REAL ? g_thr_real : g_thr_none;
  l4<KU, kScanStream | ABL>(a, s);
}
template <int KU, int ABL>
void l2(const GemmArgs& a, hipStream_t s) {
  const int tiles = a.Ncols / 32;
  const int nc = scan_n_chunks(a.Mpad, tiles);
  hipLaunchKernelGGL((scan2_kernel<uint16_t, KU, ABL>), dim3(a.Mpad / 128 * nc), dim3(256), 0, s, a, nc, tiles);
}

int main(int argc, char** argv) {
  const int M = 4096;
  const char* only = argc > 1 ? argv[1] : "0123";  // configs to run (e.g. "02")
  for (int cfg = 0; cfg < 4; ++cfg) {
    if (!strchr(only, '0' + cfg)) continue;
    const int D = cfg == 1 || cfg == 3 ? 384 : 768;
    // cfg 2: items far beyond the MALL (1.6 GB); cfg 3: the d = 384 streaming scan (configs[4]'s)
    const int N = cfg >= 2 ? 1048576 : 131072;
    uint16_t *q, *x;
    float* S;
    uint32_t *tm, *pm, *ones, *zeros;
    (void)hipMalloc(&q, (size_t)M * D * 2);
    (void)hipMalloc(&x, (size_t)N * D * 2);
    (void)hipMalloc(&S, (size_t)M * 131072 * 4);  // cfg 2 runs store-free variants only
    (void)hipMalloc(&tm, (size_t)M * N / 32 * 4);
    (void)hipMalloc(&pm, (size_t)M * N / 32 * 4);
    (void)hipMalloc(&ones, N / 8);
    (void)hipMalloc(&zeros, N / 8);
    hipLaunchKernelGGL(fill_bf16, dim3(4096), dim3(256), 0, 0, q, (size_t)M * D, 1u);
    hipLaunchKernelGGL(fill_bf16, dim3(4096), dim3(256), 0, 0, x, (size_t)N * D, 2u);
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
    struct V { const char* name; void (*f)(const GemmArgs&, hipStream_t); int chunks; };
    std::vector<V> vs;
    // streaming epilogue: one bound key per query (thr_ld 1); "nohit" = a bound no score
    // reaches, "real" = a bound ~0.2 % of the random scores reach (~2K candidates per query,
    // the K·n/n0 of configs[3])
    uint64_t *thr_none, *thr_real, *cand;
    uint32_t* cand_cnt;
    const int cap = 4 * 2048 / 32 + 32;
    (void)hipMalloc(&thr_none, M * 8);
    (void)hipMalloc(&thr_real, M * 8);
    (void)hipMalloc(&cand, (size_t)M * 32 * cap * 8);
    (void)hipMalloc(&cand_cnt, (size_t)M * 32 * 4);
    {
      std::vector<uint64_t> h(M, 0xFFFFFFFF00000000ull);
      (void)hipMemcpy(thr_none, h.data(), M * 8, hipMemcpyHostToDevice);
      const uint32_t o = ord_of(D == 384 ? 0.047f : 0.066f);  // ~0.2 % of the random scores reach it
      std::fill(h.begin(), h.end(), (uint64_t)o << 32);
      (void)hipMemcpy(thr_real, h.data(), M * 8, hipMemcpyHostToDevice);
    }
    a.thr_ld = 1;
    a.cand = cand;
    a.cand_cnt = cand_cnt;
    a.cand_cap = cap;
    g_thr_none = thr_none;
    g_thr_real = thr_real;
    if (cfg == 3)
      vs = {{"s4_no_stores", l4<48, 24>, 0}, {"s4_stream_nohit", l4s<48, 0>, 0}, {"s4_stream_real", l4s<48, 1>, 0},
            {"s4_stream_real_noflush", l4s<48, 1, 32>, 0}, {"s4_no_staging", l4<48, 2 | 24>, 0},
            {"s4_mfma_lds_only", l4<48, 7>, 0},
            // ABL 256: the compare slices without their uniform branch
            // ABL 65536: the round-4 weave (compares in slices 1-4, appends in slice 5, one branch each)
            {"s4_stream_nohit_weave", l4s<48, 0, 65536>, 0}, {"s4_stream_real_weave", l4s<48, 1, 65536>, 0},
            {"s4_stream_nohit_noepi", l4s<48, 0, 1>, 0}};
    else if (cfg == 2)
      vs = {{"s4_no_stores", l4<96, 24>, 0}, {"s4_no_stores_c32", l4<96, 24>, 32},
            {"s4_stream_nohit", l4s<96, 0>, 0}, {"s4_stream_real", l4s<96, 1>, 0},
            {"s4_stream_real_noflush", l4s<96, 1, 32>, 0}, {"s4_stream_real_nostore", l4s<96, 1, 64>, 0},
            {"s4_no_staging", l4<96, 2 | 24>, 0},
            // ABL 128: a three-deep LDS ring on the chained schedule (A/B)
            {"s4_no_stores_ring3", l4<96, 24 | 128>, 0}, {"s4_stream_nohit_ring3", l4s<96, 0, 128>, 0},
            {"s4_stream_real_ring3", l4s<96, 1, 128>, 0},
            {"s4_stream_nohit_weave", l4s<96, 0, 65536>, 0}, {"s4_stream_real_weave", l4s<96, 1, 65536>, 0}};  // (scan2 ABL 8|16 still stores the last tile: S is sized for 131072 columns)
    else if (D == 768)
      vs = {{"s4_full", l4<96, 0>, 0}, {"s4_full_ring3", l4<96, 128>, 0}, {"s4_no_stores_ring3", l4<96, 24 | 128>, 0},
            {"s4_no_stores", l4<96, 24>, 0}, {"s4_no_epi", l4<96, 1>, 0},
            {"s4_no_stores_nobarrier", l4<96, 24 | 4>, 0}, {"s4_no_stores_nostage_nobarrier", l4<96, 24 | 4 | 2>, 0},
            {"s4_no_staging", l4<96, 2 | 24>, 0}, {"s4_mfma_lds_only", l4<96, 7>, 0},
            {"s4_no_stores_c32", l4<96, 24>, 32}, {"s4_no_stores_c64", l4<96, 24>, 64},
            {"s2_full", l2<96, 0>, 0}, {"s2_no_epi", l2<96, 1>, 0}, {"s2_mfma_lds_only", l2<96, 7>, 0}};
    else
      vs = {{"s4_full", l4<48, 0>, 0}, {"s4_no_stores", l4<48, 24>, 0}, {"s4_no_epi", l4<48, 1>, 0},
            {"s4_chains_full", l4<48, 1024>, 0}, {"s4_chains_no_stores", l4<48, 24 | 1024>, 0},
            {"s4_chains_mfma_lds_only", l4<48, 7 | 1024>, 0},
            {"s4_no_staging", l4<48, 2 | 24>, 0}, {"s4_mfma_lds_only", l4<48, 7>, 0},
            {"s4_no_stores_c32", l4<48, 24>, 32}, {"s4_no_stores_c64", l4<48, 24>, 64},
            {"s2_full", l2<48, 0>, 0}, {"s2_no_epi", l2<48, 1>, 0}, {"s2_mfma_lds_only", l2<48, 7>, 0}};
    std::vector<std::vector<float>> t(vs.size());
    for (int r = 0; r < 3; ++r)
      for (size_t v = 0; v < vs.size(); ++v) {
        g_chunks = vs[v].chunks;
        vs[v].f(a, s);
        hipError_t e = hipStreamSynchronize(s);
        if (e != hipSuccess) {
          printf("{\"variant\":\"%s\",\"exec_error\":\"%s\"}\n", vs[v].name, hipGetErrorString(e));
          return 1;
        }
        (void)hipEventRecord(e0, s);
        for (int i = 0; i < 5; ++i) vs[v].f(a, s);
        (void)hipEventRecord(e1, s);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        t[v].push_back(ms * 1e3f / 5);
      }
    for (size_t v = 0; v < vs.size(); ++v) {
      std::sort(t[v].begin(), t[v].end());
      printf("{\"n\":%d,\"d\":%d,\"variant\":\"%s\",\"us_med\":%.1f,\"tflops\":%.1f}\n", N, D, vs[v].name, t[v][1],
             2.0 * M * N * D / (t[v][1] * 1e-6) / 1e12);
      fflush(stdout);
    }
    (void)hipFree(q); (void)hipFree(x); (void)hipFree(S); (void)hipFree(tm); (void)hipFree(pm);
    (void)hipFree(ones); (void)hipFree(zeros);
  }
  return 0;
}
