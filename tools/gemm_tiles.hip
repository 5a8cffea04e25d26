// gemm_tiles.hip — A/B the score-slab GEMM tile shapes in ONE process (interleaved rounds,
// cdna_hip_programming.md §5.4 rule 24).  Prints one JSON line per (dtype, M, variant) with
// the median/min kernel time and TFLOP/s, and checks every variant's S against variant 0.
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 -I../include tools/gemm_tiles.hip -o tools/gemm_tiles
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../brickbrain-rec-engine_amd/csrc/gemm_kernel.h"

using namespace bb;

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e = (x);                                                             \
    if (e != hipSuccess) {                                                          \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
      exit(1);                                                                      \
    }                                                                               \
  } while (0)

struct Variant {
  const char* name;
  int bm, bn, nt;
  void (*launch)(const GemmArgs&, int blocks, hipStream_t);
};

template <typename T, int WM, int WN, int SM, int SN, int RB>
void launch_v(const GemmArgs& a, int blocks, hipStream_t s) {
  hipLaunchKernelGGL((gemm_nt_kernel<T, WM, WN, SM, SN, RB>), dim3(blocks), dim3(WM * WN * 64), 0, s, a);
}

// bm = queries per block (WN*SN*32), bn = items per block (WM*SM*32)
#define V(T, WM, WN, SM, SN, RB)                                                                 \
  Variant {                                                                                      \
    #T "_" #WM "x" #WN "w_" #SM "x" #SN "t_kb" #RB, WN * SN * 32, WM * SM * 32, WM * WN * 64,    \
        launch_v<T, WM, WN, SM, SN, RB>                                                          \
  }

static uint16_t f2bf(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  u += 0x7FFFu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

int main(int argc, char** argv) {
  const int N = 25344, D = 384;  // 25,216 items padded to 128 (and 256)
  const int iters = argc > 1 ? atoi(argv[1]) : 30;
  const int rounds = 5;
  std::vector<int> Ms = {256, 1024, 4096};
  std::vector<Variant> vf = {V(float, 2, 2, 1, 1, 128), V(float, 2, 2, 1, 1, 256), V(float, 2, 2, 2, 2, 128),
                             V(float, 2, 2, 2, 2, 256), V(float, 2, 4, 1, 1, 128), V(float, 2, 4, 1, 1, 256),
                             V(float, 4, 2, 1, 1, 256), V(float, 2, 2, 2, 1, 256), V(float, 2, 2, 1, 2, 256)};
  std::vector<Variant> vb = {V(uint16_t, 2, 2, 2, 2, 128), V(uint16_t, 2, 2, 2, 2, 256), V(uint16_t, 2, 4, 2, 2, 128),
                             V(uint16_t, 4, 2, 2, 2, 128), V(uint16_t, 2, 2, 1, 2, 256), V(uint16_t, 2, 2, 2, 1, 256)};
  const int Mmax = 4096;
  std::vector<float> hq((size_t)Mmax * D), hx((size_t)N * D);
  srand(1);
  for (auto& v : hq) v = (float)rand() / RAND_MAX - 0.5f;
  for (auto& v : hx) v = (float)rand() / RAND_MAX - 0.5f;
  std::vector<uint16_t> bq(hq.size()), bx(hx.size());
  for (size_t i = 0; i < hq.size(); ++i) bq[i] = f2bf(hq[i]);
  for (size_t i = 0; i < hx.size(); ++i) bx[i] = f2bf(hx[i]);
  void *dq, *dx, *dqb, *dxb;
  float *S, *S0;
  CK(hipMalloc(&dq, hq.size() * 4));
  CK(hipMalloc(&dx, hx.size() * 4));
  CK(hipMalloc(&dqb, bq.size() * 2));
  CK(hipMalloc(&dxb, bx.size() * 2));
  CK(hipMalloc(&S, (size_t)Mmax * N * 4));
  CK(hipMalloc(&S0, (size_t)Mmax * N * 4));
  CK(hipMemcpy(dq, hq.data(), hq.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dx, hx.data(), hx.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dqb, bq.data(), bq.size() * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(dxb, bx.data(), bx.size() * 2, hipMemcpyHostToDevice));
  hipStream_t s;
  CK(hipStreamCreate(&s));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));

  for (int dt = 0; dt < 2; ++dt) {
    auto& vs = dt == 0 ? vf : vb;
    for (int M : Ms) {
      GemmArgs a{};
      a.Q = dt == 0 ? dq : dqb;
      a.X = dt == 0 ? dx : dxb;
      a.ldq = a.ldx = D;
      a.lds = N;
      a.Mpad = M;
      a.Ncols = N;
      a.Kpad = D;
      std::vector<std::vector<float>> t(vs.size());
      for (int r = 0; r < rounds; ++r)
        for (size_t v = 0; v < vs.size(); ++v) {
          if (M % vs[v].bm || N % vs[v].bn) continue;
          const int blocks = (M / vs[v].bm) * (N / vs[v].bn);
          a.S = S;
          vs[v].launch(a, blocks, s);  // warm
          CK(hipEventRecord(e0, s));
          for (int i = 0; i < iters; ++i) vs[v].launch(a, blocks, s);
          CK(hipEventRecord(e1, s));
          CK(hipEventSynchronize(e1));
          float ms = 0;
          CK(hipEventElapsedTime(&ms, e0, e1));
          t[v].push_back(1e3f * ms / iters);
          if (r == 0) {
            if (v == 0) CK(hipMemcpy(S0, S, (size_t)M * N * 4, hipMemcpyDeviceToDevice));
          }
        }
      // correctness vs variant 0 (same k order -> bitwise equal expected)
      std::vector<float> h0((size_t)M * N), h1((size_t)M * N);
      CK(hipMemcpy(h0.data(), S0, h0.size() * 4, hipMemcpyDeviceToHost));
      for (size_t v = 0; v < vs.size(); ++v) {
        if (t[v].empty()) continue;
        const int blocks = (M / vs[v].bm) * (N / vs[v].bn);
        a.S = S;
        CK(hipMemsetAsync(S, 0, (size_t)M * N * 4, s));
        vs[v].launch(a, blocks, s);
        CK(hipStreamSynchronize(s));
        CK(hipMemcpy(h1.data(), S, h1.size() * 4, hipMemcpyDeviceToHost));
        double md = 0;
        for (size_t i = 0; i < h1.size(); ++i) md = std::max(md, (double)std::fabs(h1[i] - h0[i]));
        std::sort(t[v].begin(), t[v].end());
        const double med = t[v][t[v].size() / 2], mn = t[v][0];
        const double tf = 2.0 * M * N * D / (med * 1e-6) / 1e12;
        printf("{\"dtype\":\"%s\",\"M\":%d,\"variant\":\"%s\",\"us_med\":%.2f,\"us_min\":%.2f,\"tflops\":%.1f,"
               "\"maxdiff_vs_v0\":%.3g}\n",
               dt == 0 ? "f32" : "bf16", M, vs[v].name, med, mn, tf, md);
      }
      fflush(stdout);
    }
  }
  return 0;
}
