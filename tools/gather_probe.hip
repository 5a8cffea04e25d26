// gather_probe.hip — achievable bandwidth of the exact re-rank's row gathers on MI355X.
//
// The re-rank select rescores ~100-200 candidate rows per query from the f32 item matrix
// (1,536 B per 384-d row).  This probe gathers random rows of a resident matrix with the
// select's access pattern (16 lanes per row, float4 chunks p, p+16, ...) and reports GB/s
// for a range of rows in flight per 16-lane group (U) and matrix sizes (MALL-resident
// 38.7 MB vs 4 GB), f32 sums vs f64 sums.  Build: hipcc -O3 --offload-arch=gfx950.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                             \
  do {                                                                                    \
    hipError_t e = (x);                                                                   \
    if (e != hipSuccess) {                                                                \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e));            \
      exit(1);                                                                            \
    }                                                                                     \
  } while (0)

typedef float f4v __attribute__((ext_vector_type(4)));

template <int U, bool F64>
__global__ __launch_bounds__(256) void gather(const float* X, int ld, const int* ids, int per_wg, float* out) {
  const int t = threadIdx.x, p = t & 15, g = t >> 4;
  const int* my = ids + (size_t)blockIdx.x * per_wg;
  float acc_out = 0.f;
  for (int c0 = g * U; c0 < per_wg; c0 += 16 * U) {
    f4v xv[U][6];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int id = c0 + u < per_wg ? my[c0 + u] : my[0];
      const f4v* xr = (const f4v*)(X + (size_t)id * ld);
#pragma unroll
      for (int j = 0; j < 6; ++j) xv[u][j] = xr[p + 16 * j];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if constexpr (F64) {
        double a = 0.0;
#pragma unroll
        for (int j = 0; j < 6; ++j) a += (double)xv[u][j].x + (double)xv[u][j].y + (double)xv[u][j].z + (double)xv[u][j].w;
        acc_out += (float)a;
      } else {
#pragma unroll
        for (int j = 0; j < 6; ++j) acc_out += xv[u][j].x + xv[u][j].y + xv[u][j].z + xv[u][j].w;
      }
    }
  }
  if (acc_out == 12345.f) out[0] = acc_out;  // keep the loads alive
}

template <int U, bool F64>
static double run(const float* X, int ld, const int* ids, int wgs, int per_wg, float* out, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  hipLaunchKernelGGL((gather<U, F64>), dim3(wgs), dim3(256), 0, 0, X, ld, ids, per_wg, out);
  CK(hipEventRecord(a));
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL((gather<U, F64>), dim3(wgs), dim3(256), 0, 0, X, ld, ids, per_wg, out);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms / reps;
}

int main() {
  const int d = 384, ld = 384;
  const size_t rows_big = 2'600'000;  // ~4 GB
  float* X;
  CK(hipMalloc(&X, rows_big * ld * 4));
  CK(hipMemset(X, 0, rows_big * ld * 4));
  float* out;
  CK(hipMalloc(&out, 64));
  for (int wgs : {256, 1024, 2048}) {
    for (int per_wg : {100, 200}) {
      for (size_t n : {(size_t)25216, rows_big}) {
        std::vector<int> h((size_t)wgs * per_wg);
        srand(7);
        for (auto& v : h) v = (int)(((uint64_t)rand() * 2654435761ull) % n);
        int* ids;
        CK(hipMalloc(&ids, h.size() * 4));
        CK(hipMemcpy(ids, h.data(), h.size() * 4, hipMemcpyHostToDevice));
        const double bytes = (double)wgs * per_wg * d * 4;
        const double t2 = run<2, true>(X, ld, ids, wgs, per_wg, out, 20);
        const double t4 = run<4, true>(X, ld, ids, wgs, per_wg, out, 20);
        const double t8 = run<8, true>(X, ld, ids, wgs, per_wg, out, 20);
        const double t4f = run<4, false>(X, ld, ids, wgs, per_wg, out, 20);
        printf("{\"wgs\": %d, \"rows_per_wg\": %d, \"matrix_rows\": %zu, \"MB\": %.1f, \"us_U2\": %.2f, \"us_U4\": %.2f, "
               "\"us_U8\": %.2f, \"us_U4_f32\": %.2f, \"GBs_U2\": %.0f, \"GBs_U4\": %.0f, \"GBs_U8\": %.0f}\n",
               wgs, per_wg, n, bytes / 1e6, t2 * 1e3, t4 * 1e3, t8 * 1e3, t4f * 1e3, bytes / t2 / 1e6, bytes / t4 / 1e6,
               bytes / t8 / 1e6);
        CK(hipFree(ids));
      }
    }
  }
  return 0;
}
