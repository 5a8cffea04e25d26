// scan3_check.hip — one launch per variant of the split-bf16 scan (Q path, q_src path,
// ABL 1), synchronised and checked against an f64 host dot product on sampled entries.
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/scan3_check.hip -o tools/scan3_check
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <algorithm>
#include <vector>

#include "../brickbrain-rec-engine_amd/csrc/scan3_kernel.h"
#include "../brickbrain-rec-engine_amd/csrc/select.hip"

using namespace bb;

static uint16_t rne(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  u += 0x7FFFu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}
static float bf(uint16_t h) {
  uint32_t u = (uint32_t)h << 16;
  float f;
  std::memcpy(&f, &u, 4);
  return f;
}

int main() {
  const int N = 25344, D = 384, M = 256;
  std::vector<float> x((size_t)N * D), q((size_t)M * D);
  uint64_t s = 12345;
  auto rnd = [&]() { s = s * 6364136223846793005ull + 1442695040888963407ull; return ((s >> 33) & 0xFFFFFF) / 16777216.0f - 0.5f; };
  for (auto& v : x) v = rnd();
  for (auto& v : q) v = rnd();
  for (int i = 0; i < N; ++i) {  // unit rows
    double n = 0;
    for (int k = 0; k < D; ++k) n += (double)x[(size_t)i * D + k] * x[(size_t)i * D + k];
    for (int k = 0; k < D; ++k) x[(size_t)i * D + k] = (float)(x[(size_t)i * D + k] / std::sqrt(n));
  }
  for (int i = 0; i < M; ++i) {
    double n = 0;
    for (int k = 0; k < D; ++k) n += (double)q[(size_t)i * D + k] * q[(size_t)i * D + k];
    for (int k = 0; k < D; ++k) q[(size_t)i * D + k] = (float)(q[(size_t)i * D + k] / std::sqrt(n));
  }
  std::vector<uint16_t> qplanes((size_t)M * 3 * D);
  for (int i = 0; i < M; ++i)
    for (int k = 0; k < D; ++k) {
      const float v = q[(size_t)i * D + k];
      const uint16_t h = rne(v);
      const float r = v - bf(h);
      const uint16_t m = rne(r);
      const size_t o = q3f_chunk_offset(i, k >> 3, 0, D / 16) / 2 + (k & 7), pl = (size_t)D / 16 * 512;
      qplanes[o] = h;
      qplanes[o + pl] = m;
      qplanes[o + 2 * pl] = rne(r - bf(m));
    }
  std::vector<uint16_t> planes((size_t)N * 3 * D);
  for (int i = 0; i < N; ++i)
    for (int k = 0; k < D; ++k) {
      const float v = x[(size_t)i * D + k];
      const uint16_t h = rne(v);
      const float r = v - bf(h);
      const uint16_t m = rne(r);
      const uint16_t l = rne(r - bf(m));
      planes[t3_chunk_offset(i, k >> 3, 0, D) / 2 + (k & 7)] = h;
      planes[t3_chunk_offset(i, k >> 3, 1, D) / 2 + (k & 7)] = m;
      planes[t3_chunk_offset(i, k >> 3, 2, D) / 2 + (k & 7)] = l;
    }
  float *dq, *dS;
  uint16_t* dx;
  uint32_t *tm, *pm, *ones, *zeros;
  (void)hipMalloc(&dq, q.size() * 4);
  (void)hipMalloc(&dx, planes.size() * 2);
  (void)hipMalloc(&dS, (size_t)M * N * 4);
  (void)hipMalloc(&tm, (size_t)M * N / 32 * 4);
  (void)hipMalloc(&pm, (size_t)M * N / 32 * 4);
  (void)hipMalloc(&ones, N / 8);
  (void)hipMalloc(&zeros, N / 8);
  uint16_t* dqp;
  (void)hipMalloc(&dqp, qplanes.size() * 2);
  (void)hipMemcpy(dqp, qplanes.data(), qplanes.size() * 2, hipMemcpyHostToDevice);
  (void)hipMemcpy(dq, q.data(), q.size() * 4, hipMemcpyHostToDevice);
  (void)hipMemcpy(dx, planes.data(), planes.size() * 2, hipMemcpyHostToDevice);
  (void)hipMemset(ones, 0xFF, N / 8);
  (void)hipMemset(zeros, 0, N / 8);
  GemmArgs a{};
  a.Q = dqp; a.ldq = 3 * D; a.X = dx; a.ldx = 3 * D; a.S = dS; a.lds = N; a.Mpad = M; a.Ncols = N; a.Kpad = D;
  a.M_valid = M; a.n_valid = N; a.mask = ones; a.present = ones; a.excl = zeros; a.excl_ld = 0;
  a.tmax = tm; a.pmax = pm; a.ldt = N / 32;
  std::vector<float> S((size_t)M * N);
  std::vector<uint32_t> T((size_t)M * N / 32);
  for (int variant = 0; variant < 1; ++variant) {
    (void)hipMemset(dS, 0, (size_t)M * N * 4);
    (void)hipMemset(tm, 0, (size_t)M * N / 32 * 4);
    const int chunks = 128;
    hipLaunchKernelGGL((scan3_kernel<48, 0>), dim3(2 * chunks), dim3(256), 0, 0, a, chunks, N / 32);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = hipDeviceSynchronize();
    if (e != hipSuccess) { printf("{\"variant\":%d,\"error\":\"%s\"}\n", variant, hipGetErrorString(e)); return 1; }
    (void)hipMemcpy(S.data(), dS, S.size() * 4, hipMemcpyDeviceToHost);
    auto SV = [&](int i, int j) { return S[sblk_quad(i, j >> 5, (j >> 2) & 7, N / 32) + (j & 3)]; };
    (void)hipMemcpy(T.data(), tm, T.size() * 4, hipMemcpyDeviceToHost);
    double maxerr = 0;
    for (int i = 0; i < M; i += 7)
      for (int j = 0; j < N; j += 13) {
        double ref = 0;
        for (int k = 0; k < D; ++k) ref += (double)q[(size_t)i * D + k] * x[(size_t)j * D + k];
        maxerr = std::fmax(maxerr, std::fabs(ref - SV(i, j)));
      }
    {
      // locate wrong scores: by tile position inside its workgroup chunk, and by query row
      long nbad = 0, first = 0, last = 0, mid = 0, bad_q[8] = {0};
      const int tiles = N / 32;
      for (int i = 0; i < M; ++i)
        for (int t = 0; t < tiles; ++t) {
          long b = 0;
          for (int j = 0; j < 32; j += 3) {
            const int col = t * 32 + j;
            double ref = 0;
            for (int k = 0; k < D; ++k) ref += (double)q[(size_t)i * D + k] * x[(size_t)col * D + k];
            if (std::fabs(ref - SV(i, col)) > 1e-5) ++b;
          }
          if (!b) continue;
          nbad += b;
          int c = (int)((int64_t)t * chunks / tiles);
          int lo = (int)((int64_t)c * tiles / chunks), hi = (int)((int64_t)(c + 1) * tiles / chunks);
          while (t < lo) { --c; lo = (int)((int64_t)c * tiles / chunks); }
          while (t >= hi) { ++c; hi = (int)((int64_t)(c + 1) * tiles / chunks); lo = (int)((int64_t)c * tiles / chunks); }
          if (t == lo) ++first; else if (t == hi - 1) ++last; else ++mid;
          bad_q[(i % 32) / 4]++;
        }
      printf("{\"bad_elems_sampled\":%ld,\"bad_tiles_first\":%ld,\"mid\":%ld,\"last\":%ld,\"by_q8\":[%ld,%ld,%ld,%ld,%ld,%ld,%ld,%ld]}\n",
             nbad, first, mid, last, bad_q[0], bad_q[1], bad_q[2], bad_q[3], bad_q[4], bad_q[5], bad_q[6], bad_q[7]);
    }
    long bad = 0, lower = 0, zero = 0;
    for (int i = 0; i < M; ++i)
      for (int t = 0; t < N / 32; ++t) {
        float mx = -1e30f;
        for (int j = 0; j < 32; ++j) mx = std::fmax(mx, SV(i, t * 32 + j));
        const uint32_t want = ord_of(mx + 0.0f), got = T[(size_t)i * (N / 32) + t];
        if (got != want) { ++bad; if (got < want) ++lower; if (got == 0) ++zero; }
      }
    printf("{\"variant\":%d,\"ok\":true,\"max_abs_err\":%.3e,\"tmax_bad\":%ld,\"tmax_lower\":%ld,\"tmax_zero\":%ld,\"tiles\":%d}\n",
           variant, maxerr, bad, lower, zero, M * N / 32);
  }
  // timing of ablation variants (20 launches each, after one synchronised check launch)
  auto timeit = [&](const char* name, auto launch) {
    launch();
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = hipDeviceSynchronize();
    if (e != hipSuccess) { printf("{\"timing\":\"%s\",\"error\":\"%s\"}\n", name, hipGetErrorString(e)); return false; }
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0, 0);
    for (int i = 0; i < 20; ++i) launch();
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    printf("{\"timing\":\"%s\",\"us\":%.2f}\n", name, ms * 1e3 / 20);
    return true;
  };
  const int chunks = 128;
  if (!timeit("full", [&] { hipLaunchKernelGGL((scan3_kernel<48, 0>), dim3(2 * chunks), dim3(256), 0, 0, a, chunks, N / 32); })) return 1;
  if (!timeit("no_epilogue", [&] { hipLaunchKernelGGL((scan3_kernel<48, 1>), dim3(2 * chunks), dim3(256), 0, 0, a, chunks, N / 32); })) return 1;
  if (!timeit("no_staging", [&] { hipLaunchKernelGGL((scan3_kernel<48, 2>), dim3(2 * chunks), dim3(256), 0, 0, a, chunks, N / 32); })) return 1;
  if (!timeit("no_barrier", [&] { hipLaunchKernelGGL((scan3_kernel<48, 4>), dim3(2 * chunks), dim3(256), 0, 0, a, chunks, N / 32); })) return 1;
  if (!timeit("mfma_lds_only", [&] { hipLaunchKernelGGL((scan3_kernel<48, 7>), dim3(2 * chunks), dim3(256), 0, 0, a, chunks, N / 32); })) return 1;
  // fixed cost vs per-tile slope: k tiles per workgroup (chunks * k <= N / 32 tiles exist)
  auto run = [&](const char* base, int k, auto kern) {
    char nm[64];
    snprintf(nm, sizeof nm, "%s_k%d", base, k);
    return timeit(nm, [&] { hipLaunchKernelGGL(kern, dim3(2 * chunks), dim3(256), 0, 0, a, chunks, chunks * k); });
  };
  for (int k : {1, 6}) {
    if (!run("full", k, scan3_kernel<48, 0>)) return 1;
    if (!run("no_S_store", k, scan3_kernel<48, 8>)) return 1;
    if (!run("no_max_store", k, scan3_kernel<48, 16>)) return 1;
    if (!run("no_tile_maxima", k, scan3_kernel<48, 32>)) return 1;
    if (!run("no_epilogue", k, scan3_kernel<48, 1>)) return 1;
    if (!run("mfma_lds_only", k, scan3_kernel<48, 7>)) return 1;
    if (!run("mfma_lds_noq", k, scan3_kernel<48, 7 | 64>)) return 1;
    if (!run("mfma_lds_nofirst", k, scan3_kernel<48, 7 | 128>)) return 1;
    if (!run("mfma_lds_noq_nofirst", k, scan3_kernel<48, 7 | 64 | 128>)) return 1;
    if (!run("full_noq", k, scan3_kernel<48, 64>)) return 1;
  }
  // timelines (ABL 256): per workgroup, s_memrealtime at entry / queries loaded / first
  // tile staged / after each tile / end, and the core-clock span
  uint64_t* dtr;
  (void)hipMalloc(&dtr, 2 * chunks * 32 * 8);
  a.trace = dtr;
  auto trace = [&](const char* name, int tiles, auto kern) {
    for (int w = 0; w < 5; ++w) hipLaunchKernelGGL(kern, dim3(2 * chunks), dim3(256), 0, 0, a, chunks, tiles);
    (void)hipMemset(dtr, 0, 2 * chunks * 32 * 8);
    hipLaunchKernelGGL(kern, dim3(2 * chunks), dim3(256), 0, 0, a, chunks, tiles);
    if (hipDeviceSynchronize() != hipSuccess) return false;
    std::vector<uint64_t> tr(2 * chunks * 32);
    (void)hipMemcpy(tr.data(), dtr, tr.size() * 8, hipMemcpyDeviceToHost);
    uint64_t t0 = ~0ull, tend = 0;
    double qload = 0, first = 0, span = 0, ghz = 0, tiles_sum[8] = {0}, start_max = 0;
    int nt_cnt[8] = {0};
    for (int b = 0; b < 2 * chunks; ++b) t0 = std::min(t0, tr[b * 32]);
    for (int b = 0; b < 2 * chunks; ++b) {
      const uint64_t* r = &tr[b * 32];
      const int nt = (int)r[31];
      qload += (r[1] - r[0]) * 10.0;
      first += (r[2] - r[1]) * 10.0;
      span += (r[29] - r[0]) * 10.0;
      ghz += r[30] / ((r[29] - r[0]) * 10.0);
      start_max = std::max(start_max, (r[0] - t0) * 10.0);
      tend = std::max(tend, r[29]);
      for (int j = 0; j < nt && j < 8; ++j) { tiles_sum[j] += (r[3 + j] - r[2 + j]) * 10.0; nt_cnt[j]++; }
    }
    const double n = 2 * chunks;
    printf("{\"trace\":\"%s\",\"ns_qload\":%.0f,\"ns_first_tile\":%.0f,\"ns_wg_span\":%.0f,\"ns_grid\":%.0f,"
           "\"ns_last_start\":%.0f,\"memtime_per_ns\":%.3f,\"ns_tiles\":[",
           name, qload / n, first / n, span / n, (tend - t0) * 10.0, start_max, ghz / n);
    for (int j = 0; j < 8; ++j) printf("%s%.0f", j ? "," : "", nt_cnt[j] ? tiles_sum[j] / nt_cnt[j] : 0.0);
    printf("]}\n");
    return true;
  };
  if (!trace("full", N / 32, scan3_kernel<48, 256>)) return 1;
  if (!trace("no_epilogue", N / 32, scan3_kernel<48, 256 | 1>)) return 1;
  if (!trace("mfma_lds_only", N / 32, scan3_kernel<48, 256 | 7>)) return 1;
  if (!trace("no_staging", N / 32, scan3_kernel<48, 256 | 2>)) return 1;
  if (!trace("no_S_store", N / 32, scan3_kernel<48, 256 | 8>)) return 1;
  if (!trace("no_max_store", N / 32, scan3_kernel<48, 256 | 16>)) return 1;
  if (!trace("no_tile_maxima", N / 32, scan3_kernel<48, 256 | 32>)) return 1;
  if (!trace("no_stage_no_epi", N / 32, scan3_kernel<48, 256 | 3>)) return 1;
  if (!trace("full_k1", chunks, scan3_kernel<48, 256>)) return 1;
  a.trace = nullptr;
  // ---- select over the blocked scores of one full scan launch (similar-sets shape:
  // rank-0 drop, K_int = k + 1 = 51): results against a host top-k, timings, timeline ----
  {
    hipLaunchKernelGGL((scan3_kernel<48, 0>), dim3(2 * chunks), dim3(256), 0, 0, a, chunks, N / 32);
    (void)hipDeviceSynchronize();
    const int k = 50, Kint = 51;
    float* osc;
    int64_t* oid;
    int32_t* ocnt;
    uint64_t *keys, *maxk, *sel_tr;
    (void)hipMalloc(&osc, M * k * 4);
    (void)hipMalloc(&oid, M * k * 8);
    (void)hipMalloc(&ocnt, M * 4);
    (void)hipMalloc(&keys, M * Kint * 8);
    (void)hipMalloc(&maxk, M * 8);
    (void)hipMalloc(&sel_tr, M * 8 * 8);
    SelectArgs sa{};
    sa.S = dS; sa.lds = N; sa.tmax = tm; sa.pmax = pm; sa.ldt = N / 32; sa.n_cols = N; sa.slab_start = 0;
    sa.gid0 = 0; sa.present = ones; sa.K = Kint; sa.keys_out = keys; sa.max_inout = maxk; sa.first_slab = 1;
    sa.out_scores = osc; sa.out_ids = oid; sa.out_counts = ocnt; sa.k_final = k; sa.s_blocked = 1;
    if (launch_select(sa, M, 0) != hipSuccess || hipDeviceSynchronize() != hipSuccess) { printf("{\"select\":\"error\"}\n"); return 1; }
    (void)hipMemcpy(S.data(), dS, S.size() * 4, hipMemcpyDeviceToHost);
    auto SV = [&](int i, int j) { return S[sblk_quad(i, j >> 5, (j >> 2) & 7, N / 32) + (j & 3)]; };
    std::vector<int64_t> ids(M * k);
    (void)hipMemcpy(ids.data(), oid, ids.size() * 8, hipMemcpyDeviceToHost);
    long wrong = 0;
    std::vector<int> ord(N);
    for (int i = 0; i < M; ++i) {
      for (int j = 0; j < N; ++j) ord[j] = j;
      std::partial_sort(ord.begin(), ord.begin() + k + 1, ord.end(), [&](int x, int y) {
        const float fx = SV(i, x), fy = SV(i, y);
        return fx > fy || (fx == fy && x < y);
      });
      for (int r = 0; r < k; ++r) wrong += ids[i * k + r] != ord[r + 1];  // rank 0 dropped
    }
    printf("{\"select_ids_wrong\":%ld}\n", wrong);
    auto stime = [&](const char* name, auto kern) {
      for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(kern, dim3(M), dim3(kSelectThreads), 0, 0, sa);
      hipEvent_t e0, e1;
      (void)hipEventCreate(&e0);
      (void)hipEventCreate(&e1);
      (void)hipEventRecord(e0, 0);
      for (int w = 0; w < 20; ++w) hipLaunchKernelGGL(kern, dim3(M), dim3(kSelectThreads), 0, 0, sa);
      (void)hipEventRecord(e1, 0);
      (void)hipEventSynchronize(e1);
      float ms = 0;
      (void)hipEventElapsedTime(&ms, e0, e1);
      printf("{\"select_timing\":\"%s\",\"us\":%.2f}\n", name, ms * 1e3 / 20);
    };
    stime("full", select_kernel<0>);
    stime("loads", select_kernel<1>);
    stime("bound", select_kernel<2>);
    stime("gather", select_kernel<4>);
    // timeline of one launch right behind a scan (as in a search)
    auto strace = [&](const char* name, auto kern) {
      sa.trace = sel_tr;
      (void)hipMemset(sel_tr, 0, M * 64);
      hipLaunchKernelGGL((scan3_kernel<48, 0>), dim3(2 * chunks), dim3(256), 0, 0, a, chunks, N / 32);
      hipLaunchKernelGGL(kern, dim3(M), dim3(kSelectThreads), 0, 0, sa);
      (void)hipDeviceSynchronize();
      std::vector<uint64_t> tr(M * 8);
      (void)hipMemcpy(tr.data(), sel_tr, tr.size() * 8, hipMemcpyDeviceToHost);
      uint64_t t0 = ~0ull, t5 = 0;
      double ph[5] = {0}, cnt = 0, ntl = 0;
      for (int i = 0; i < M; ++i) {
        const uint64_t* r = &tr[i * 8];
        t0 = std::min(t0, r[0]);
        t5 = std::max(t5, r[5]);
        for (int p = 0; p < 5; ++p) ph[p] += r[p + 1] > r[p] ? (r[p + 1] - r[p]) * 10.0 : 0.0;
        cnt += r[6];
        ntl += r[7];
      }
      printf("{\"select_trace\":\"%s\",\"ns_loads_B1\":%.0f,\"ns_bound\":%.0f,\"ns_tiles_B3\":%.0f,\"ns_gather_B4\":%.0f,"
             "\"ns_sort_emit\":%.0f,\"ns_grid\":%.0f,\"cand\":%.1f,\"tiles\":%.1f}\n",
             name, ph[0] / M, ph[1] / M, ph[2] / M, ph[3] / M, ph[4] / M, (t5 - t0) * 10.0, cnt / M, ntl / M);
    };
    strace("full", select_kernel<0>);
    strace("no_S_loads", select_kernel<16>);
    strace("no_elig_loads", select_kernel<32>);
    strace("no_gather_loads", select_kernel<48>);
    sa.trace = nullptr;
  }
  // empty grid (tiles 0: every workgroup returns at once) = launch + gap
  if (!timeit("empty_grid", [&] { hipLaunchKernelGGL((scan3_kernel<48, 0>), dim3(2 * chunks), dim3(256), 0, 0, a, chunks, 0); })) return 1;
  return 0;
}
