// select_util.h — device helpers shared by the select kernels (select.hip, select_list.hip):
// score-slab loads, block scans, radix select, register bitonic sorts and the exact f32
// rescoring of candidate rows (f64 sums in one fixed order).
#pragma once
#include <type_traits>

#include "common.h"

namespace bb {

// Scores of the slab: element index of item quad g of tile t of a row (row-major S, or the
// blocked image), and the loads — f32, or int16 codes times the row's quantum (s_h).
__device__ __forceinline__ size_t s_elem(const SelectArgs& a, int row, int t, int g) {
  return a.s_blocked ? sblk_quad(row, t, g, a.ldt) : (size_t)row * a.lds + t * 32 + 4 * g;
}
__device__ __forceinline__ float4 s_quad_ld(const SelectArgs& a, int row, int t, int g, float sh) {
  const size_t e = s_elem(a, row, t, g);
  if (a.s_h) {
    const uint2 w = *(const uint2*)((const int16_t*)a.S + e);
    return make_float4(s16_lo(w.x, sh), s16_hi(w.x, sh), s16_lo(w.y, sh), s16_hi(w.y, sh));
  }
  return *(const float4*)(a.S + e);
}
__device__ __forceinline__ float s_at_ld(const SelectArgs& a, int row, int j, float sh) {
  const size_t e = s_elem(a, row, j >> 5, (j >> 2) & 7) + (j & 3);
  return a.s_h ? (float)((const int16_t*)a.S)[e] * sh : a.S[e];
}

__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* sh, uint32_t& total) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(x, o);
    if (lane >= o) x += y;
  }
  if (lane == 63) sh[w] = x;
  __syncthreads();
  uint32_t pre = 0, tot = 0;
#pragma unroll
  for (int i = 0; i < kSelectThreads / 64; ++i) {
    const uint32_t s = sh[i];
    pre += (i < w) ? s : 0u;
    tot += s;
  }
  __syncthreads();
  total = tot;
  return pre + x - v;
}

// Bin holding the Kneed-th largest element of hist[0..nb) (nb = 4096 or 256).
// misc[0] = bin, misc[1] = count strictly above it; misc[0] = ~0u when fewer than Kneed.
__device__ __forceinline__ void find_bin(const uint32_t* hist, int nb, uint32_t Kneed, uint32_t* misc,
                                         uint32_t* scan_sh) {
  const int per = nb / kSelectThreads;
  const int hi = nb - per * (int)threadIdx.x;  // this thread: bins [hi-per, hi), top first
  uint32_t s = 0;
  for (int b = hi - 1; b >= hi - per; --b) s += hist[b];
  uint32_t tot;
  const uint32_t above = block_excl_scan(s, scan_sh, tot);
  if (tot < Kneed) {
    if (threadIdx.x == 0) misc[0] = 0xFFFFFFFFu;
  } else if (above < Kneed && above + s >= Kneed) {
    uint32_t acc = above;
    for (int b = hi - 1; b >= hi - per; --b) {
      const uint32_t c = hist[b];
      if (acc + c >= Kneed) {
        misc[0] = (uint32_t)b;
        misc[1] = acc;
        break;
      }
      acc += c;
    }
  }
  __syncthreads();
}

__device__ __forceinline__ void bitonic_desc_u64(uint64_t* v, int P) {
  for (int k = 2; k <= P; k <<= 1)
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = threadIdx.x; i < P; i += kSelectThreads) {
        const int ixj = i ^ j;
        if (ixj > i) {
          const uint64_t x = v[i], y = v[ixj];
          const bool desc = (i & k) == 0;
          if (desc ? (x < y) : (x > y)) {
            v[i] = y;
            v[ixj] = x;
          }
        }
      }
      __syncthreads();
    }
}

// Exact radix fallback over the whole row (+ carried keys); ord_at(j) = order-image of
// column j or 0 when ineligible.  Leaves cnt (<= K) keys in cand[0..cnt), returns cnt.
template <typename OrdAt>
__device__ uint32_t radix_select(OrdAt ord_at, int n, uint32_t gid0, const uint64_t* carry, int K, uint64_t* cand,
                                 uint32_t* hist, uint32_t* misc, uint32_t* scan_sh) {
  const int tid = threadIdx.x;
  for (int i = tid; i < 4096; i += kSelectThreads) hist[i] = 0;
  __syncthreads();
  for (int j = tid; j < n; j += kSelectThreads) {
    const uint32_t o = ord_at(j);
    if (o) atomicAdd(&hist[o >> 20], 1u);
  }
  if (carry)
    for (int c = tid; c < K; c += kSelectThreads) {
      const uint64_t key = carry[c];
      if (key) atomicAdd(&hist[ordk_of(key) >> 20], 1u);
    }
  __syncthreads();
  find_bin(hist, 4096, (uint32_t)K, misc, scan_sh);
  const bool take_all = misc[0] == 0xFFFFFFFFu;
  uint32_t T = 1u, above_T = 0u, eqc = 0u;
  if (!take_all) {
    const uint32_t b1 = misc[0], above1 = misc[1];
    __syncthreads();
    for (int i = tid; i < 4096; i += kSelectThreads) hist[i] = 0;
    __syncthreads();
    for (int j = tid; j < n; j += kSelectThreads) {
      const uint32_t o = ord_at(j);
      if (o && (o >> 20) == b1) atomicAdd(&hist[(o >> 8) & 0xFFFu], 1u);
    }
    if (carry)
      for (int c = tid; c < K; c += kSelectThreads) {
        const uint32_t o = ordk_of(carry[c]);
        if (o && (o >> 20) == b1) atomicAdd(&hist[(o >> 8) & 0xFFFu], 1u);
      }
    __syncthreads();
    find_bin(hist, 4096, (uint32_t)K - above1, misc, scan_sh);
    const uint32_t b2 = misc[0], above2 = misc[1];
    const uint32_t p24 = (b1 << 12) | b2;
    __syncthreads();
    for (int i = tid; i < 256; i += kSelectThreads) hist[i] = 0;
    __syncthreads();
    for (int j = tid; j < n; j += kSelectThreads) {
      const uint32_t o = ord_at(j);
      if (o && (o >> 8) == p24) atomicAdd(&hist[o & 0xFFu], 1u);
    }
    if (carry)
      for (int c = tid; c < K; c += kSelectThreads) {
        const uint32_t o = ordk_of(carry[c]);
        if (o && (o >> 8) == p24) atomicAdd(&hist[o & 0xFFu], 1u);
      }
    __syncthreads();
    find_bin(hist, 256, (uint32_t)K - above1 - above2, misc, scan_sh);
    const uint32_t b3 = misc[0], above3 = misc[1];
    T = (p24 << 8) | b3;
    above_T = above1 + above2 + above3;
    eqc = hist[b3];
  }
  const uint32_t need = take_all ? 0u : (uint32_t)K - above_T;  // ties to take at T
  const bool ordered_ties = !take_all && eqc > need;
  __syncthreads();
  if (tid == 0) misc[4] = 0;
  __syncthreads();
  const uint32_t lo = ordered_ties ? T + 1u : T;  // take ords >= lo without ordering
  for (int j = tid; j < n; j += kSelectThreads) {
    const uint32_t o = ord_at(j);
    if (o && o >= lo) cand[atomicAdd(&misc[4], 1u)] = make_key(o, gid0 + (uint32_t)j);
  }
  if (carry)
    for (int c = tid; c < K; c += kSelectThreads) {
      const uint64_t key = carry[c];
      if (key && ordk_of(key) >= lo) cand[atomicAdd(&misc[4], 1u)] = key;
    }
  __syncthreads();
  uint32_t cnt = misc[4];
  if (ordered_ties) {
    if (tid == 0) {  // carried ties first (smaller ids), in list order = id asc
      uint32_t c2 = cnt, rem = need;
      for (int c = 0; carry && c < K && rem; ++c) {
        const uint64_t key = carry[c];
        if (key && ordk_of(key) == T) {
          cand[c2++] = key;
          --rem;
        }
      }
      misc[4] = c2;
      misc[5] = rem;
    }
    __syncthreads();
    cnt = misc[4];
    uint32_t rem = misc[5];
    for (int base = 0; base < n && rem; base += kSelectThreads) {
      const int j = base + tid;
      const uint32_t o = j < n ? ord_at(j) : 0u;
      const uint32_t tie = (o == T) ? 1u : 0u;
      uint32_t tot;
      const uint32_t rk = block_excl_scan(tie, scan_sh, tot);
      if (tie && rk < rem) cand[cnt + rk] = make_key(o, gid0 + (uint32_t)j);
      const uint32_t take = tot < rem ? tot : rem;
      cnt += take;
      rem -= take;
    }
    __syncthreads();
  }
  return cnt;
}

// Register-resident bitonic sort of up to 64·E keys by one wave (element e = s·64 + lane
// lives in v[s]); descending.  No LDS, no barriers.
template <int E>
__device__ __forceinline__ void wave_bitonic_desc(uint64_t (&v)[E], int lane) {
#pragma unroll
  for (int k = 2; k <= 64 * E; k <<= 1) {
#pragma unroll
    for (int j = k >> 1; j > 0; j >>= 1) {
      if (j >= 64) {
        const int js = j >> 6;
#pragma unroll
        for (int s = 0; s < E; ++s) {
          if ((s & js) == 0) {
            const bool desc = ((s * 64) & k) == 0;  // lane bits are below k here
            const uint64_t x = v[s], y = v[s | js];
            const bool sw = desc ? (x < y) : (x > y);
            v[s] = sw ? y : x;
            v[s | js] = sw ? x : y;
          }
        }
      } else {
#pragma unroll
        for (int s = 0; s < E; ++s) {
          const int e = s * 64 + lane;
          const uint64_t y = __shfl_xor(v[s], j);
          const bool lower = (lane & j) == 0;
          const bool desc = (e & k) == 0;
          const bool keep_max = lower == desc;
          v[s] = keep_max ? (v[s] > y ? v[s] : y) : (v[s] < y ? v[s] : y);
        }
      }
    }
  }
}

// Sort cnt (<= 64·E) candidates with one wave and emit the final list / the key list.
template <int E>
__device__ __forceinline__ void wave_sort_emit(const uint64_t* cand, int cnt, const SelectArgs& a, int row, uint64_t gmax) {
  const int lane = threadIdx.x & 63;
  uint64_t v[E];
#pragma unroll
  for (int s = 0; s < E; ++s) {
    const int e = s * 64 + lane;
    v[s] = e < cnt ? cand[e] : 0ull;
  }
  wave_bitonic_desc<E>(v, lane);
  if (a.out_scores) {
    const uint64_t head = __shfl(v[0], 0);
    const int start = (gmax && cnt && head == gmax) ? 1 : 0;
    const int c = min(a.k_final, cnt - start);
    float* sc = a.out_scores + (size_t)row * a.k_final;
    int64_t* id = a.out_ids + (size_t)row * a.k_final;
#pragma unroll
    for (int s = 0; s < E; ++s) {
      const int i = s * 64 + lane - start;
      if (i >= 0 && i < a.k_final) {
        sc[i] = i < c ? float_of_ord(ordk_of(v[s])) : 0.f;
        id[i] = i < c ? out_id(a.idmap, gid_of(v[s])) : (int64_t)-1;
      }
    }
    for (int i = 64 * E - start + lane; i < a.k_final; i += 64) {
      sc[i] = 0.f;
      id[i] = -1;
    }
    if (a.out_counts && lane == 0) a.out_counts[row] = c;
    return;
  }
  uint64_t* out = a.keys_out + (size_t)row * a.K;
#pragma unroll
  for (int s = 0; s < E; ++s) {
    const int e = s * 64 + lane;
    if (e < a.K) out[e] = v[s];  // keys past cnt are 0
  }
  for (int e = 64 * E + lane; e < a.K; e += 64) out[e] = 0ull;
}

// ---- exact re-rank helpers (SelectArgs.rr_*) ----------------------------------------------
// Margin between an approximate score and the exact one, both ways: 2ε plus slack for the
// f32 evaluation of ε and for ties created by rounding the exact f64 sums to f32.
__device__ __forceinline__ float rr_margin(float eps) { return eps > 0.f ? 2.f * eps * (1.f + 0x1p-10f) + 0x1p-20f : 0.f; }
// ord image of (score(o) − m), rounded down; never below 1 (1 = "every eligible item")
__device__ __forceinline__ uint32_t ord_sub(uint32_t o, float m) {
  if (o <= 1u || m <= 0.f) return o;
  const float g = __double2float_rd((double)float_of_ord(o) - (double)m);
  const uint32_t r = ord_of(g);
  return r > 1u ? r : 1u;
}
// Exact score of one item row against the query row: f32 products summed in f64, 16 lanes
// per row — lane p takes the float4 chunks p, p+16, ... in order, the 16 partials are then
// combined by DPP (quad swaps, row half-mirror, row mirror) — one fixed order for every path
// (candidates, rank 0, slow paths), so an item rescored twice gets the same bits.
typedef float f4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ f4v lds_f4(const float* qs, int c) {
  return *(const __attribute__((address_space(3))) f4v*)((const __attribute__((address_space(3))) char*)
                                                            ((size_t)(const void*)qs) + c * 16);
}
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v) {
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), CTRL, 0xF, 0xF, false);
  return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double sum16_f64(double v) {
  v += dpp_f64<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp_f64<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp_f64<0x141>(v);  // row_half_mirror: quad 0 <-> 1, 2 <-> 3
  v += dpp_f64<0x140>(v);  // row_mirror: half 0 <-> 1
  return v;
}
__device__ __forceinline__ uint64_t rr_key(float e, uint32_t gid) { return make_key(ord_of(e + 0.0f), gid); }

// Rescore keys[0..m) in place (approximate / placeholder -> exact keys).  NG lane groups of
// 16 (NG·16 threads call it together), U rows per group in flight (U·CPL <= 12 chunks per
// lane: the select's register budget, not its row latency, bounds the in-flight throughput —
// a fat select wave keeps the next batch's scan off the CU).
template <int CPL, int U, int NG, bool QF64 = true>
__device__ __forceinline__ void rescore_rows(uint64_t* keys, int m, const SelectArgs& a, const float* qs, int t) {
  const int p = t & 15, g = t >> 4;
  const int nch = a.rr_d >> 2;
  // the query chunks of this lane (zero past the row: those FMAs add exact zeros, so the sum
  // — and its order — is the same for every row width; no per-chunk branches, which put
  // every FMA in a basic block of its own behind its own s_waitcnt); widened to f64 once
  // (QF64) or at each use (half the registers: occupancy of the list select)
  // (the lean variant re-reads its query chunks from LDS every round: the compiler hoists
  // any register copy's f32 -> f64 conversions out of the loop, 2·4·CPL registers)
  double qd[QF64 ? CPL : 1][4];
  auto load_q = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < (QF64 ? CPL : 1); ++j) {
      const int c = p + 16 * j;
      const f4v q = c < nch ? lds_f4(qs, c) : f4v{0.f, 0.f, 0.f, 0.f};
      qd[j][0] = (double)q.x;
      qd[j][1] = (double)q.y;
      qd[j][2] = (double)q.z;
      qd[j][3] = (double)q.w;
    }
  };
  if constexpr (QF64) load_q();
  for (int c0 = g * U; c0 < m; c0 += NG * U) {
    uint32_t gid[U];
    f4v xv[U][CPL];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      // branch-free (a clamped re-read of the last key): a conditional read splits the
      // rows into blocks of their own and leaves one row's loads in flight at a time
      gid[u] = gid_of(keys[min(c0 + u, m - 1)]);
      const f4v* xr = (const f4v*)(a.rr_x + (a.ablate & 1 ? (size_t)0 : (size_t)(gid[u] - a.rr_gid_base) * a.rr_ld));
#pragma unroll
      for (int j = 0; j < CPL; ++j) xv[u][j] = xr[min(p + 16 * j, nch - 1)];
    }
    f4v ql[QF64 ? 1 : CPL];
    if constexpr (!QF64) {
#pragma unroll
      for (int j = 0; j < CPL; ++j) {
        const int c = p + 16 * j;
        ql[j] = c < nch ? lds_f4(qs, c) : f4v{0.f, 0.f, 0.f, 0.f};
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      double acc = 0.0;
#pragma unroll
      for (int j = 0; j < CPL; ++j) {
        const double q0 = QF64 ? qd[QF64 ? j : 0][0] : (double)ql[QF64 ? 0 : j].x;
        const double q1 = QF64 ? qd[QF64 ? j : 0][1] : (double)ql[QF64 ? 0 : j].y;
        const double q2 = QF64 ? qd[QF64 ? j : 0][2] : (double)ql[QF64 ? 0 : j].z;
        const double q3 = QF64 ? qd[QF64 ? j : 0][3] : (double)ql[QF64 ? 0 : j].w;
        acc = fma((double)xv[u][j].x, q0, acc);
        acc = fma((double)xv[u][j].y, q1, acc);
        acc = fma((double)xv[u][j].z, q2, acc);
        acc = fma((double)xv[u][j].w, q3, acc);
      }
      acc = sum16_f64(acc);
      if (p == 0 && c0 + u < m) keys[c0 + u] = rr_key((float)acc, gid[u]);
    }
  }
}
// block select (256 threads)
__device__ __forceinline__ void rr_rescore_any(uint64_t* keys, int m, const SelectArgs& a, const float* qs) {
  const int cpl = ((a.rr_d >> 2) + 15) >> 4;
  const int t = threadIdx.x;
  if (cpl <= 1) rescore_rows<1, 12, 16>(keys, m, a, qs, t);
  else if (cpl <= 2) rescore_rows<2, 6, 16>(keys, m, a, qs, t);
  else if (cpl <= 4) rescore_rows<4, 3, 16>(keys, m, a, qs, t);
  else if (cpl <= 6) rescore_rows<6, 2, 16>(keys, m, a, qs, t);
  else rescore_rows<8, 1, 16>(keys, m, a, qs, t);   // rows up to kRrMaxD = 512 wide
}

}  // namespace bb
