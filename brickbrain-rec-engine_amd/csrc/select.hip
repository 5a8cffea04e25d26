// select.hip — exact per-query top-K over a score slab (gfx950).
//
// Replaces np.argsort(sim)[::-1] + the Python filter walk of get_similar_sets
// (recommendation_system.py:217-247), the rated/valid filter loop + list.sort of the CF
// path (:441-461) and pgvector's ORDER BY <=> LIMIT k.  One workgroup (4 waves) per query
// row.  Eligible = in the slab ∧ present bit (structural: the side's item space) ∧ mask
// bit (valid_set_filter, :229/:454) ∧ ¬exclusion bit (items the user rated, :441-451).
//
// Inputs from the GEMM epilogue: per (query, 32-item tile) the maximum order-image over
// eligible items (tmax) and over present items (pmax, similar-sets only).
//   rank 0  the unmasked arg-max key (dropped by the similar-sets path, :217) = the first
//           present item holding the largest pmax, found by reading one tile
//   bound   T0 = the K-th largest per-thread max of tmax (and the carried list's K-th key):
//           at least K eligible items are >= T0, so every top-K member is
//   gather  read only the tiles with tmax >= T0 (~K of N/32), append eligible items >= T0
//   sort    bitonic sort of the candidates by the full key (score desc, id asc) -> top K
// Exact fallback (candidates overflow the LDS buffer, e.g. masses of equal scores): a
//   3-level radix select (12/12/8 bits) over the whole row for the K-th score T; take all
//   above T and the ties at T in ascending global id (carried keys first: earlier slabs
//   hold smaller ids).
#include "common.h"

#include <cstdlib>

namespace bb {

constexpr int kCandCap = 2048;                  // candidate capacity
constexpr int kOffHist = kMaxKInt * 8;          // radix path: cand[0..kMaxKInt) then hist
constexpr int kRegionA = kOffHist + 4096 * 4;   // 20 KiB, reused by both paths
static_assert(kCandCap * 8 <= kRegionA, "candidate buffer must fit region A");
constexpr int kOffTmax = kRegionA;              // u32[256] per-thread maxima
constexpr int kTileCap = 1024;                  // qualifying-tile list capacity
constexpr int kOffTlist = kOffTmax + kSelectThreads * 4;
constexpr int kOffMisc = kOffTlist + kTileCap * 4;
constexpr int kSelectLds = kOffMisc + 256;

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
__device__ void wave_sort_emit(const uint64_t* cand, int cnt, const SelectArgs& a, int row, uint64_t gmax) {
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
        id[i] = i < c ? (int64_t)gid_of(v[s]) : (int64_t)-1;
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

__device__ const uint32_t kWordOnes = 0xFFFFFFFFu;
__device__ const uint32_t kWordZero = 0u;

template <int ABL>
__global__ __launch_bounds__(kSelectThreads) void select_kernel(SelectArgs a) {
  __shared__ __attribute__((aligned(16))) char dsm[kSelectLds];
  uint64_t* cand = (uint64_t*)dsm;
  uint32_t* hist = (uint32_t*)(dsm + kOffHist);
  uint32_t* tmx = (uint32_t*)(dsm + kOffTmax);
  uint32_t* tlist = (uint32_t*)(dsm + kOffTlist);
  uint32_t* misc = (uint32_t*)(dsm + kOffMisc);  // [0..15] scalars
  uint32_t* scan_sh = misc + 16;                  // 8 words
  uint64_t* red = (uint64_t*)(misc + 32);         // 4 u64

  const int row = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int n = a.n_cols, K = a.K;
  const int ntiles = (n + 31) >> 5;
  const float* Srow = a.S + (size_t)row * a.lds;
  // four scores of items 4g..4g+3 of tile t (row-major S or the scan3 blocked image)
  auto s_quad = [&](int t, int g) -> float4 {
    return a.s_blocked ? *(const float4*)(a.S + sblk_quad(row, t, g, a.ldt)) : *(const float4*)(Srow + t * 32 + 4 * g);
  };
  auto s_at = [&](int j) -> float {
    return a.s_blocked ? a.S[sblk_quad(row, j >> 5, (j >> 2) & 7, a.ldt) + (j & 3)] : Srow[j];
  };
  const uint32_t* trow = a.tmax + (size_t)row * a.ldt;
  const uint32_t* prow = a.max_inout ? a.pmax + (size_t)row * a.ldt : nullptr;
  const uint32_t* excl = a.excl ? a.excl + (size_t)row * a.excl_ld : nullptr;
  const uint64_t* carry = a.carry_in ? a.carry_in + (size_t)row * K : nullptr;
  const int64_t w0 = a.slab_start >> 5;

  // eligibility word of a tile: present ∧ mask ∧ ¬excl, three loads issued together
  // (a null bitset reads a constant word instead of branching)
  auto elig = [&](int tile) -> uint32_t {
    const uint32_t* pp = a.present ? a.present + w0 + tile : &kWordOnes;
    const uint32_t* mp = a.mask ? a.mask + w0 + tile : &kWordOnes;
    const uint32_t* ep = excl ? excl + w0 + tile : &kWordZero;
    return *pp & *mp & ~*ep;
  };

  // probe-only phase timeline (s_memrealtime, 100 MHz), thread 0
  auto stamp = [&](int slot) {
    if (a.trace && tid == 0) a.trace[row * 8 + slot] = __builtin_amdgcn_s_memrealtime();
  };
  stamp(0);
  if (tid == 0) {
    misc[7] = 0;  // candidate count
    misc[8] = 0;  // qualifying-tile count
    *(uint64_t*)(misc + 10) = 0ull;  // rank-0 key of this query
  }

  // ---- one round of loads: tile maxima (and present maxima for rank 0) ----
  constexpr int kB = 4;
  uint32_t v0[kB], p0[kB];
#pragma unroll
  for (int b = 0; b < kB; ++b) {
    const int t = tid + b * kSelectThreads;
    v0[b] = t < ntiles ? trow[t] : 0u;
    p0[b] = (prow && t < ntiles) ? prow[t] : 0u;
  }
  uint32_t tm = 0;
  uint64_t best = 0;  // (present max << 32) | ~tile : larger = higher ord, then lower tile
#pragma unroll
  for (int b = 0; b < kB; ++b) {
    const int t = tid + b * kSelectThreads;
    tm = v0[b] > tm ? v0[b] : tm;
    const uint64_t pv = ((uint64_t)p0[b] << 32) | (uint32_t)(0xFFFFFFFFu - (uint32_t)t);
    best = (p0[b] && pv > best) ? pv : best;
  }
  for (int t = tid + kB * kSelectThreads; t < ntiles; t += kSelectThreads) {  // slabs > 32K columns
    const uint32_t v = trow[t];
    tm = v > tm ? v : tm;
    if (prow) {
      const uint32_t pm = prow[t];
      const uint64_t pv = ((uint64_t)pm << 32) | (uint32_t)(0xFFFFFFFFu - (uint32_t)t);
      best = (pm && pv > best) ? pv : best;
    }
  }
  tmx[tid] = tm;
  if (prow) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const uint64_t y = __shfl_xor(best, o);
      best = y > best ? y : best;
    }
    if (lane == 0) red[wave] = best;
  }
  if constexpr (ABL == 1) { if (tm == 0x12345u) a.keys_out[row] = tm; return; }
  __syncthreads();  // B1
  stamp(1);

  // ---- rank 0 (similar / hybrid content side): wave 0 reads the winning tile now and
  // resolves it after the bound, so its latency hides behind it ----
  uint32_t P0 = 0, r0_word = 0;
  int r0_tile = 0;
  float r0_val = 0.f;
  if (prow && wave == 0) {
    uint64_t b = red[0];
#pragma unroll
    for (int i = 1; i < kSelectThreads / 64; ++i) b = red[i] > b ? red[i] : b;
    P0 = (uint32_t)(b >> 32);
    r0_tile = (int)(0xFFFFFFFFu - (uint32_t)b);
    if (P0 && lane < 32) {
      const int j = r0_tile * 32 + lane;
      r0_val = j < n ? s_at(j) : 0.f;
      r0_word = a.present ? a.present[w0 + r0_tile] : ~0u;
    }
  }

  // ---- bound: T0 = K-th largest per-thread max of the tile maxima (at least K eligible
  // items are >= T0, so every top-K member is).  Every wave finds it on its own, no
  // barrier: the 256 maxima as 4 per lane, then the largest C with #(maxima >= C) >= K,
  // decided bit by bit below the common prefix of the extremes (ballot counts, scalar
  // loop).  Fewer than K non-zero maxima: T0 = 0, i.e. every eligible item. ----
  uint32_t T0 = 0;
  {
    const uint4 x = *(const uint4*)(tmx + 4 * lane);
    auto cnt_ge = [&](uint32_t c) -> uint32_t {
      return (uint32_t)(__popcll(__ballot(x.x >= c)) + __popcll(__ballot(x.y >= c)) + __popcll(__ballot(x.z >= c)) +
                        __popcll(__ballot(x.w >= c)));
    };
    if (cnt_ge(1u) >= (uint32_t)K) {
      uint32_t hi = max(max(x.x, x.y), max(x.z, x.w));
      uint32_t lo = min(min(x.x ? x.x : ~0u, x.y ? x.y : ~0u), min(x.z ? x.z : ~0u, x.w ? x.w : ~0u));
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        hi = max(hi, (uint32_t)__shfl_xor((int)hi, o));
        lo = min(lo, (uint32_t)__shfl_xor((int)lo, o));
      }
      hi = __builtin_amdgcn_readfirstlane(hi);
      lo = __builtin_amdgcn_readfirstlane(lo);
      const uint32_t d = hi ^ lo;
      // bits above the highest differing one are shared by every non-zero maximum
      const int top = d ? 31 - __builtin_clz(d) : -1;
      uint32_t P = top < 0 ? hi : top >= 31 ? 0u : hi & ~((2u << top) - 1u);
      for (int b = top; b >= 0; --b) {
        const uint32_t c = P | (1u << b);
        if (cnt_ge(c) >= (uint32_t)K) P = c;
      }
      T0 = P;
    }
  }
  if (carry) {
    const uint32_t ck = ordk_of(carry[K - 1]);  // K carried keys are >= ck
    T0 = ck > T0 ? ck : T0;
  }
  if (T0 == 0) T0 = 1;  // fewer than K threads see eligible items: take every eligible one
  stamp(2);
  if constexpr (ABL == 2) { if (T0 == 0x12345u) a.keys_out[row] = T0; return; }

  if (prow && wave == 0) {
    uint64_t key = 0;
    if (P0) {
      // float compare: the maxima fold -0 into +0, and numpy's argmax treats them as equal
      const bool hit = lane < 32 && r0_tile * 32 + lane < n && ((r0_word >> lane) & 1u) && r0_val == float_of_ord(P0);
      const uint64_t m = __ballot(hit);
      if (m) {
        const int j0 = (int)__builtin_ctzll(m);
        key = make_key(ord_of(__shfl(r0_val, j0)), a.gid0 + (uint32_t)(r0_tile * 32 + j0));
      }
    }
    if (lane == 0) {
      const uint64_t prev = a.first_slab ? 0ull : a.max_inout[row];
      const uint64_t m = key > prev ? key : prev;
      a.max_inout[row] = m;
      *(uint64_t*)(misc + 10) = m;  // for the final-output drop below
    }
  }

  // ---- qualifying tiles -> compact list (one LDS atomic per wave); carried keys ->
  // candidates ----
  {
    uint64_t qm[kB];
    uint32_t tot = 0;
#pragma unroll
    for (int b = 0; b < kB; ++b) {
      const int t = tid + b * kSelectThreads;
      qm[b] = __ballot(t < ntiles && v0[b] >= T0);
      tot += (uint32_t)__popcll(qm[b]);
    }
    if (tot) {
      uint32_t base = 0;
      if (lane == 0) base = atomicAdd(&misc[8], tot);
      base = (uint32_t)__shfl((int)base, 0);
#pragma unroll
      for (int b = 0; b < kB; ++b) {
        const uint32_t lo32 = (uint32_t)qm[b], hi32 = (uint32_t)(qm[b] >> 32);
        if ((qm[b] >> lane) & 1ull) {
          const uint32_t p = base + __builtin_amdgcn_mbcnt_hi(hi32, __builtin_amdgcn_mbcnt_lo(lo32, 0u));
          if (p < (uint32_t)kTileCap) tlist[p] = (uint32_t)(tid + b * kSelectThreads);
        }
        base += (uint32_t)__popcll(qm[b]);
      }
    }
  }
  for (int t = tid + kB * kSelectThreads; t < ntiles; t += kSelectThreads)
    if (trow[t] >= T0) {
      const uint32_t p = atomicAdd(&misc[8], 1u);
      if (p < (uint32_t)kTileCap) tlist[p] = (uint32_t)t;
    }
  if (carry)
    for (int c = tid; c < K; c += kSelectThreads) {
      const uint64_t key = carry[c];
      if (key && ordk_of(key) >= T0) {
        const uint32_t p = atomicAdd(&misc[7], 1u);
        if (p < kCandCap) cand[p] = key;
      }
    }
  __syncthreads();  // B3
  stamp(3);

  // ---- gather: each thread takes whole qualifying tiles (one latency round when the
  // list has <= 256 tiles): eligibility words and the tile's eight 16-B score loads ----
  auto gather_tile = [&](int t) {
    float4 v[8];
#pragma unroll
    for (int c4 = 0; c4 < 8; ++c4)
      v[c4] = (ABL & 16) ? make_float4(t * 1e-3f, c4 * 1e-3f, 0.f, 0.f) : s_quad(t, c4);
    const uint32_t ok = (ABL & 32) ? ~0u : elig(t);
    uint32_t m = 0;  // items of the tile that become candidates
#pragma unroll
    for (int c4 = 0; c4 < 8; ++c4) {
      const float f[4] = {v[c4].x, v[c4].y, v[c4].z, v[c4].w};
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int it = 4 * c4 + c;
        m |= (t * 32 + it < n && ((ok >> it) & 1u) && ord_of(f[c]) >= T0) ? (1u << it) : 0u;
      }
    }
    if (!m) return;
    uint32_t p = atomicAdd(&misc[7], (uint32_t)__popc(m));  // one LDS atomic per tile
#pragma unroll
    for (int c4 = 0; c4 < 8; ++c4) {
      const float f[4] = {v[c4].x, v[c4].y, v[c4].z, v[c4].w};
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int it = 4 * c4 + c;
        if ((m >> it) & 1u) {
          if (p < (uint32_t)kCandCap) cand[p] = make_key(ord_of(f[c]), a.gid0 + (uint32_t)(t * 32 + it));
          ++p;
        }
      }
    }
  };
  const uint32_t ntl = misc[8];
  if (ntl <= (uint32_t)kTileCap) {
    // list slot i -> thread (i % 4)·64 + i / 4: a short list spreads over all four waves
    const uint32_t slot = ((uint32_t)lane << 2) | (uint32_t)wave;
    for (uint32_t i = slot; i < ntl; i += kSelectThreads) gather_tile((int)tlist[i]);
  } else {  // list overflow (masses of ties at the bound): every tile reaching T0
    for (int t = tid; t < ntiles; t += kSelectThreads)
      if (trow[t] >= T0) gather_tile(t);
  }
  __syncthreads();  // B4
  stamp(4);
  uint32_t cnt = misc[7];
  if constexpr (ABL == 4) { if (cnt == 0x12345u) a.keys_out[row] = cnt; return; }
  if (cnt > (uint32_t)kCandCap) {
    __syncthreads();
    auto ord_at = [&](int j) -> uint32_t {
      const uint32_t ok = elig(j >> 5);
      return ((ok >> (j & 31)) & 1u) ? ord_of(s_at(j)) : 0u;
    };
    cnt = radix_select(ord_at, n, a.gid0, carry, K, cand, hist, misc, scan_sh);
  }
  const uint64_t gmax = *(const uint64_t*)(misc + 10);  // 0 = no rank-0 drop

  // ---- sort candidates by full key, emit the top K ----
  if (cnt <= 256) {  // one wave, registers only
    if (wave != 0) return;
    if (cnt <= 64) wave_sort_emit<1>(cand, (int)cnt, a, row, gmax);
    else if (cnt <= 128) wave_sort_emit<2>(cand, (int)cnt, a, row, gmax);
    else wave_sort_emit<4>(cand, (int)cnt, a, row, gmax);
    if (a.trace && tid == 0) {
      stamp(5);
      a.trace[row * 8 + 6] = cnt;
      a.trace[row * 8 + 7] = misc[8];
    }
    return;
  }
  int P = 1;
  while (P < (int)cnt) P <<= 1;
  for (int i = (int)cnt + tid; i < P; i += kSelectThreads) cand[i] = 0ull;
  __syncthreads();
  if constexpr (ABL != 8) bitonic_desc_u64(cand, P);
  if (a.out_scores) {
    // final list of a single-list mode (semantic / similar / CF) on its last slab: drop
    // rank 0 when it is the head of the list (a present-but-masked rank 0 is not in it),
    // then emit k_final (score, id) pairs — what finalize does for one shard.
    const int start = (gmax && cnt && cand[0] == gmax) ? 1 : 0;
    const int c = min(a.k_final, (int)cnt - start);
    float* sc = a.out_scores + (size_t)row * a.k_final;
    int64_t* id = a.out_ids + (size_t)row * a.k_final;
    for (int i = tid; i < a.k_final; i += kSelectThreads) {
      if (i < c) {
        const uint64_t key = cand[start + i];
        sc[i] = float_of_ord(ordk_of(key));
        id[i] = (int64_t)gid_of(key);
      } else {
        sc[i] = 0.f;
        id[i] = -1;
      }
    }
    if (a.out_counts && tid == 0) a.out_counts[row] = c;
    return;
  }
  uint64_t* out = a.keys_out + (size_t)row * K;
  for (int i = tid; i < K; i += kSelectThreads) out[i] = i < (int)cnt ? cand[i] : 0ull;
}

// ---- streaming top-K, second stage -------------------------------------------------------
// The K-th largest of n distinct keys (get(i), non-zero) by a 64-bit radix select in six
// digit passes (12/12/12/12/8/8 bits); 0 when n < K (take every key).
template <typename Get>
__device__ uint64_t kth_key(Get get, int n, uint32_t K, uint32_t* hist, uint32_t* misc, uint32_t* scan_sh) {
  if ((uint32_t)n < K) return 0ull;
  const int tid = threadIdx.x;
  uint64_t prefix = 0, pmask = 0;
  uint32_t need = K;
#pragma unroll 1
  for (int pass = 0; pass < 6; ++pass) {
    const int shift = pass < 4 ? 52 - 12 * pass : 8 * (5 - pass);
    const int nb = pass < 4 ? 4096 : 256;
    for (int i = tid; i < nb; i += kSelectThreads) hist[i] = 0;
    __syncthreads();
    for (int i = tid; i < n; i += kSelectThreads) {
      const uint64_t key = get(i);
      if ((key & pmask) == prefix) atomicAdd(&hist[(uint32_t)(key >> shift) & (uint32_t)(nb - 1)], 1u);
    }
    __syncthreads();
    find_bin(hist, nb, need, misc, scan_sh);
    const uint32_t b = misc[0], above = misc[1];
    prefix |= (uint64_t)b << shift;
    pmask |= (uint64_t)(nb - 1) << shift;
    need -= above;
    __syncthreads();
  }
  return prefix;
}

constexpr int kCsRegionsMax = 1024;
constexpr int kCsOffHist = kCandCap * 8;
constexpr int kCsOffSel = kCsOffHist + 4096 * 4;
constexpr int kCsOffPre = kCsOffSel + kMaxKInt * 8;
constexpr int kCsOffMisc = kCsOffPre + (kCsRegionsMax + 1) * 4;
constexpr int kCsLds = kCsOffMisc + 256;

// One workgroup per query: gather the appended candidates of its regions (LDS when they fit),
// select the K largest keys exactly, sort them and emit the final list (rank 0 dropped when
// it heads it) or the key list — the same outputs as select_kernel on a single slab.
__global__ __launch_bounds__(kSelectThreads) void cand_select_kernel(CandSelectArgs a) {
  __shared__ __attribute__((aligned(16))) char dsm[kCsLds];
  uint64_t* cand = (uint64_t*)dsm;
  uint32_t* hist = (uint32_t*)(dsm + kCsOffHist);
  uint64_t* sel = (uint64_t*)(dsm + kCsOffSel);
  uint32_t* pre = (uint32_t*)(dsm + kCsOffPre);
  uint32_t* misc = (uint32_t*)(dsm + kCsOffMisc);
  uint32_t* scan_sh = misc + 16;
  uint64_t* red = (uint64_t*)(misc + 32);
  const int row = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int R = a.regions;
  const size_t rbase = (size_t)row * R;

  // region counts -> exclusive prefix (each thread owns up to 4 consecutive regions)
  uint32_t c[4], sum = 0, ovf = 0;
  uint64_t gm = (a.cand_pmax && a.max_in && tid == 0) ? a.max_in[row] : 0ull;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int r = 4 * tid + j;
    const uint32_t raw = r < R ? a.cand_cnt[rbase + r] : 0u;
    ovf |= raw > (uint32_t)a.cap ? 1u : 0u;
    c[j] = raw < (uint32_t)a.cap ? raw : (uint32_t)a.cap;
    sum += c[j];
    if (a.cand_pmax && r < R) {
      const uint64_t k = a.cand_pmax[rbase + r];
      gm = k > gm ? k : gm;
    }
  }
  if (__any(ovf) && lane == 0) atomicOr(a.overflow, 1u);
  uint32_t total;
  uint32_t off = block_excl_scan(sum, scan_sh, total);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int r = 4 * tid + j;
    if (r < R) pre[r] = off;
    off += c[j];
  }
  if (tid == 0) pre[R] = total;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const uint64_t y = __shfl_xor(gm, o);
    gm = y > gm ? y : gm;
  }
  if (lane == 0) red[wave] = gm;
  __syncthreads();
  uint64_t gmax = 0;
  if (a.cand_pmax) {
#pragma unroll
    for (int i = 0; i < kSelectThreads / 64; ++i) gmax = red[i] > gmax ? red[i] : gmax;
    if (a.max_out && tid == 0) a.max_out[row] = gmax;
  }
  // candidate i -> region by binary search over the prefix; i >= total: the carried list
  const uint64_t* carry = a.carry_in ? a.carry_in + (size_t)row * a.K : nullptr;
  auto global_key = [&](int i) -> uint64_t {
    if (i >= (int)total) return carry[i - (int)total];
    int lo = 0, hi = R;  // pre[lo] <= i < pre[hi]
    while (hi - lo > 1) {
      const int mid = (lo + hi) >> 1;
      if (pre[mid] <= (uint32_t)i) lo = mid;
      else hi = mid;
    }
    return a.cand[(rbase + lo) * (size_t)a.cap + (i - pre[lo])];
  };
  const int n = (int)total + (carry ? a.K : 0);
  const uint64_t* src = nullptr;
  if (n <= kCandCap) {
    // gather by region (each region's keys are contiguous): a group of threads per region,
    // four independent loads in flight per thread — no per-key binary search and no chain
    // of dependent global loads
    const int tpr = R >= kSelectThreads ? 1 : kSelectThreads / R;
    for (int r = tid / tpr; r < R; r += kSelectThreads / tpr) {
      const int base = (int)pre[r], cnt = (int)pre[r + 1] - base;
      const uint64_t* sp = a.cand + (rbase + r) * (size_t)a.cap;
      int i = tid % tpr;
      for (; i + 3 * tpr < cnt; i += 4 * tpr) {
        const uint64_t k0 = sp[i], k1 = sp[i + tpr], k2 = sp[i + 2 * tpr], k3 = sp[i + 3 * tpr];
        cand[base + i] = k0;
        cand[base + i + tpr] = k1;
        cand[base + i + 2 * tpr] = k2;
        cand[base + i + 3 * tpr] = k3;
      }
      for (; i < cnt; i += tpr) cand[base + i] = sp[i];
    }
    for (int i = (int)total + tid; i < n; i += kSelectThreads) cand[i] = carry[i - (int)total];
    __syncthreads();
    src = cand;
  }
  SelectArgs sa{};
  sa.K = a.K;
  sa.keys_out = a.keys_out;
  sa.out_scores = a.out_scores;
  sa.out_ids = a.out_ids;
  sa.out_counts = a.out_counts;
  sa.k_final = a.k_final;
  const uint64_t drop = a.cand_pmax ? gmax : 0ull;
  if (src && n <= 256) {
    if (wave != 0) return;
    if (n <= 64) wave_sort_emit<1>(src, n, sa, row, drop);
    else if (n <= 128) wave_sort_emit<2>(src, n, sa, row, drop);
    else wave_sort_emit<4>(src, n, sa, row, drop);
    return;
  }
  if (src && n <= 4 * 512 && a.K <= 128) {
    // up to 2048 candidates in LDS and K <= 128 (every configs[3]/[4] search): each wave
    // sorts its 512-key quarter in registers (no barriers) and writes its top K, packed;
    // wave 0 sorts the <= 4·K survivors and emits.  Replaces the 6-pass radix select
    // (4096-bin histograms and a barrier per phase) for the common case.
    const int nw = min(max(n - wave * 512, 0), 512);
    int off = 0;
    for (int w = 0; w < wave; ++w) off += min(min(max(n - w * 512, 0), 512), a.K);
    uint64_t v[8];
#pragma unroll
    for (int s8 = 0; s8 < 8; ++s8) {
      const int e = s8 * 64 + lane;
      v[s8] = e < nw ? src[wave * 512 + e] : 0ull;
    }
    wave_bitonic_desc<8>(v, lane);
#pragma unroll
    for (int s8 = 0; s8 < 8; ++s8) {
      const int e = s8 * 64 + lane;
      if (e < min(nw, a.K)) sel[off + e] = v[s8];
    }
    __syncthreads();
    if (wave != 0) return;
    int m = 0;
    for (int w = 0; w < kSelectThreads / 64; ++w) m += min(min(max(n - w * 512, 0), 512), a.K);
    if (m <= 64) wave_sort_emit<1>(sel, m, sa, row, drop);
    else if (m <= 128) wave_sort_emit<2>(sel, m, sa, row, drop);
    else if (m <= 256) wave_sort_emit<4>(sel, m, sa, row, drop);
    else wave_sort_emit<8>(sel, m, sa, row, drop);
    return;
  }
  // more than 256: the K-th largest key, then the keys >= it (exactly min(K, n) of them)
  uint64_t kth;
  if (src) kth = kth_key([&](int i) { return src[i]; }, n, (uint32_t)a.K, hist, misc, scan_sh);
  else kth = kth_key(global_key, n, (uint32_t)a.K, hist, misc, scan_sh);
  if (tid == 0) misc[4] = 0;
  __syncthreads();
  for (int i = tid; i < n; i += kSelectThreads) {
    const uint64_t key = src ? src[i] : global_key(i);
    if (key >= kth) {
      const uint32_t p = atomicAdd(&misc[4], 1u);
      if (p < (uint32_t)kMaxKInt) sel[p] = key;
    }
  }
  __syncthreads();
  const int m = (int)min(misc[4], (uint32_t)kMaxKInt);
  if (wave != 0) return;
  if (m <= 64) wave_sort_emit<1>(sel, m, sa, row, drop);
  else if (m <= 128) wave_sort_emit<2>(sel, m, sa, row, drop);
  else if (m <= 256) wave_sort_emit<4>(sel, m, sa, row, drop);
  else wave_sort_emit<8>(sel, m, sa, row, drop);
}

hipError_t launch_cand_select(const CandSelectArgs& a, int B, hipStream_t s) {
  if (a.K <= 0 || a.K > kMaxKInt || B <= 0 || a.regions <= 0 || a.regions > kCsRegionsMax || a.cap <= 0 ||
      !a.cand || !a.cand_cnt || !a.overflow || (!a.out_scores && !a.keys_out))
    return hipErrorInvalidValue;
  hipLaunchKernelGGL(cand_select_kernel, dim3(B), dim3(kSelectThreads), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_select(const SelectArgs& a, int B, hipStream_t s) {
  if (a.K <= 0 || a.K > kMaxKInt || B <= 0 || a.n_cols <= 0 || !a.tmax || (a.max_inout && !a.pmax) ||
      (a.slab_start & 31))
    return hipErrorInvalidValue;
  static const int abl = getenv("BB_SELECT_ABLATE") ? atoi(getenv("BB_SELECT_ABLATE")) : 0;
  switch (abl) {
    case 1: hipLaunchKernelGGL(select_kernel<1>, dim3(B), dim3(kSelectThreads), 0, s, a); break;
    case 2: hipLaunchKernelGGL(select_kernel<2>, dim3(B), dim3(kSelectThreads), 0, s, a); break;
    case 4: hipLaunchKernelGGL(select_kernel<4>, dim3(B), dim3(kSelectThreads), 0, s, a); break;
    case 8: hipLaunchKernelGGL(select_kernel<8>, dim3(B), dim3(kSelectThreads), 0, s, a); break;
    default: hipLaunchKernelGGL(select_kernel<0>, dim3(B), dim3(kSelectThreads), 0, s, a);
  }
  return hipGetLastError();
}

}  // namespace bb
