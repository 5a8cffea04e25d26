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
#include "select_util.h"

#include <cstdlib>

namespace bb {

// The streaming path's overflow flag lives in pinned host memory (the host reads it after its
// one wait, no copy back): every writer stores 1 — a system-scope store, not a read-modify-
// write, so it needs no PCIe atomics.
__device__ __forceinline__ void flag_set(uint32_t* f) {
  __hip_atomic_store(f, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

constexpr int kCandCap = 2048;                  // candidate capacity
constexpr int kOffHist = kMaxKInt * 8;          // radix path: cand[0..kMaxKInt) then hist
constexpr int kRegionA = kOffHist + 4096 * 4;   // 20 KiB, reused by both paths
static_assert(kCandCap * 8 <= kRegionA, "candidate buffer must fit region A");
constexpr int kOffTmax = kRegionA;              // u32[256] per-thread maxima
constexpr int kTileCap = 1024;                  // qualifying-tile list capacity
constexpr int kOffTlist = kOffTmax + kSelectThreads * 4;
constexpr int kOffMisc = kOffTlist + kTileCap * 4;
constexpr int kOffR0 = kOffMisc + 256;          // re-rank: rank-0 tile list
constexpr int kR0Cap = 32;
constexpr int kOffQs = kOffR0 + kR0Cap * 4;       // fused re-rank: the f32 query row
constexpr int kSelectLds = kOffQs + kRrMaxD * 4;


// Re-rank with masses of items at the gather bound (more than kCandCap): an exact running
// top-K over every eligible item whose approximate score reaches Tg, collected 256 per round,
// rescored in batches (rr_rescore_any, 16 lanes per row) and merged into the list 1024+ keys
// at a time; then the final list / key list.
template <typename Elig, typename SAt>
__device__ __forceinline__ void rr_slow_path(const SelectArgs& a, int row, int n, uint32_t Tg, int K, uint64_t* cand,
                                             uint32_t* misc, const float* qs, Elig elig, SAt s_at) {
  const int tid = threadIdx.x;
  uint64_t* sel = cand + 2048;  // the running list: K <= kMaxKInt keys, sorted desc
  uint64_t* buf = cand;         // fresh keys [0, nb) + the list appended for the merge
  for (int i = tid; i < K; i += kSelectThreads) sel[i] = 0ull;
  if (tid == 0) misc[12] = 0;
  __syncthreads();
  auto merge = [&](int nb) {
    rr_rescore_any(buf, nb, a, qs);  // placeholder keys -> exact keys
    __syncthreads();
    for (int i = tid; i < K; i += kSelectThreads) buf[nb + i] = sel[i];
    int P = 1;
    while (P < nb + K) P <<= 1;
    for (int i = nb + K + tid; i < P; i += kSelectThreads) buf[i] = 0ull;
    __syncthreads();
    bitonic_desc_u64(buf, P);
    for (int i = tid; i < K; i += kSelectThreads) sel[i] = buf[i];
    __syncthreads();
    if (tid == 0) misc[12] = 0;
    __syncthreads();
  };
  for (int base = 0; base < n; base += kSelectThreads) {
    const int j = base + tid;
    if (j < n && ((elig(j >> 5) >> (j & 31)) & 1u) && ord_of(s_at(j)) >= Tg)
      buf[atomicAdd(&misc[12], 1u)] = make_key(1u, a.gid0 + (uint32_t)j);
    __syncthreads();
    const int nb = (int)misc[12];
    __syncthreads();  // every thread holds nb before the next round's appends
    if (nb > 2048 - kMaxKInt - kSelectThreads) merge(nb);
  }
  {
    const int nb = (int)misc[12];
    if (nb) merge(nb);
  }
  const uint64_t gmax = *(const uint64_t*)(misc + 10);
  int cnt = 0;
  for (int i = 0; i < K; ++i) cnt += sel[i] != 0ull;  // uniform: every thread counts
  if (a.out_scores) {
    const int start = (gmax && cnt && sel[0] == gmax) ? 1 : 0;
    const int c = min(a.k_final, cnt - start);
    float* sc = a.out_scores + (size_t)row * a.k_final;
    int64_t* id = a.out_ids + (size_t)row * a.k_final;
    for (int i = tid; i < a.k_final; i += kSelectThreads) {
      sc[i] = i < c ? float_of_ord(ordk_of(sel[start + i])) : 0.f;
      id[i] = i < c ? out_id(a.idmap, gid_of(sel[start + i])) : (int64_t)-1;
    }
    if (a.out_counts && tid == 0) a.out_counts[row] = c;
    return;
  }
  uint64_t* out = a.keys_out + (size_t)row * K;
  for (int i = tid; i < K; i += kSelectThreads) out[i] = sel[i];
}

__device__ const uint32_t kWordOnes = 0xFFFFFFFFu;
__device__ const uint32_t kWordZero = 0u;

// RR: the re-rank variant (rr_eps set) — a separate instance, so the plain select keeps its
// register budget
template <int ABL, bool RR = false>
__device__ __forceinline__ void select_body(const SelectArgs& a, int row) {
  __shared__ __attribute__((aligned(16))) char dsm[kSelectLds];
  uint64_t* cand = (uint64_t*)dsm;
  uint32_t* hist = (uint32_t*)(dsm + kOffHist);
  uint32_t* tmx = (uint32_t*)(dsm + kOffTmax);
  uint32_t* tlist = (uint32_t*)(dsm + kOffTlist);
  uint32_t* misc = (uint32_t*)(dsm + kOffMisc);  // [0..15] scalars
  uint32_t* scan_sh = misc + 16;                  // 8 words
  uint64_t* red = (uint64_t*)(misc + 32);         // 4 u64

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (RR && a.rr_flags && a.rr_flags[row] == 0u) return;  // finished by select_rr_wave_kernel
  const int n = a.n_cols, K = a.K;
  const int ntiles = (n + 31) >> 5;
  // four scores of items 4g..4g+3 of tile t (row-major S or the scan3 blocked image)
  const float sh = a.s_h ? a.s_h[row] : 0.f;  // int16 score image: decode quantum
  auto s_quad = [&](int t, int g) -> float4 { return s_quad_ld(a, row, t, g, sh); };
  auto s_at = [&](int j) -> float { return s_at_ld(a, row, j, sh); };
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
  constexpr bool rr = RR;
  float eps2 = 0.f;
  if (rr) eps2 = rr_margin(a.rr_eps[row]);
  if (tid == 0) {
    misc[7] = 0;  // candidate count
    misc[8] = 0;  // qualifying-tile count
    misc[13] = 0;  // re-rank: rank-0 tiles
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
  // fused re-rank: the f32 query row goes to LDS (issued behind the maxima loads, so its
  // wait is theirs)
  float* qs = (float*)(dsm + kOffQs);
  const bool rr_fused = RR && a.rr_out == nullptr;
  float4 qv = make_float4(0.f, 0.f, 0.f, 0.f);
  if (rr_fused && tid < (a.rr_d >> 2)) qv = ((const float4*)(a.rr_q + (size_t)row * a.rr_ld))[tid];
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
  if (rr_fused && tid < (a.rr_d >> 2)) ((float4*)qs)[tid] = qv;
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
  if (prow && wave == 0 && !rr) {
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
  // re-rank: gather every item whose approximate score may still hold an exact top-K place
  const uint32_t Tg = rr ? ord_sub(T0, eps2) : T0;
  stamp(2);
  if constexpr (ABL == 2) { if (T0 == 0x12345u) a.keys_out[row] = T0; return; }

  if (prow && wave == 0 && !rr) {
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
      qm[b] = __ballot(t < ntiles && v0[b] >= Tg);
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
    if (trow[t] >= Tg) {
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
        m |= (t * 32 + it < n && ((ok >> it) & 1u) && ord_of(f[c]) >= Tg) ? (1u << it) : 0u;
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
  } else {  // list overflow (masses of ties at the bound): every tile reaching the bound
    for (int t = tid; t < ntiles; t += kSelectThreads)
      if (trow[t] >= Tg) gather_tile(t);
  }
  __syncthreads();  // B4
  stamp(4);
  uint32_t cnt = misc[7];
  if constexpr (ABL == 4) { if (cnt == 0x12345u) a.keys_out[row] = cnt; return; }
  if constexpr (rr) {
    // ---- exact re-rank.  Fused (rr_out == null): this workgroup rescores the candidates
    // from the f32 rows and emits (rr_finish); otherwise the hand-off to rerank_kernel.
    // Rank 0: the present items whose approximate score is within the margin of the
    // approximate present maximum (typically the liked set alone) ----
    const bool fuse = a.rr_out == nullptr;
    uint32_t r0n = 0, thr0 = 0;
    if (prow) {
      uint64_t b = red[0];
#pragma unroll
      for (int i = 1; i < kSelectThreads / 64; ++i) b = red[i] > b ? red[i] : b;
      const uint32_t Pm = (uint32_t)(b >> 32);
      thr0 = ord_sub(Pm, eps2);
      uint32_t* r0t = (uint32_t*)(dsm + kOffR0);
      if (Pm) {
#pragma unroll
        for (int bb = 0; bb < kB; ++bb) {
          const int t = tid + bb * kSelectThreads;
          if (t < ntiles && p0[bb] >= thr0) {
            const uint32_t q = atomicAdd(&misc[13], 1u);
            if (q < (uint32_t)kR0Cap) r0t[q] = (uint32_t)t;
          }
        }
        for (int t = tid + kB * kSelectThreads; t < ntiles; t += kSelectThreads)
          if (prow[t] >= thr0) {
            const uint32_t q = atomicAdd(&misc[13], 1u);
            if (q < (uint32_t)kR0Cap) r0t[q] = (uint32_t)t;
          }
      }
      if (tid == 0) misc[14] = 0;
      __syncthreads();
      const uint32_t nt0 = misc[13];
      uint32_t* r0g = fuse ? nullptr : a.rr_r0 + (size_t)row * kRrR0Cap;
      if (Pm && nt0 <= (uint32_t)kR0Cap)
        for (int i = tid; i < (int)nt0 * 32; i += kSelectThreads) {
          const int t = (int)r0t[i >> 5], it = i & 31, j = t * 32 + it;
          const uint32_t pw = a.present ? a.present[w0 + t] : ~0u;
          if (j < n && ((pw >> it) & 1u) && ord_of(s_at(j)) >= thr0) {
            const uint32_t q = atomicAdd(&misc[14], 1u);
            if (q < (uint32_t)kRrR0Cap) {
              if (fuse) cand[2048 + q] = make_key(1u, a.gid0 + (uint32_t)j);
              else r0g[q] = a.gid0 + (uint32_t)j;
            }
          }
        }
      __syncthreads();
      r0n = !Pm ? 0u : (nt0 > (uint32_t)kR0Cap || misc[14] > (uint32_t)kRrR0Cap) ? kRrSlow : misc[14];
      if (!fuse && tid == 0) {
        a.rr_r0n[row] = r0n;
        a.rr_thr[2 * row + 1] = thr0;
      }
    }
    uint32_t m = kRrSlow;  // masses of items at the bound: the exact slow path
    if (cnt <= 256u) {
      // ---- the K-th approximate score by ballots (wave 0, four candidates per lane), then
      // the candidates within 2ε of it compacted to cand[0..m) — no sort needed here:
      // rr_finish rescores and sorts them ----
      if (wave == 0) {
        uint64_t v[4];
        uint32_t o[4];
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4) {
          const int i = s4 * 64 + lane;
          v[s4] = i < (int)cnt ? cand[i] : 0ull;
          o[s4] = ordk_of(v[s4]);
        }
        uint32_t thr = 1u;
        if (cnt >= (uint32_t)K) {
          auto cnt_ge = [&](uint32_t c) -> uint32_t {
            return (uint32_t)(__popcll(__ballot(o[0] >= c)) + __popcll(__ballot(o[1] >= c)) +
                              __popcll(__ballot(o[2] >= c)) + __popcll(__ballot(o[3] >= c)));
          };
          uint32_t hi = max(max(o[0], o[1]), max(o[2], o[3]));
          uint32_t lo = min(min(o[0] ? o[0] : ~0u, o[1] ? o[1] : ~0u), min(o[2] ? o[2] : ~0u, o[3] ? o[3] : ~0u));
#pragma unroll
          for (int sh = 32; sh > 0; sh >>= 1) {
            hi = max(hi, (uint32_t)__shfl_xor((int)hi, sh));
            lo = min(lo, (uint32_t)__shfl_xor((int)lo, sh));
          }
          hi = __builtin_amdgcn_readfirstlane(hi);
          lo = __builtin_amdgcn_readfirstlane(lo);
          const uint32_t dd = hi ^ lo;
          const int top = dd ? 31 - __builtin_clz(dd) : -1;
          uint32_t P = top < 0 ? hi : top >= 31 ? 0u : hi & ~((2u << top) - 1u);
          for (int bt = top; bt >= 0; --bt) {
            const uint32_t c = P | (1u << bt);
            if (cnt_ge(c) >= (uint32_t)K) P = c;
          }
          thr = ord_sub(P, eps2);
        }
        uint32_t base = 0;
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4) {
          const bool keep = v[s4] != 0ull && o[s4] >= thr;
          const uint64_t bm = __ballot(keep);
          const uint32_t pos = base + __builtin_amdgcn_mbcnt_hi((uint32_t)(bm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bm, 0u));
          if (keep) cand[pos] = v[s4];
          base += (uint32_t)__popcll(bm);
        }
        if (lane == 0) misc[12] = base;
      }
      __syncthreads();
      m = misc[12];
    } else if (cnt <= (uint32_t)kCandCap) {
      // ---- approximate order -> the K-th approximate score -> the candidates within 2ε ----
      int P = 1;
      while (P < (int)cnt) P <<= 1;
      for (int i = (int)cnt + tid; i < P; i += kSelectThreads) cand[i] = 0ull;
      __syncthreads();
      bitonic_desc_u64(cand, P);
      m = cnt;
      if (cnt >= (uint32_t)K) {
        const uint32_t thr = ord_sub(ordk_of(cand[K - 1]), eps2);
        // sorted: the prefix of keys reaching thr (thread-parallel boundary search)
        if (tid == 0) misc[12] = cnt;
        __syncthreads();
        for (int i = tid; i < (int)cnt; i += kSelectThreads)
          if (ordk_of(cand[i]) >= thr && (i + 1 == (int)cnt || ordk_of(cand[i + 1]) < thr)) misc[12] = (uint32_t)(i + 1);
        __syncthreads();
        m = misc[12];
      }
    }
    if (m > (uint32_t)kRrCap) m = kRrSlow;
    if (fuse) {
      stamp(5);
      rr_finish(a, row, n, cand, misc, qs, m, r0n, Tg, thr0, elig, s_at);
      stamp(7);
      return;
    }
    if (tid == 0) {
      a.rr_cnt[row] = m;
      if (m == kRrSlow) a.rr_thr[2 * row] = Tg;
    }
    if (m == kRrSlow) return;
    uint64_t* out = a.rr_out + (size_t)row * kRrCap;
    for (int i = tid; i < (int)m; i += kSelectThreads) out[i] = cand[i];
    return;
  } else if (cnt > (uint32_t)kCandCap) {
    __syncthreads();
    auto ord_at = [&](int j) -> uint32_t {
      const uint32_t ok = elig(j >> 5);
      return ((ok >> (j & 31)) & 1u) ? ord_of(s_at(j)) : 0u;
    };
    cnt = radix_select(ord_at, n, a.gid0, carry, K, cand, hist, misc, scan_sh);
  }
  const uint64_t gmax = *(const uint64_t*)(misc + 10);  // 0 = no rank-0 drop

  // ---- sort candidates by full key, emit the top K ----
  if (cnt <= 256 || (rr && cnt <= 512)) {  // one wave, registers only
    if (wave != 0) return;
    if (cnt <= 64) wave_sort_emit<1>(cand, (int)cnt, a, row, gmax);
    else if (cnt <= 128) wave_sort_emit<2>(cand, (int)cnt, a, row, gmax);
    else if (cnt <= 256) wave_sort_emit<4>(cand, (int)cnt, a, row, gmax);
    else wave_sort_emit<8>(cand, (int)cnt, a, row, gmax);
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
        id[i] = out_id(a.idmap, gid_of(key));
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

template <int ABL, bool RR = false>
__global__ __launch_bounds__(kSelectThreads) void select_kernel(SelectArgs a) {
  select_body<ABL, RR>(a, xcd_row(blockIdx.x, gridDim.x));
}
// re-rank rows the hybrid's dual wave select left (rr_flags), both sides in one launch
__global__ __launch_bounds__(kSelectThreads) void select_rr_dual_kernel(SelectArgs a0, SelectArgs a1, int B0, int B1) {
  if ((int)blockIdx.x < B0)
    select_body<0, true>(a0, xcd_row(blockIdx.x, B0));
  else
    select_body<0, true>(a1, xcd_row(blockIdx.x - B0, B1));
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
// sel aliases the histogram: the radix path writes sel only after kth_key's last barrier,
// and the four-segment path never touches the histogram.  37.1 KB instead of 41.2 KB: four
// workgroups per CU instead of three (configs[3]'s 4,096 rows in four rounds, not six)
constexpr int kCsOffSel = kCsOffHist;
constexpr int kCsOffPre = kCsOffHist + 4096 * 4;
static_assert(kMaxKInt * 8 <= 4096 * 4, "sel must fit in the histogram it aliases");
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
  const int row = xcd_row(blockIdx.x, gridDim.x), tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
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
  if (__any(ovf) && lane == 0) flag_set(a.overflow);
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
    // merge the four sorted segments by rank: a key's output position is its position in
    // its own segment plus the keys above it in the other three (binary searches; keys are
    // distinct) — every thread emits its own keys, no second sort
    int seg_off[kSelectThreads / 64 + 1], m = 0;
#pragma unroll
    for (int w = 0; w < kSelectThreads / 64; ++w) {
      seg_off[w] = m;
      m += min(min(max(n - w * 512, 0), 512), a.K);
    }
    seg_off[kSelectThreads / 64] = m;
    uint64_t mk[2];
    int rk[2];
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int i = tid + e * kSelectThreads;
      mk[e] = i < m ? sel[i] : 0ull;
      rk[e] = 0;
      if (i >= m) continue;
#pragma unroll
      for (int w = 0; w < kSelectThreads / 64; ++w) {
        const int b = seg_off[w], L = seg_off[w + 1] - b;
        if (i >= b && i < b + L) {
          rk[e] += i - b;
          continue;
        }
        int lo = 0, hi = L;  // keys of segment w above mk: the first index below it
        while (lo < hi) {
          const int mid = (lo + hi) >> 1;
          if (sel[b + mid] > mk[e]) lo = mid + 1;
          else hi = mid;
        }
        rk[e] += lo;
      }
    }
    uint64_t* head = red;  // the rank-0 key (red[0..3] were consumed above)
#pragma unroll
    for (int e = 0; e < 2; ++e)
      if (tid + e * kSelectThreads < m && rk[e] == 0) *head = mk[e];
    __syncthreads();
    if (sa.out_scores) {
      const int start = (drop && m && *head == drop) ? 1 : 0;
      const int c = min(sa.k_final, m - start);
      float* sc = sa.out_scores + (size_t)row * sa.k_final;
      int64_t* id = sa.out_ids + (size_t)row * sa.k_final;
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const int pos = rk[e] - start;
        if (tid + e * kSelectThreads < m && pos >= 0 && pos < c) {
          sc[pos] = float_of_ord(ordk_of(mk[e]));
          id[pos] = out_id(sa.idmap, gid_of(mk[e]));
        }
      }
      for (int i = c + tid; i < sa.k_final; i += kSelectThreads) {
        sc[i] = 0.f;
        id[i] = -1;
      }
      if (sa.out_counts && tid == 0) sa.out_counts[row] = c;
      return;
    }
    uint64_t* out = sa.keys_out + (size_t)row * sa.K;
#pragma unroll
    for (int e = 0; e < 2; ++e)
      if (tid + e * kSelectThreads < m && rk[e] < sa.K) out[rk[e]] = mk[e];
    for (int i = m + tid; i < sa.K; i += kSelectThreads) out[i] = 0ull;
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

// ---- streaming top-K, second stage: one wave per query ---------------------------------------
// The workgroup-per-query kernel above spends its time in a full bitonic sort of every
// candidate (~8·K_int per query at configs[3]) by four waves and a merge by binary searches.
// Here one wave owns a query and only finds the K-th largest key: the candidates sit in
// registers (up to 2,048 per wave, 32 per lane), the K-th largest score image by bisection
// over its 32 bits (per step: a compare and a ballot popcount per register — no LDS, no
// barriers), starting below the common prefix of the smallest and largest image; equal
// images at the K-th place (rare) are split by a second bisection over the item word.  The
// K keys above it are compacted by ballot and sorted by wave_sort_emit.  More than 2,048
// candidates (a bound far from the data): the top K of every 1,024-key page, then the top K
// of those; past kMaxKInt survivors, the bisection over pages re-read at every step.  Same
// outputs as cand_select_kernel, bit for bit.
constexpr int kCswWaves = kSelectThreads / 64;  // queries per workgroup
constexpr int kCswNJ = 32;                      // candidate registers per lane (2,048 per wave)

template <int NJ, typename Fetch>
__device__ __forceinline__ int csw_select(Fetch fetch, int n, uint32_t K, uint64_t* sel, int lane) {
  const int pages = (n + 64 * NJ - 1) / (64 * NJ);
  uint64_t v[NJ];
  auto load = [&](int pg) __attribute__((always_inline)) {
    int idx[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) idx[j] = pg * 64 * NJ + j * 64 + lane;
#pragma unroll
    for (int j = 0; j < NJ; ++j) v[j] = idx[j] < n ? fetch(idx[j]) : 0ull;
  };
  // keys satisfying pred over all pages (real keys have a non-zero score image; empty slots 0)
  auto count = [&](auto pred) __attribute__((always_inline)) {
    uint32_t c = 0;
    for (int pg = 0; pg < pages; ++pg) {
      if (pages > 1) load(pg);
#pragma unroll
      for (int j = 0; j < NJ; ++j) c += (uint32_t)__popcll(__ballot(pred(v[j])));
    }
    return c;
  };
  load(0);
  uint32_t mn = 0xFFFFFFFFu, mx = 0u;
  for (int pg = 0; pg < pages; ++pg) {
    if (pages > 1) load(pg);
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const uint32_t h = (uint32_t)(v[j] >> 32);
      mn = v[j] && h < mn ? h : mn;
      mx = h > mx ? h : mx;
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const uint32_t a = (uint32_t)__shfl_xor((int)mn, o), b = (uint32_t)__shfl_xor((int)mx, o);
    mn = a < mn ? a : mn;
    mx = b > mx ? b : mx;
  }
  // p = the K-th largest image: the largest t with count(image >= t) >= K; mn <= p <= mx, so
  // the bits above their highest differing bit are fixed
  const uint32_t d = mn ^ mx;
  const int hb = d ? 31 - __builtin_clz(d) : -1;
  uint32_t p = hb < 0 ? mx : hb >= 31 ? 0u : (mx & ~((2u << hb) - 1u));
  for (int b = hb; b >= 0; --b) {
    const uint32_t t = p | (1u << b);
    if (count([&](uint64_t k) { return (uint32_t)(k >> 32) >= t; }) >= K) p = t;
  }
  const uint32_t c_ge = count([&](uint64_t k) { return (uint32_t)(k >> 32) >= p; });
  uint32_t pl = 0u;  // item word bound among the keys whose image is p (when they tie there)
  if (c_ge > K) {
    const uint32_t need = K - count([&](uint64_t k) { return (uint32_t)(k >> 32) > p; });
    for (int b = 31; b >= 0; --b) {
      const uint32_t t = pl | (1u << b);
      if (count([&](uint64_t k) { return (uint32_t)(k >> 32) == p && (uint32_t)k >= t; }) >= need) pl = t;
    }
  }
  const uint64_t kth = ((uint64_t)p << 32) | pl;
  uint32_t m = 0;
  for (int pg = 0; pg < pages; ++pg) {
    if (pages > 1) load(pg);
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      // empty keys (0: padding, a carry list shorter than K) never count: with fewer than K
      // real keys kth is 0, and a page must still return at most K keys
      const bool take = v[j] != 0ull && v[j] >= kth;
      const uint64_t bal = __ballot(take);
      const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
      if (take && m + below < (uint32_t)kMaxKInt) sel[m + below] = v[j];
      m += (uint32_t)__popcll(bal);
    }
  }
  return (int)(m < (uint32_t)kMaxKInt ? m : (uint32_t)kMaxKInt);
}

__global__ __launch_bounds__(kSelectThreads) void cand_select_wave_kernel(CandSelectArgs a, int B) {
  __shared__ uint32_t pre_all[kCswWaves][kCsRegionsMax + 1];
  __shared__ __attribute__((aligned(16))) uint64_t sel_all[kCswWaves][kMaxKInt];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int row = xcd_row(blockIdx.x, gridDim.x) * kCswWaves + wave;
  if (row >= B) return;  // whole wave; no workgroup barriers below
  uint32_t* pre = pre_all[wave];
  uint64_t* sel = sel_all[wave];
  const int R = a.regions, Q = (R + 63) >> 6;  // regions per lane, consecutive
  const size_t rbase = (size_t)row * R;
  uint32_t c[16], sum = 0, ovf = 0;
  uint64_t gm = (a.cand_pmax && a.max_in && lane == 0) ? a.max_in[row] : 0ull;
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int r = lane * Q + q;
    const bool in = q < Q && r < R;
    const uint32_t raw = in ? a.cand_cnt[rbase + r] : 0u;
    ovf |= raw > (uint32_t)a.cap ? 1u : 0u;
    c[q] = raw < (uint32_t)a.cap ? raw : (uint32_t)a.cap;
    sum += c[q];
    if (a.cand_pmax && in) {
      const uint64_t k = a.cand_pmax[rbase + r];
      gm = k > gm ? k : gm;
    }
  }
  if (__any(ovf) && lane == 0) flag_set(a.overflow);
  uint32_t incl = sum;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = (uint32_t)__shfl_up((int)incl, o);
    incl += lane >= o ? y : 0u;
  }
  const uint32_t total = (uint32_t)__shfl((int)incl, 63);
  uint32_t off = incl - sum;
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int r = lane * Q + q;
    if (q < Q && r < R) pre[r] = off;
    off += c[q];
  }
  if (lane == 0) pre[R] = total;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const uint64_t y = __shfl_xor(gm, o);
    gm = y > gm ? y : gm;
  }
  const uint64_t gmax = a.cand_pmax ? gm : 0ull;
  if (a.cand_pmax && a.max_out && lane == 0) a.max_out[row] = gmax;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

  const uint64_t* carry = a.carry_in ? a.carry_in + (size_t)row * a.K : nullptr;
  int top = 1;  // the largest power of two <= R
  while (2 * top <= R) top <<= 1;
  // candidate i -> its region (the last region starting at or below i) and slot
  auto fetch = [&](int i) __attribute__((always_inline)) -> uint64_t {
    if (i >= (int)total) return carry[i - (int)total];
    int lo = 0;
    for (int st = top; st > 0; st >>= 1) {
      const int m = lo + st;
      if (m < R && pre[m] <= (uint32_t)i) lo = m;
    }
    return a.cand[(rbase + lo) * (size_t)a.cap + (i - (int)pre[lo])];
  };
  const int n = (int)total + (carry ? a.K : 0);
  int m;
  if (n <= a.K || n <= 256) {  // every candidate goes to the sort (n <= kMaxKInt)
    for (int i = lane; i < n; i += 64) sel[i] = fetch(i);
    m = n;
  } else if (n <= 512) {
    m = csw_select<8>(fetch, n, (uint32_t)a.K, sel, lane);
  } else if (n <= 1024) {
    m = csw_select<16>(fetch, n, (uint32_t)a.K, sel, lane);
  } else if (n <= 64 * kCswNJ) {
    m = csw_select<kCswNJ>(fetch, n, (uint32_t)a.K, sel, lane);
  } else if ((n + 1023) / 1024 * a.K <= kMaxKInt) {
    // more than 2,048: the top K of each 1,024-key page (the global top K is among them),
    // then the top K of those survivors — every step on registers, no re-reads (pages of
    // 1,024, not 2,048: a second 32-register set would cost the kernel a wave per SIMD)
    int ms = 0;
    for (int b0 = 0; b0 < n; b0 += 1024) {
      const int np = min(1024, n - b0);
      auto fp = [&](int i) __attribute__((always_inline)) { return fetch(b0 + i); };
      if (np <= a.K) {
        for (int i = lane; i < np; i += 64) sel[ms + i] = fp(i);
        ms += np;
      } else {
        ms += csw_select<16>(fp, np, (uint32_t)a.K, sel + ms, lane);
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    auto fs = [&](int i) __attribute__((always_inline)) { return sel[i]; };
    m = ms <= a.K ? ms : csw_select<8>(fs, ms, (uint32_t)a.K, sel, lane);  // ms <= kMaxKInt
  } else {  // (pages·K > kMaxKInt) the bisection over pages re-read at every step
    m = csw_select<kCswNJ>(fetch, n, (uint32_t)a.K, sel, lane);
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  SelectArgs sa{};
  sa.K = a.K;
  sa.keys_out = a.keys_out;
  sa.out_scores = a.out_scores;
  sa.out_ids = a.out_ids;
  sa.out_counts = a.out_counts;
  sa.k_final = a.k_final;
  if (m <= 64) wave_sort_emit<1>(sel, m, sa, row, gmax);
  else if (m <= 128) wave_sort_emit<2>(sel, m, sa, row, gmax);
  else if (m <= 256) wave_sort_emit<4>(sel, m, sa, row, gmax);
  else wave_sort_emit<8>(sel, m, sa, row, gmax);
}

// ---- exact re-rank, second stage (SelectArgs.rr_*) ------------------------------------------
// One workgroup per query: the exact rank 0 from its approximate candidates, then the
// candidates within 2ε of the K-th approximate score rescored from the f32 rows (16-lane
// groups, four rows in flight per group), sorted by the exact key and emitted as the final
// list (rank 0 dropped when it heads it) or the key list.  Rows the select flagged kRrSlow
// (masses of items at the bound) take the exact running top-K over the whole row.
constexpr int kRrOffQ = 2560 * 8;
constexpr int kRrOffMisc = kRrOffQ + kRrMaxD * 4;
constexpr int kRrLds = kRrOffMisc + 256;

// Exact finish of a re-rank row (shared by select_kernel's fused path and rerank_kernel):
// cand[0..m) holds the approximate candidates within 2ε of the K-th (m = kRrSlow: masses at
// the gather bound Tg, the exact slow path), cand[2048..2048+n0) the rank-0 candidates
// (n0 = kRrSlow: every present item within thr0 of the present maximum).  Rescores them from
// the f32 rows, resolves rank 0 into max_inout and emits the final list / key list.
template <typename Elig, typename SAt>
__device__ __forceinline__ void rr_finish(const SelectArgs& a, int row, int n, uint64_t* cand, uint32_t* misc, const float* qs,
                          uint32_t m, uint32_t n0, uint32_t Tg, uint32_t thr0, Elig elig, SAt s_at) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int K = a.K, ntiles = (n + 31) >> 5;
  const int64_t w0 = a.slab_start >> 5;
  if (tid == 0) *(uint64_t*)(misc + 10) = 0ull;
  __syncthreads();
  // ---- exact rank 0 ----
  if (a.max_inout) {
    uint64_t best0 = 0;
    if (n0 != kRrSlow) {
      rr_rescore_any(cand + 2048, (int)n0, a, qs);
      __syncthreads();
      for (int i = tid; i < (int)n0; i += kSelectThreads) best0 = cand[2048 + i] > best0 ? cand[2048 + i] : best0;
    } else {  // masses of near-duplicates at the top: every present item within the margin,
              // collected 256 per round into cand[2048..2560) and rescored in batches
      const uint32_t* prow = a.pmax + (size_t)row * a.ldt;
      uint64_t* rb = cand + 2048;
      if (tid == 0) misc[15] = 0;
      __syncthreads();
      const int nall = ntiles * 32;
      for (int base = 0; base < nall; base += kSelectThreads) {
        const int i = base + tid;
        if (i < n && prow[i >> 5] >= thr0) {
          const int t = i >> 5, it = i & 31;
          const uint32_t pw = a.present ? a.present[w0 + t] : ~0u;
          if (((pw >> it) & 1u) && ord_of(s_at(i)) >= thr0) rb[atomicAdd(&misc[15], 1u)] = make_key(1u, a.gid0 + (uint32_t)i);
        }
        __syncthreads();
        const int nb = (int)misc[15];
        __syncthreads();  // every thread holds nb before the next round's appends
        if (nb > 256 || (base + kSelectThreads >= nall && nb > 0)) {
          rr_rescore_any(rb, nb, a, qs);
          __syncthreads();
          for (int k = tid; k < nb; k += kSelectThreads) best0 = rb[k] > best0 ? rb[k] : best0;
          __syncthreads();
          if (tid == 0) misc[15] = 0;
          __syncthreads();
        }
      }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const uint64_t y = __shfl_xor(best0, o);
      best0 = y > best0 ? y : best0;
    }
    if (lane == 0) atomicMax((unsigned long long*)(misc + 10), (unsigned long long)best0);
    __syncthreads();
    if (tid == 0) a.max_inout[row] = *(const uint64_t*)(misc + 10);
  }
  if (m == kRrSlow) {
    rr_slow_path(a, row, n, Tg, K, cand, misc, qs, elig, s_at);
    return;
  }
  rr_rescore_any(cand, (int)m, a, qs);
  __syncthreads();
  if (a.trace && threadIdx.x == 0) a.trace[row * 8 + 6] = __builtin_amdgcn_s_memrealtime();
  const uint64_t gmax = *(const uint64_t*)(misc + 10);
  if (wave != 0) return;
  if (m <= 64) wave_sort_emit<1>(cand, (int)m, a, row, gmax);
  else if (m <= 128) wave_sort_emit<2>(cand, (int)m, a, row, gmax);
  else if (m <= 256) wave_sort_emit<4>(cand, (int)m, a, row, gmax);
  else wave_sort_emit<8>(cand, (int)m, a, row, gmax);
}

__global__ __launch_bounds__(kSelectThreads) void rerank_kernel(SelectArgs a) {
  __shared__ __attribute__((aligned(16))) char dsm[kRrLds];
  uint64_t* cand = (uint64_t*)dsm;
  float* qs = (float*)(dsm + kRrOffQ);
  uint32_t* misc = (uint32_t*)(dsm + kRrOffMisc);
  const int row = xcd_row(blockIdx.x, gridDim.x), tid = threadIdx.x;
  const int n = a.n_cols;
  const float sh = a.s_h ? a.s_h[row] : 0.f;
  auto s_at = [&](int j) -> float { return s_at_ld(a, row, j, sh); };
  const uint32_t* excl = a.excl ? a.excl + (size_t)row * a.excl_ld : nullptr;
  const int64_t w0 = a.slab_start >> 5;
  auto elig = [&](int tile) -> uint32_t {
    const uint32_t* pp = a.present ? a.present + w0 + tile : &kWordOnes;
    const uint32_t* mp = a.mask ? a.mask + w0 + tile : &kWordOnes;
    const uint32_t* ep = excl ? excl + w0 + tile : &kWordZero;
    return *pp & *mp & ~*ep;
  };
  const uint32_t m = a.rr_cnt[row];
  const uint64_t* src = a.rr_out + (size_t)row * kRrCap;
  const float4* qg = (const float4*)(a.rr_q + (size_t)row * a.rr_ld);
  for (int i = tid; i < (a.rr_d >> 2); i += kSelectThreads) ((float4*)qs)[i] = qg[i];
  if (m != kRrSlow)
    for (int i = tid; i < (int)m; i += kSelectThreads) cand[i] = src[i];
  uint32_t n0 = 0;
  if (a.max_inout) {
    n0 = a.rr_r0n[row];
    if (n0 != kRrSlow)
      for (int i = tid; i < (int)n0; i += kSelectThreads) cand[2048 + i] = make_key(1u, a.rr_r0[(size_t)row * kRrR0Cap + i]);
  }
  __syncthreads();
  rr_finish(a, row, n, cand, misc, qs, m, n0, a.rr_thr[2 * row], a.max_inout ? a.rr_thr[2 * row + 1] : 0u, elig, s_at);
}

// ---- one wave per query: the exact re-rank select of a one-slab search ----------------------
// The block select above keeps four waves resident per query for ~25 us, mostly waiting on
// memory; with three batches in flight that residency, not the scan, capped throughput
// (r02t: 256 scan CUs x 18 us + 256 select workgroups x 25 us per batch).  Here one wave
// carries a query through the whole chain and ~8 queries share a CU:
//   maxima   lane l holds the eligible / present maxima of tiles l, l+64, ... (<= 16 each)
//   bound    T0 = the K-th largest TILE maximum (ballot bit loop over 16 values per lane):
//            tighter than the block select's per-thread bound, so ~K tiles qualify
//   gather   tiles with maxima >= Tg = T0 - 2ε; their eligible items >= Tg (approximate keys)
//   rank 0   (similar / hybrid content side) present items within 2ε of the present maximum
//   rescore  every candidate and rank-0 item from the f32 rows (16 lanes per row, U rows in
//            flight per lane group, f64 sums in rr_rescore's fixed order)
//   emit     register bitonic sort, rank-0 drop, final list or key list
// A query that overflows a cap (masses of near-ties) sets rr_flags[row]; the block select
// then runs that row alone (its launch returns at once for every other row).
constexpr int kWvTPL = 16;     // tile maxima per lane: slabs of up to 1024 tiles (32,768 columns)
constexpr int kWvCand = 256;   // candidates (sorted by one wave in registers)
constexpr int kWvTiles = 256;  // qualifying tiles
constexpr int kWvR0 = 64;      // rank-0 items
constexpr int kWvR0Tiles = 16;
constexpr int kWvOffCand = 0;                              // u64 [kWvCand + kWvR0]
constexpr int kWvOffTl = kWvOffCand + (kWvCand + kWvR0) * 8;  // u32 [kWvTiles]
constexpr int kWvOffR0t = kWvOffTl + kWvTiles * 4;        // u32 [kWvR0Tiles]
constexpr int kWvOffQs = kWvOffR0t + kWvR0Tiles * 4;      // f32 [kRrMaxD]
constexpr int kWvOffMisc = kWvOffQs + kRrMaxD * 4;        // u32 [8]
constexpr int kWvLds = kWvOffMisc + 32;

// UM: rows in flight per lane group, as a multiple of the block select's budget.  The
// rescore is a chain of dependent row gathers (~1 us each from the MALL), so with one query
// wave per SIMD (B <= ~1K) more rows per round pay; with several waves per SIMD the extra
// registers cost occupancy instead (launch_select_rr_wave picks).
template <int UM>
__device__ __forceinline__ void wave_rescore_any(uint64_t* keys, int m, const SelectArgs& a, const float* qs, int lane) {
  const int cpl = ((a.rr_d >> 2) + 15) >> 4;
  if (cpl <= 1) rescore_rows<1, 12 * UM, 4>(keys, m, a, qs, lane);
  else if (cpl <= 2) rescore_rows<2, 6 * UM, 4>(keys, m, a, qs, lane);
  else if (cpl <= 4) rescore_rows<4, 3 * UM, 4>(keys, m, a, qs, lane);
  else if (cpl <= 6) rescore_rows<6, 2 * UM, 4>(keys, m, a, qs, lane);
  else rescore_rows<8, 1 * UM, 4>(keys, m, a, qs, lane);
}

template <int UM>
__device__ __forceinline__ void select_rr_wave_body(const SelectArgs& a, int row) {
  __shared__ __attribute__((aligned(16))) char dsm[kWvLds];
  uint64_t* cand = (uint64_t*)(dsm + kWvOffCand);
  uint32_t* tl = (uint32_t*)(dsm + kWvOffTl);
  uint32_t* r0t = (uint32_t*)(dsm + kWvOffR0t);
  float* qs = (float*)(dsm + kWvOffQs);
  uint32_t* misc = (uint32_t*)(dsm + kWvOffMisc);
  const int lane = threadIdx.x;
  const int n = a.n_cols, K = a.K;
  const int ntiles = (n + 31) >> 5;
  const float sh = a.s_h ? a.s_h[row] : 0.f;  // int16 score image: decode quantum
  auto s_quad = [&](int t, int g) -> float4 { return s_quad_ld(a, row, t, g, sh); };
  auto s_at = [&](int j) -> float { return s_at_ld(a, row, j, sh); };
  const uint32_t* trow = a.tmax + (size_t)row * a.ldt;
  const uint32_t* prow = a.max_inout ? a.pmax + (size_t)row * a.ldt : nullptr;
  const uint32_t* excl = a.excl ? a.excl + (size_t)row * a.excl_ld : nullptr;
  const int64_t w0 = a.slab_start >> 5;
  auto elig = [&](int tile) -> uint32_t {
    const uint32_t* pp = a.present ? a.present + w0 + tile : &kWordOnes;
    const uint32_t* mp = a.mask ? a.mask + w0 + tile : &kWordOnes;
    const uint32_t* ep = excl ? excl + w0 + tile : &kWordZero;
    return *pp & *mp & ~*ep;
  };
  auto flag = [&]() {
    if (lane == 0) a.rr_flags[row] = 1u;
  };
  auto stamp = [&](int slot) {  // probe-only phase timeline (s_memrealtime, 100 MHz)
    if (a.trace && lane == 0) a.trace[row * 8 + slot] = __builtin_amdgcn_s_memrealtime();
  };
  stamp(0);

  // ---- loads: maxima (and present maxima), the f32 query row, ε ----
  uint32_t tm[kWvTPL], pm[kWvTPL];
#pragma unroll
  for (int j = 0; j < kWvTPL; ++j) {
    const int t = lane + 64 * j;
    tm[j] = t < ntiles ? trow[t] : 0u;
    pm[j] = (prow && t < ntiles) ? prow[t] : 0u;
  }
  const int nq4 = a.rr_d >> 2;
  float4 qv0 = make_float4(0.f, 0.f, 0.f, 0.f), qv1 = qv0;
  const float4* qg = (const float4*)(a.rr_q + (size_t)row * a.rr_ld);
  if (lane < nq4) qv0 = qg[lane];
  if (lane + 64 < nq4) qv1 = qg[lane + 64];
  const float eps2 = rr_margin(a.rr_eps[row]);
  if (lane < nq4) ((float4*)qs)[lane] = qv0;
  if (lane + 64 < nq4) ((float4*)qs)[lane + 64] = qv1;

  // ---- bound: T0 = K-th largest tile maximum (0 maxima = no eligible item) ----
  auto cnt_ge = [&](uint32_t c) -> uint32_t {
    uint32_t s = 0;
#pragma unroll
    for (int j = 0; j < kWvTPL; ++j) s += (uint32_t)__popcll(__ballot(tm[j] >= c));
    return s;
  };
  uint32_t T0 = 1;  // fewer than K tiles with eligible items: every eligible item
  if (cnt_ge(1u) >= (uint32_t)K) {
    uint32_t hi = 0, lo = ~0u;
#pragma unroll
    for (int j = 0; j < kWvTPL; ++j) {
      hi = max(hi, tm[j]);
      lo = min(lo, tm[j] ? tm[j] : ~0u);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      hi = max(hi, (uint32_t)__shfl_xor((int)hi, o));
      lo = min(lo, (uint32_t)__shfl_xor((int)lo, o));
    }
    hi = __builtin_amdgcn_readfirstlane(hi);
    lo = __builtin_amdgcn_readfirstlane(lo);
    const uint32_t d = hi ^ lo;
    const int top = d ? 31 - __builtin_clz(d) : -1;
    uint32_t P = top < 0 ? hi : top >= 31 ? 0u : hi & ~((2u << top) - 1u);
    for (int b = top; b >= 0; --b) {
      const uint32_t c = P | (1u << b);
      if (cnt_ge(c) >= (uint32_t)K) P = c;
    }
    T0 = P ? P : 1u;
  }
  const uint32_t Tg = ord_sub(T0, eps2);
  stamp(1);

  // ---- qualifying tiles -> list ----
  uint32_t ntl = 0;
#pragma unroll
  for (int j = 0; j < kWvTPL; ++j) {
    const uint64_t qm = __ballot(tm[j] >= Tg && lane + 64 * j < ntiles);
    const uint32_t pos = ntl + __builtin_amdgcn_mbcnt_hi((uint32_t)(qm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)qm, 0u));
    if (((qm >> lane) & 1ull) && pos < (uint32_t)kWvTiles) tl[pos] = (uint32_t)(lane + 64 * j);
    ntl += (uint32_t)__popcll(qm);
  }
  // rank 0: the present maximum (order image, lowest tile) and its margin
  uint32_t Pm = 0, thr0 = 0, nt0 = 0;
  if (prow) {
#pragma unroll
    for (int j = 0; j < kWvTPL; ++j) Pm = max(Pm, pm[j]);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) Pm = max(Pm, (uint32_t)__shfl_xor((int)Pm, o));
    Pm = __builtin_amdgcn_readfirstlane(Pm);
    thr0 = ord_sub(Pm, eps2);
    if (Pm) {
#pragma unroll
      for (int j = 0; j < kWvTPL; ++j) {
        const uint64_t qm = __ballot(pm[j] >= thr0 && lane + 64 * j < ntiles);
        const uint32_t pos = nt0 + __builtin_amdgcn_mbcnt_hi((uint32_t)(qm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)qm, 0u));
        if (((qm >> lane) & 1ull) && pos < (uint32_t)kWvR0Tiles) r0t[pos] = (uint32_t)(lane + 64 * j);
        nt0 += (uint32_t)__popcll(qm);
      }
    }
  }
  if (ntl > (uint32_t)kWvTiles || nt0 > (uint32_t)kWvR0Tiles) return flag();
  stamp(2);
  if (lane == 0) misc[0] = 0u, misc[1] = 0u;
  __syncthreads();  // (one wave: orders the LDS list writes before the reads below)

  // ---- gather: eight lanes per qualifying tile (one 16-B score quad each, so a wave load
  // reads eight whole 128-B tile rows), up to 128 tiles per round with every load issued
  // before any is used ----
  // candidates are compacted by ballots (a uniform running count, no LDS atomics: the
  // lanes of a round hitting one counter serialised the atomics)
  uint32_t nc = 0;
  {
    constexpr int kGP = 24;  // tiles per lane group per round: one round up to 192 tiles
    const int sub = lane & 7, grp = lane >> 3;
    for (uint32_t base = 0; base < ntl; base += 8 * kGP) {
      float4 v[kGP];
      uint32_t okw[kGP];
      int tt[kGP];
#pragma unroll
      for (int p = 0; p < kGP; ++p) {
        const uint32_t i = base + 8 * p + grp;
        tt[p] = i < ntl ? (int)tl[i] : -1;
      }
#pragma unroll
      for (int p = 0; p < kGP; ++p) {
        const int t = tt[p] < 0 ? (int)tl[0] : tt[p];
        v[p] = s_quad(t, sub);
        okw[p] = elig(t);
      }
#pragma unroll
      for (int p = 0; p < kGP; ++p) {
        const int t = tt[p];
        const float f[4] = {v[p].x, v[p].y, v[p].z, v[p].w};
        uint32_t m = 0;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const int it = 4 * sub + c;
          m |= (t >= 0 && t * 32 + it < n && ((okw[p] >> it) & 1u) && ord_of(f[c]) >= Tg) ? (1u << c) : 0u;
        }
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const uint64_t bm = __ballot((m >> c) & 1u);
          if ((m >> c) & 1u) {
            const uint32_t q = nc + __builtin_amdgcn_mbcnt_hi((uint32_t)(bm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bm, 0u));
            if (q < (uint32_t)kWvCand) cand[q] = make_key(ord_of(f[c]), a.gid0 + (uint32_t)(t * 32 + 4 * sub + c));
          }
          nc += (uint32_t)__popcll(bm);
        }
      }
    }
  }
  if (lane == 0) misc[0] = nc;
  // rank-0 items: present, within the margin of the present maximum
  uint64_t* r0k = cand + kWvCand;
  for (uint32_t i = lane; i < nt0 * 32; i += 64) {
    const int t = (int)r0t[i >> 5], it = (int)(i & 31), j = t * 32 + it;
    const uint32_t pw = a.present ? a.present[w0 + t] : ~0u;
    if (j < n && ((pw >> it) & 1u) && ord_of(s_at(j)) >= thr0) {
      const uint32_t q = atomicAdd(&misc[1], 1u);
      if (q < (uint32_t)kWvR0) r0k[q] = make_key(1u, a.gid0 + (uint32_t)j);
    }
  }
  __syncthreads();
  const uint32_t cnt = __builtin_amdgcn_readfirstlane(misc[0]);
  const uint32_t n0 = __builtin_amdgcn_readfirstlane(misc[1]);
  if (cnt > (uint32_t)kWvCand || n0 > (uint32_t)kWvR0) return flag();
  stamp(3);

  // ---- rescore candidates and rank-0 items (rank-0 keys right behind the candidates) ----
  for (uint32_t i = lane; i < n0; i += 64) cand[cnt + i] = r0k[i];
  __syncthreads();
  wave_rescore_any<UM>(cand, (int)(cnt + n0), a, qs, lane);
  __syncthreads();
  stamp(4);
  uint64_t gmax = 0;
  for (uint32_t i = lane; i < n0; i += 64) gmax = cand[cnt + i] > gmax ? cand[cnt + i] : gmax;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const uint64_t y = __shfl_xor(gmax, o);
    gmax = y > gmax ? y : gmax;
  }
  if (a.max_inout && lane == 0) a.max_inout[row] = gmax;
  if (lane == 0) a.rr_flags[row] = 0u;
  if (cnt <= 64) wave_sort_emit<1>(cand, (int)cnt, a, row, gmax);
  else if (cnt <= 128) wave_sort_emit<2>(cand, (int)cnt, a, row, gmax);
  else wave_sort_emit<4>(cand, (int)cnt, a, row, gmax);
  stamp(5);
  if (a.trace && lane == 0) a.trace[row * 8 + 6] = cnt, a.trace[row * 8 + 7] = ntl;
}

template <int UM>
__global__ __launch_bounds__(64) void select_rr_wave_kernel(SelectArgs a) {
  select_rr_wave_body<UM>(a, xcd_row(blockIdx.x, gridDim.x));
}
// both sides of a hybrid search: workgroups [0, B0) side 0, the rest side 1
__global__ __launch_bounds__(64) void select_rr_wave_dual_kernel(SelectArgs a0, SelectArgs a1, int B0, int B1) {
  if ((int)blockIdx.x < B0)
    select_rr_wave_body<2>(a0, xcd_row(blockIdx.x, B0));
  else
    select_rr_wave_body<2>(a1, xcd_row(blockIdx.x - B0, B1));
}

hipError_t launch_select_rr_wave(const SelectArgs& a, int B, hipStream_t s) {
  if (!a.rr_eps || !a.rr_x || !a.rr_q || !a.rr_flags || a.rr_out || a.carry_in || a.rr_d <= 0 || a.rr_d > kRrMaxD ||
      (a.rr_d & 3) || a.K <= 0 || a.K > kWvCand || B <= 0 || a.n_cols <= 0 || a.n_cols > 64 * kWvTPL * 32 || !a.tmax ||
      (a.max_inout && !a.pmax) || (a.slab_start & 31) || (a.out_scores && a.k_final > kWvCand))
    return hipErrorInvalidValue;
  // two waves per SIMD at most for the fat variant: 256 CUs x 4 SIMDs x 2
  static const int um_env = ab_env("BB_WAVE_UM") ? atoi(ab_env("BB_WAVE_UM")) : 0;
  const bool fat = um_env ? um_env == 2 : true;
  if (fat)
    bb_launch(select_rr_wave_kernel<2>, dim3(B), dim3(64), 0, s, a);
  else
    bb_launch(select_rr_wave_kernel<1>, dim3(B), dim3(64), 0, s, a);
  return hipGetLastError();
}

// Both sides of a hybrid re-rank search (one slab, query chunks > 256 rows): the one-wave
// selects of the two sides in one launch, then the block select of the rows they left.
hipError_t launch_select_rr_wave_dual(const SelectArgs& a0, const SelectArgs& a1, int B, hipStream_t s) {
  for (const SelectArgs* a : {&a0, &a1})
    if (!a->rr_eps || !a->rr_x || !a->rr_q || !a->rr_flags || a->rr_out || a->carry_in || a->rr_d <= 0 ||
        a->rr_d > kRrMaxD || (a->rr_d & 3) || a->K <= 0 || a->K > kWvCand || B <= 0 || a->n_cols <= 0 ||
        a->n_cols > 64 * kWvTPL * 32 || !a->tmax || (a->max_inout && !a->pmax) || (a->slab_start & 31) ||
        a->out_scores || a->rr_d > 4 * kSelectThreads)
      return hipErrorInvalidValue;
  bb_launch(select_rr_wave_dual_kernel, dim3(2 * B), dim3(64), 0, s, a0, a1, B, B);
  bb_launch(select_rr_dual_kernel, dim3(2 * B), dim3(kSelectThreads), 0, s, a0, a1, B, B);
  return hipGetLastError();
}

hipError_t launch_rerank(const SelectArgs& a, int B, hipStream_t s) {
  if (!a.rr_eps || !a.rr_x || !a.rr_q || !a.rr_out || !a.rr_cnt || !a.rr_thr || (a.max_inout && (!a.rr_r0 || !a.rr_r0n)) ||
      a.rr_d <= 0 || a.rr_d > kRrMaxD || (a.rr_d & 3) || a.K <= 0 || a.K > kMaxKInt || B <= 0)
    return hipErrorInvalidValue;
  bb_launch(rerank_kernel, dim3(B), dim3(kSelectThreads), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_cand_select(const CandSelectArgs& a, int B, hipStream_t s) {
  if (a.K <= 0 || a.K > kMaxKInt || B <= 0 || a.regions <= 0 || a.regions > kCsRegionsMax || a.cap <= 0 ||
      !a.cand || !a.cand_cnt || !a.overflow || (!a.out_scores && !a.keys_out))
    return hipErrorInvalidValue;
  static const bool wg_path = ab_env("BB_CS_WG") != nullptr;  // A/B: the workgroup-per-query kernel
  if (wg_path)
    bb_launch(cand_select_kernel, dim3(B), dim3(kSelectThreads), 0, s, a);
  else
    bb_launch(cand_select_wave_kernel, dim3((B + kCswWaves - 1) / kCswWaves), dim3(kSelectThreads), 0, s, a, B);
  return hipGetLastError();
}

hipError_t launch_select(const SelectArgs& a, int B, hipStream_t s) {
  if (a.K <= 0 || a.K > kMaxKInt || B <= 0 || a.n_cols <= 0 || !a.tmax || (a.max_inout && !a.pmax) ||
      (a.slab_start & 31))
    return hipErrorInvalidValue;
  // re-rank (rr_eps set): operands always; the hand-off buffers only for the split launch
  if (a.rr_eps && (!a.rr_x || !a.rr_q || a.rr_d <= 0 || a.rr_d > kRrMaxD || (a.rr_d & 3) || a.rr_d > 4 * kSelectThreads ||
                   (a.rr_out && (!a.rr_cnt || !a.rr_thr || (a.max_inout && (!a.rr_r0 || !a.rr_r0n))))))
    return hipErrorInvalidValue;
  if (a.rr_eps) {
    bb_launch((select_kernel<0, true>), dim3(B), dim3(kSelectThreads), 0, s, a);
    return hipGetLastError();
  }
  static const int abl = ab_env("BB_SELECT_ABLATE") ? atoi(ab_env("BB_SELECT_ABLATE")) : 0;
  switch (abl) {
    case 1: bb_launch(select_kernel<1>, dim3(B), dim3(kSelectThreads), 0, s, a); break;
    case 2: bb_launch(select_kernel<2>, dim3(B), dim3(kSelectThreads), 0, s, a); break;
    case 4: bb_launch(select_kernel<4>, dim3(B), dim3(kSelectThreads), 0, s, a); break;
    case 8: bb_launch(select_kernel<8>, dim3(B), dim3(kSelectThreads), 0, s, a); break;
    default: bb_launch(select_kernel<0>, dim3(B), dim3(kSelectThreads), 0, s, a);
  }
  return hipGetLastError();
}

}  // namespace bb
