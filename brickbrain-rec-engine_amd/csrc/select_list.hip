// select_list.hip — exact per-query top-K from the bounded candidate lists of a kScanList scan.
//
// Replaces the score-image select + rerank pair of the exact re-rank path (one slab, f32
// index) — np.argsort(sim)[::-1] + the filter walk of get_similar_sets
// (recommendation_system.py:214-247), the CF loop + sort (:438-461) and pgvector's
// ORDER BY <=> LIMIT k — for the 25K-row configs.  One workgroup (4 waves) per query row:
//
//   lists   every lane's top-5 keys per period (list_epi.h), packed: u16 codes + 7-bit positions
//   bound   T0 = the K-th largest code over ALL list keys (two-level histogram): K distinct
//           items have codes >= T0, so the exact K-th score is >= dec(T0) − ε', and every
//           exact top-K member has code >= Tg = T0 − Δ (Δ = the re-rank margin
//           2ε'(1+2^-10)+2^-20 in codes, + 2 codes of slack)
//   gather  keys >= Tg of the lists whose 5th key is below Tg (they dropped nothing that
//           matters); a list whose 5th key reaches Tg may have dropped candidates, so every
//           eligible item of its period joins the buffer instead (an overflowed list: a few
//           rows per batch at configs[1])
//   rank 0  (similar / hybrid content side) the present half tiles whose maximum is within Δ
//           of the largest; a lane whose 2nd-best half tile is also within Δ contributes its
//           whole chunk half.  Their present items join the same buffer (a region of their
//           own); the exact maximum among them is the unmasked arg-max key that the
//           similar-sets path drops (:217)
//   rescore the whole buffer in ONE pass from the f32 rows (f64 sums in rescore_rows' fixed
//           order, rounded to f32: the same bits as every other path), 64 rows in flight
//   emit    sort the candidates by (score desc, id asc) — one wave in registers up to 512,
//           an LDS bitonic network up to kLsCand — drop rank 0, write the list
// Buffer overflow (masses of near-duplicates, all-equal scores): an exact running top-K over
// every eligible item of the row (slow, never taken on distinct data; tests drive it).
#include "common.h"
#include "list_epi.h"
#include "qnorm.h"
#include "select_util.h"

namespace bb {

constexpr int kLsCand = 2048;   // rescore buffer (u64 keys): candidates + overflow items + rank-0 items
constexpr int kLsFlush = 1024;  // fallback: batch size that triggers a merge of the running top-K
constexpr int kLsSeg = 64;      // overflowed lists
constexpr int kLsR0Seg = 64;    // rank-0 segments
constexpr int kLsMaxLists = kListMaxPerRow;
constexpr int kLsOffCand = 0;
constexpr int kLsOffSel = kLsOffCand + kLsCand * 8;          // u64 [kMaxKInt] running top-K (fallback)
constexpr int kLsOffHist = kLsOffSel + kMaxKInt * 8;         // u32 [256] bound histogram
constexpr int kLsOffSeg = kLsOffHist + 256 * 4;              // u32 [kLsSeg][2] (t0, nt << 1 | h)
constexpr int kLsOffR0 = kLsOffSeg + kLsSeg * 8;             // u32 [kLsR0Seg][2]
constexpr int kLsOffQs = kLsOffR0 + kLsR0Seg * 8;            // f32 [kRrMaxD]
constexpr int kLsOffMisc = kLsOffQs + kRrMaxD * 4;           // u32 [16]
constexpr int kLsOffScan = kLsOffMisc + 64;                  // u32 [8]: block scan / find_bin words
constexpr int kLsOffAll = kLsOffScan + 32;                   // u32 [4] + [3]: every item of the row
constexpr int kLsLds = kLsOffAll + 32;
static_assert(kLsOffQs % 16 == 0, "query row must be 16-B aligned");
static_assert(kSelectThreads == 256, "one histogram bin per thread");
// misc words; M_GMAX is a u64 (8-byte aligned: misc starts 8-aligned)
enum { M_CAND = 0, M_SEG, M_R0SEG, M_BUF, M_PM, M_SEGN, M_R0N, M_GMAX = 8 };
static_assert(kLsOffMisc % 8 == 0, "u64 misc word must be 8-byte aligned");

// Fallback enumeration of segments (tile ranges of one lane half) in rounds of 256 items:
// item i of the concatenation -> (segment, tile, register) by binary search over the item
// prefix; items passing `keep` are appended to buf as placeholder keys; a batch reaching
// `flush` items is reduced (merge or max); at most flush - 1 + 256 items are buffered.  Every
// thread returns holding the same buffer count.
template <typename Keep, typename Reduce>
__device__ __forceinline__ void ls_stream(const uint32_t* seg, const uint32_t* pre, int nseg, uint64_t* buf, uint32_t* misc,
                          uint32_t gid0, int n, int flush, Keep keep, Reduce reduce) {
  const int tid = threadIdx.x;
  const uint32_t total = pre[nseg];
  for (uint32_t base = 0; base < total; base += kSelectThreads) {
    const uint32_t i = base + tid;
    if (i < total) {
      int lo = 0, hi = nseg;  // pre[lo] <= i < pre[hi]
      while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (pre[mid] <= i) lo = mid;
        else hi = mid;
      }
      const uint32_t off = i - pre[lo], t0 = seg[2 * lo], hh = seg[2 * lo + 1] & 1u;
      const int tile = (int)(t0 + (off >> 4)), g = (int)(off & 15u);
      const int it = (g & 3) + 8 * (g >> 2) + 4 * (int)hh, j = tile * 32 + it;
      if (j < n && keep(tile, it)) buf[atomicAdd(&misc[M_BUF], 1u)] = make_key(1u, gid0 + (uint32_t)j);
    }
    __syncthreads();
    const int nb = (int)misc[M_BUF];
    __syncthreads();  // every thread holds nb before anyone resets it
    if (nb >= flush || (base + kSelectThreads >= total && nb > 0)) reduce(nb);
  }
}

// Append the items of segments seg[0..ns) (tile t0, nt tiles, lane half h) that pass `keep`
// to buf at misc[M_CAND] (no capacity check beyond the buffer: the caller sized it).
template <typename Keep>
__device__ __forceinline__ void ls_append(const uint32_t* seg, int ns, uint64_t* buf, uint32_t* misc, uint32_t gid0, int n,
                                          Keep keep) {
  for (int s = 0; s < ns; ++s) {
    const int t0 = (int)seg[2 * s], hh = (int)(seg[2 * s + 1] & 1u), cnt = (int)(seg[2 * s + 1] >> 1) * 16;
    for (int i = threadIdx.x; i < cnt; i += kSelectThreads) {
      const int tile = t0 + (i >> 4), g = i & 15;
      const int it = (g & 3) + 8 * (g >> 2) + 4 * hh, j = tile * 32 + it;
      if (j < n && keep(tile, it)) {
        const uint32_t p = atomicAdd(&misc[M_CAND], 1u);
        if (p < (uint32_t)kLsCand) buf[p] = make_key(1u, gid0 + (uint32_t)j);
      }
    }
  }
}

// The rescore of the list select: 32 rows in flight per workgroup at d = 384, the query
// chunks re-read from LDS each round — the kernel fits 138 VGPRs, three workgroups per CU
// (the hybrid select runs 2·B of them).  The gathers are bound by the chip's bandwidth, not
// by rows in flight: at configs[1] 256 rows x ~90 candidates x 1.5 KB = 36 MB in ~6 us, and
// 3 us with every row gathering the same (cache-resident) item (r03_ab); 96 rows in flight
// (one round) measured no faster (r03_w).
__device__ __forceinline__ void ls_rescore(uint64_t* keys, int m, const SelectArgs& a, const float* qs) {
  const int cpl = ((a.rr_d >> 2) + 15) >> 4;
  const int t = threadIdx.x;
  if (cpl <= 1) rescore_rows<1, 8, 16, false>(keys, m, a, qs, t);
  else if (cpl <= 2) rescore_rows<2, 4, 16, false>(keys, m, a, qs, t);
  else if (cpl <= 4) rescore_rows<4, 2, 16, false>(keys, m, a, qs, t);
  else if (cpl <= 6) rescore_rows<6, 2, 16, false>(keys, m, a, qs, t);
  else rescore_rows<8, 1, 16, false>(keys, m, a, qs, t);   // rows up to kRrMaxD = 512 wide
}

__device__ __forceinline__ void select_list_body(const SelectArgs& a, int row) {
  __shared__ __attribute__((aligned(16))) char dsm[kLsLds];
  uint64_t* cand = (uint64_t*)(dsm + kLsOffCand);
  uint64_t* sel = (uint64_t*)(dsm + kLsOffSel);
  uint32_t* hist = (uint32_t*)(dsm + kLsOffHist);
  uint32_t* seg = (uint32_t*)(dsm + kLsOffSeg);
  uint32_t* r0s = (uint32_t*)(dsm + kLsOffR0);
  float* qs = (float*)(dsm + kLsOffQs);
  uint32_t* misc = (uint32_t*)(dsm + kLsOffMisc);
  uint32_t* allseg = (uint32_t*)(dsm + kLsOffAll);  // both halves of every tile
  uint32_t* allpre = allseg + 4;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int K = a.K, n = a.n_cols;
  const int NC = a.l_chunks, NP = a.l_np, G = a.l_period, T = a.l_tiles;
  const int L = 2 * NC * NP;
  const int blk = row >> 5, r = row & 31;
  const bool want_r0 = a.max_inout != nullptr;
  auto stamp = [&](int slot) {  // BB_SELECT_TRACE probe runs: phase timeline (100 MHz), 16 words per row
    if (a.trace && tid == 0) a.trace[row * 16 + slot] = __builtin_amdgcn_s_memrealtime();
  };
  stamp(0);

  if (tid < 16) misc[tid] = 0u;
  hist[tid] = 0u;  // kSelectThreads == 256 bins
  if (tid == 0) {
    allseg[0] = 0u;
    allseg[1] = (uint32_t)T << 1;
    allseg[2] = 0u;
    allseg[3] = ((uint32_t)T << 1) | 1u;
    allpre[0] = 0u;
    allpre[1] = (uint32_t)T * 16;
    allpre[2] = (uint32_t)T * 32;
  }
  const int nq4 = a.rr_d >> 2;
  const float hq = a.s_h[row];
  // (loaded with the lists: the first barrier waits for every outstanding load, so a load
  // issued after it would stall the bound search's first step instead)
  const float eps_row = a.rr_eps[row];
  // raw-query lists (GemmArgs.q_raw): wave 0 loads the raw row now and normalises it into
  // the LDS query after the classification (prep_kernel's arithmetic, qnorm.h: the same f32
  // row bit for bit), so its latency hides under the bound search
  float xq[kQnC];
  if (a.rr_q_raw) {
    if (wave == 0) {
      const float* qr = a.rr_q_raw + (size_t)row * a.rr_q_raw_ld;
#pragma unroll
      for (int c = 0; c < kQnC; ++c) {
        const int i = lane + 64 * c;
        xq[c] = i < a.rr_q_raw_d ? qr[i] : 0.f;
      }
    }
  } else if (tid < nq4) {
    ((float4*)qs)[tid] = ((const float4*)(a.rr_q + (size_t)row * a.rr_ld))[tid];
  }

  // ---- lists of this row: thread t holds lists t, t + 256, ... ----
  constexpr int kLPT = kLsMaxLists / kSelectThreads;
  uint4 v[kLPT];
  int vt0[kLPT];  // first tile of the list's period (absolute), or -1: no such period
#pragma unroll
  for (int i = 0; i < kLPT; ++i) {
    const int j = tid + i * kSelectThreads;
    v[i] = make_uint4(0u, 0u, 0u, 0u);
    vt0[i] = -1;
    if (j < L) {
      const int cp = j >> 1, hh = j & 1, c = cp / NP, p = cp - c * NP;
      const int tlo = chunk_tile_lo(c, T, NC), thi = chunk_tile_lo(c + 1, T, NC);
      if (p * G < thi - tlo) {
        v[i] = *(const uint4*)(a.lists + 4 * list_slot(c, p, NP, a.l_nb, blk, hh * 32 + r));
        vt0[i] = tlo + p * G;
      }
    }
  }
  constexpr int kRPT = 2;  // rank-0 (chunk, half) entries per thread: 2·NC <= 512
  uint2 rv[kRPT];
  uint32_t pm = 0;
#pragma unroll
  for (int i = 0; i < kRPT; ++i) {
    const int e = tid + i * kSelectThreads, c = e >> 1, hh = e & 1;
    rv[i] = make_uint2(0u, 0u);
    if (want_r0 && c < NC && chunk_tile_lo(c + 1, T, NC) > chunk_tile_lo(c, T, NC))
      rv[i] = *(const uint2*)(a.r0lists + 2 * list_slot(c, 0, 1, a.l_nb, blk, hh * 32 + r));
    pm = max(pm, rv[i].x >> 16);
  }
  __syncthreads();  // hist and misc cleared
  stamp(1);
  // Δ: the re-rank margin in codes (h = 0: a zero query row, every code equal -> take all)
  const uint32_t delta = hq > 0.f ? (uint32_t)fminf(ceilf(rr_margin(eps_row) / hq), 60000.f) + 2u : 0x10000u;

  // ---- bound: T0 = K-th largest code over every list key, by a bitwise search: each wave
  // counts its lanes' keys >= c with ballots, the four wave counts meet in LDS (two
  // alternating slots, one barrier per step); only the bits below the highest bit in which
  // the largest and smallest codes differ are searched ----
  const int nlw = (L - wave * 64 + kSelectThreads - 1) / kSelectThreads;  // lists of this wave's lanes (upper bound)
  auto wave_count_ge = [&](uint32_t c) -> uint32_t {
    uint32_t cnt = 0;
#pragma unroll
    for (int i = 0; i < kLPT; ++i) {
      if (i < nlw) {
        cnt += (uint32_t)__popcll(__ballot((v[i].x >> 16) >= c));
        cnt += (uint32_t)__popcll(__ballot((v[i].x & 0xFFFFu) >= c));
        cnt += (uint32_t)__popcll(__ballot((v[i].y >> 16) >= c));
        cnt += (uint32_t)__popcll(__ballot((v[i].y & 0xFFFFu) >= c));
        cnt += (uint32_t)__popcll(__ballot((v[i].z >> 16) >= c));
      }
    }
    return cnt;
  };
  uint32_t Tg = 1u;
  if (a.ablate & 4) {  // BB_LS_BITWISE (A/B runs): the round-3 bitwise search, one barrier per bit
  uint32_t* xch = hist;  // [2][4] count slots + [4] hi / [4] lo
  {
    uint32_t hi = 0, lo = 0xFFFFu;
#pragma unroll
    for (int i = 0; i < kLPT; ++i) {
      hi = max(hi, v[i].x >> 16);  // codes are sorted within a list: c0 is the largest
      const uint32_t c4 = v[i].z >> 16, c3 = v[i].y & 0xFFFFu, c2 = v[i].y >> 16, c1 = v[i].x & 0xFFFFu,
                     c0 = v[i].x >> 16;
      const uint32_t mn = c4 ? c4 : c3 ? c3 : c2 ? c2 : c1 ? c1 : c0;
      lo = mn ? min(lo, mn) : lo;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      hi = max(hi, (uint32_t)__shfl_xor((int)hi, o));
      lo = min(lo, (uint32_t)__shfl_xor((int)lo, o));
    }
    const uint32_t c1 = wave_count_ge(1u);
    if (lane == 0) {
      xch[8 + wave] = hi;
      xch[12 + wave] = lo;
      xch[wave] = c1;
    }
  }
  if (want_r0) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) pm = max(pm, (uint32_t)__shfl_xor((int)pm, o));
    if (lane == 0) atomicMax(&misc[M_PM], pm);
  }
  __syncthreads();
  const uint32_t hi = max(max(xch[8], xch[9]), max(xch[10], xch[11]));
  const uint32_t lo = min(min(xch[12], xch[13]), min(xch[14], xch[15]));
  if (xch[0] + xch[1] + xch[2] + xch[3] >= (uint32_t)K) {
    const uint32_t d = hi ^ lo;
    const int top = d ? 31 - __builtin_clz(d) : -1;
    uint32_t P = top < 0 ? hi : hi & ~((2u << top) - 1u);
    for (int bit = top, st = 1; bit >= 0; --bit, ++st) {
      const uint32_t c = P | (1u << bit);
      const uint32_t wc = wave_count_ge(c);
      uint32_t* slot = xch + 4 * (st & 1);
      if (lane == 0) slot[wave] = wc;
      __syncthreads();
      if (slot[0] + slot[1] + slot[2] + slot[3] >= (uint32_t)K) P = c;
    }
    Tg = P > delta ? P - delta : 1u;
  }
  } else {
    // Two-level histogram of the 16-bit codes (hist cleared at the start): the bin of the K-th
    // largest code's high byte, then its low byte among the codes of that bin — two passes of
    // LDS atomics and two block scans (find_bin), nine barriers in all, against one barrier
    // per bit of the bitwise search (15-16 at a row's usual code range)
    uint32_t* scan = (uint32_t*)(dsm + kLsOffScan);
    auto codes_of = [&](int i, uint32_t (&c)[5]) __attribute__((always_inline)) {
      c[0] = v[i].x >> 16;
      c[1] = v[i].x & 0xFFFFu;
      c[2] = v[i].y >> 16;
      c[3] = v[i].y & 0xFFFFu;
      c[4] = v[i].z >> 16;
    };
#pragma unroll
    for (int i = 0; i < kLPT; ++i) {
      if (i >= nlw) continue;  // wave-uniform
      uint32_t c[5];
      codes_of(i, c);
#pragma unroll
      for (int e = 0; e < 5; ++e)
        if (c[e]) atomicAdd(&hist[c[e] >> 8], 1u);
    }
    if (want_r0) {
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) pm = max(pm, (uint32_t)__shfl_xor((int)pm, o));
      if (lane == 0) atomicMax(&misc[M_PM], pm);
    }
    __syncthreads();
    uint32_t* fb = scan + 4;
    find_bin(hist, 256, (uint32_t)K, fb, scan);
    const uint32_t b1 = fb[0], above1 = fb[1];
    if (b1 != 0xFFFFFFFFu) {  // (uniform) at least K codes
      hist[tid] = 0u;
      __syncthreads();
#pragma unroll
      for (int i = 0; i < kLPT; ++i) {
        if (i >= nlw) continue;
        uint32_t c[5];
        codes_of(i, c);
#pragma unroll
        for (int e = 0; e < 5; ++e)
          if (c[e] && (c[e] >> 8) == b1) atomicAdd(&hist[c[e] & 0xFFu], 1u);
      }
      __syncthreads();
      find_bin(hist, 256, (uint32_t)K - above1, fb, scan);
      const uint32_t T0 = (b1 << 8) | fb[0];
      Tg = T0 > delta ? T0 - delta : 1u;
    }
  }
  stamp(2);

  // ---- classify: candidates of complete lists (one LDS atomic per wave and list slot),
  // overflowed lists as segments ----
  const uint64_t lt_mask = (1ull << lane) - 1ull;
#pragma unroll
  for (int i = 0; i < kLPT; ++i) {
    if (i >= nlw) continue;  // wave-uniform
    uint32_t cc[5], pp[5];
    list_unpack5(v[i], cc, pp);
    const bool live = vt0[i] >= 0 && cc[0] != 0u;
    const int j = tid + i * kSelectThreads, hh = j & 1;
    const int c = live ? (j >> 1) / NP : 0;
    const bool ovf = live && cc[4] >= Tg;  // all five within the margin: the period may hold more
    if (ovf) {
      const uint32_t sidx = atomicAdd(&misc[M_SEG], 1u);
      const int thi = chunk_tile_lo(c + 1, T, NC), nt = min(G, thi - vt0[i]);
      atomicAdd(&misc[M_SEGN], (uint32_t)nt * 16u);
      if (sidx < (uint32_t)kLsSeg) {
        seg[2 * sidx] = (uint32_t)vt0[i];
        seg[2 * sidx + 1] = ((uint32_t)nt << 1) | (uint32_t)hh;
      }
    }
    // codes are sorted: the keys at or above Tg form a prefix (at most 4 when not overflowed)
    const uint32_t m = live && !ovf ? (uint32_t)(cc[0] >= Tg) + (uint32_t)(cc[1] >= Tg) + (uint32_t)(cc[2] >= Tg) +
                                          (uint32_t)(cc[3] >= Tg)
                                    : 0u;
    const uint64_t b0 = __ballot(m & 1u), b1 = __ballot((m >> 1) & 1u), b2 = __ballot((m >> 2) & 1u);
    const uint32_t tot = (uint32_t)__popcll(b0) + 2u * (uint32_t)__popcll(b1) + 4u * (uint32_t)__popcll(b2);
    if (!tot) continue;
    uint32_t base = 0;
    if (lane == 0) base = atomicAdd(&misc[M_CAND], tot);
    base = (uint32_t)__shfl((int)base, 0);
    const uint32_t p0 = base + (uint32_t)__popcll(b0 & lt_mask) + 2u * (uint32_t)__popcll(b1 & lt_mask) +
                        4u * (uint32_t)__popcll(b2 & lt_mask);
    // position -> item: tile vt0 + (pos >> 4), register g = pos & 15 of lane half hh
    const uint32_t gb = a.gid0 + (uint32_t)(vt0[i] * 32 + 4 * hh);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const uint32_t g = pp[e] & 15u;
      const uint32_t item = (pp[e] >> 4) * 32u + (g & 3u) + 8u * (g >> 2);
      if ((uint32_t)e < m && p0 + e < (uint32_t)kLsCand) cand[p0 + e] = make_key(1u, gb + item);
    }
  }
  // rank 0: present half tiles within Δ of the largest present maximum
  if (want_r0) {
    const uint32_t Pm = misc[M_PM];  // settled by the barriers of the bound
    const uint32_t thr0 = Pm > delta ? Pm - delta : 1u;
#pragma unroll
    for (int i = 0; i < kRPT; ++i) {
      const int e = tid + i * kSelectThreads, c = e >> 1, hh = e & 1;
      if (!Pm || c >= NC || (rv[i].x >> 16) < thr0) continue;
      const int tlo = chunk_tile_lo(c, T, NC), thi = chunk_tile_lo(c + 1, T, NC);
      const bool whole = (rv[i].y >> 16) >= thr0;  // a 2nd half tile within Δ: the whole chunk half
      const uint32_t s = atomicAdd(&misc[M_R0SEG], 1u);
      const int nt = whole ? thi - tlo : 1;
      atomicAdd(&misc[M_R0N], (uint32_t)nt * 16u);
      if (s < (uint32_t)kLsR0Seg) {
        r0s[2 * s] = whole ? (uint32_t)tlo : (uint32_t)(tlo + (rv[i].x & 0xFFFFu));
        r0s[2 * s + 1] = ((uint32_t)nt << 1) | (uint32_t)hh;
      }
    }
  }
  if (a.rr_q_raw && wave == 0) {
    double xd[kQnC];
#pragma unroll
    for (int c = 0; c < kQnC; ++c) xd[c] = (double)xq[c];
    const double nrm = qn_norm(xd), rinv = 1.0 / nrm;
#pragma unroll
    for (int c = 0; c < kQnC; ++c) {
      const int i = lane + 64 * c;
      if (i < a.rr_d) qs[i] = qn_elem(xd[c], nrm, rinv);
    }
  }
  __syncthreads();
  const uint32_t ncand0 = misc[M_CAND], nseg = misc[M_SEG], nr0 = misc[M_R0SEG];
  const bool full_scan = nseg > (uint32_t)kLsSeg || nr0 > (uint32_t)kLsR0Seg ||
                         ncand0 + misc[M_SEGN] + misc[M_R0N] > (uint32_t)kLsCand;
  stamp(3);

  const int64_t w0 = a.slab_start >> 5;
  const uint32_t* excl = a.excl ? a.excl + (size_t)row * a.excl_ld : nullptr;
  auto present_bit = [&](int tile, int it) -> bool {
    return !a.present || ((a.present[w0 + tile] >> it) & 1u);
  };
  auto elig_bit = [&](int tile, int it) -> bool {
    const uint32_t w = (a.present ? a.present[w0 + tile] : ~0u) & (a.mask ? a.mask[w0 + tile] : ~0u) &
                       ~(excl ? excl[w0 + tile] : 0u);
    return (w >> it) & 1u;
  };

  if (!full_scan) {
    // ---- the one-pass path: [candidates | overflowed lists' eligible items | rank-0 items] ----
    if (nseg) ls_append(seg, (int)nseg, cand, misc, a.gid0, n, elig_bit);
    __syncthreads();
    const int Mc = (int)misc[M_CAND];
    if (nr0) ls_append(r0s, (int)nr0, cand, misc, a.gid0, n, present_bit);
    __syncthreads();
    const int M = (int)misc[M_CAND];
    stamp(4);
    ls_rescore(cand, M, a, qs);
    __syncthreads();
    stamp(5);
    uint64_t gmax = 0;
    if (want_r0) {
      uint64_t best = 0;
      for (int i = Mc + tid; i < M; i += kSelectThreads) best = cand[i] > best ? cand[i] : best;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        const uint64_t y = __shfl_xor(best, o);
        best = y > best ? y : best;
      }
      if (lane == 0) atomicMax((unsigned long long*)(misc + M_GMAX), (unsigned long long)best);
      __syncthreads();
      gmax = *(const uint64_t*)(misc + M_GMAX);
      if (tid == 0) a.max_inout[row] = gmax;
    }
    stamp(6);
    if (a.trace && tid == 0) {
      a.trace[row * 16 + 8] = ncand0 | ((uint64_t)nseg << 32);
      a.trace[row * 16 + 9] = (uint64_t)(Mc - (int)ncand0) | ((uint64_t)(M - Mc) << 32);
    }
    // ranks by counting: key i's position = #keys larger (keys are distinct: distinct ids);
    // every thread ranks its keys against the whole buffer with broadcast LDS reads, 8 keys
    // per step with the next 8 already in flight (LDS latency bounds this loop).  The
    // buffer is zero-padded to a multiple of 16 first (the rank-0 items there are consumed).
    const int Mc16 = (Mc + 15) & ~15;
    __syncthreads();
    if (tid < Mc16 - Mc) cand[Mc + tid] = 0ull;
    const int ne = (Mc + kSelectThreads - 1) / kSelectThreads;  // keys per thread (uniform)
    const ulonglong2* c2 = (const ulonglong2*)cand;
    const int cnt = min(Mc, K);
    // one instance per keys-per-thread count E: only its own E keys and ranks live
    auto rank_emit = [&](auto NE) __attribute__((always_inline)) {
      constexpr int E = decltype(NE)::value;
      uint64_t mk[E];
      uint32_t rk[E];
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const int i = tid + e * kSelectThreads;
        mk[e] = i < Mc ? cand[i] : 0ull;
        rk[e] = 0;
      }
      __syncthreads();
      ulonglong2 ya[4], yb[4];
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) ya[jj] = c2[jj];
      for (int k = 0; k < Mc16; k += 8) {
        const int kn = k + 8 < Mc16 ? k + 8 : k;  // (the last step re-reads, harmlessly)
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) yb[jj] = c2[(kn >> 1) + jj];
#pragma unroll
        for (int e = 0; e < E; ++e)
#pragma unroll
          for (int jj = 0; jj < 4; ++jj) rk[e] += (ya[jj].x > mk[e] ? 1u : 0u) + (ya[jj].y > mk[e] ? 1u : 0u);
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) ya[jj] = yb[jj];
      }
      if (a.out_scores) {
        // rank 0 dropped when it heads the list (the head is the unmasked arg-max iff that
        // item is eligible: gmax is then among the candidates)
        if (tid == 0) misc[M_BUF] = 0u;
        __syncthreads();
#pragma unroll
        for (int e = 0; e < E; ++e)
          if (tid + e * kSelectThreads < Mc && rk[e] == 0 && gmax && mk[e] == gmax) misc[M_BUF] = 1u;
        __syncthreads();
        const int start = (int)misc[M_BUF];
        const int c = min(a.k_final, cnt - start);
        float* sc = a.out_scores + (size_t)row * a.k_final;
        int64_t* id = a.out_ids + (size_t)row * a.k_final;
#pragma unroll
        for (int e = 0; e < E; ++e) {
          const int pos = (int)rk[e] - start;
          if (tid + e * kSelectThreads < Mc && pos >= 0 && pos < c) {
            sc[pos] = float_of_ord(ordk_of(mk[e]));
            id[pos] = out_id(a.idmap, gid_of(mk[e]));
          }
        }
        for (int i = c + tid; i < a.k_final; i += kSelectThreads) {
          sc[i] = 0.f;
          id[i] = -1;
        }
        if (a.out_counts && tid == 0) a.out_counts[row] = c;
      } else {
        uint64_t* out = a.keys_out + (size_t)row * K;
#pragma unroll
        for (int e = 0; e < E; ++e)
          if (tid + e * kSelectThreads < Mc && rk[e] < (uint32_t)K) out[rk[e]] = mk[e];
        for (int i = cnt + tid; i < K; i += kSelectThreads) out[i] = 0ull;
      }
    };
    if (ne <= 1) rank_emit(std::integral_constant<int, 1>{});
    else if (ne <= 2) rank_emit(std::integral_constant<int, 2>{});
    else if (ne <= 4) rank_emit(std::integral_constant<int, 4>{});
    else rank_emit(std::integral_constant<int, kLsCand / kSelectThreads>{});
    stamp(7);
    return;
  }

  // ---- fallback: exact rank 0 over every present item, exact running top-K over every
  // eligible item (masses of near-ties overflowing the buffer) ----
  uint64_t gmax = 0;
  if (want_r0) {
    uint64_t* rb = cand + kLsCand / 2;
    if (tid == 0) misc[M_BUF] = 0u;
    __syncthreads();
    uint64_t best = 0;
    auto r0_reduce = [&](int nb) {
      ls_rescore(rb, nb, a, qs);
      __syncthreads();
      for (int i = tid; i < nb; i += kSelectThreads) best = rb[i] > best ? rb[i] : best;
      __syncthreads();
      if (tid == 0) misc[M_BUF] = 0u;
      __syncthreads();
    };
    ls_stream(allseg, allpre, 2, rb, misc, a.gid0, n, 512, present_bit, r0_reduce);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const uint64_t y = __shfl_xor(best, o);
      best = y > best ? y : best;
    }
    if (lane == 0) atomicMax((unsigned long long*)(misc + M_GMAX), (unsigned long long)best);
    __syncthreads();
    gmax = *(const uint64_t*)(misc + M_GMAX);
    if (tid == 0) a.max_inout[row] = gmax;
    __syncthreads();
  }
  for (int i = tid; i < K; i += kSelectThreads) sel[i] = 0ull;
  if (tid == 0) misc[M_BUF] = 0u;
  __syncthreads();
  auto merge = [&](int nb) {
    ls_rescore(cand, nb, a, qs);
    __syncthreads();
    for (int i = tid; i < K; i += kSelectThreads) cand[nb + i] = sel[i];
    int P = 1;
    while (P < nb + K) P <<= 1;
    for (int i = nb + K + tid; i < P; i += kSelectThreads) cand[i] = 0ull;
    __syncthreads();
    bitonic_desc_u64(cand, P);
    for (int i = tid; i < K; i += kSelectThreads) sel[i] = cand[i];
    __syncthreads();
    if (tid == 0) misc[M_BUF] = 0u;
    __syncthreads();
  };
  ls_stream(allseg, allpre, 2, cand, misc, a.gid0, n, kLsFlush, elig_bit, merge);
  // ---- emit the running list (rank 0 dropped when it heads it) ----
  int cnt = 0;
  for (int i = 0; i < K; ++i) cnt += sel[i] != 0ull;  // uniform: every thread counts
  if (a.trace && tid == 0) a.trace[row * 16 + 10] = 1;
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

__global__ __launch_bounds__(kSelectThreads) __attribute__((amdgpu_waves_per_eu(4))) void select_list_kernel(SelectArgs a, int B) {
  select_list_body(a, xcd_row(blockIdx.x, B));
}
// both sides of a hybrid search: workgroups [0, B) side 0, the rest side 1.  Four workgroups
// per CU (128 VGPRs, 44 B/lane of spills outside the rescore loop): configs[2]'s 2·B = 2,048
// workgroups run in two full rounds instead of 2.67 — 50.4 -> 41.1 us per batch, 10.76 ->
// 11.45 M q/s (r03j).  Five per CU (96 VGPRs, 176 B/lane spilled) is slower (55 us).  The
// single-side kernel above runs at four per CU too: neutral at configs[1] (B = 256 is one
// round either way), select 36.4 -> 32.3 us at B = 1024 and 99.8 -> 94.6 us at 4096 (r03m).
__global__ __launch_bounds__(kSelectThreads) __attribute__((amdgpu_waves_per_eu(4))) void select_list_dual_kernel(SelectArgs a0, SelectArgs a1, int B) {
  if ((int)blockIdx.x < B)
    select_list_body(a0, xcd_row(blockIdx.x, B));
  else
    select_list_body(a1, xcd_row(blockIdx.x - B, B));
}
static bool list_args_ok(const SelectArgs& a) {
  const int L = 2 * a.l_chunks * a.l_np;
  return a.lists && a.s_h && a.rr_x && a.rr_d > 0 && a.rr_d <= kRrMaxD && !(a.rr_d & 3) &&
         a.rr_eps && (a.rr_q_raw ? a.rr_q_raw_d > 0 && a.rr_q_raw_d <= a.rr_d && a.rr_q_raw_ld >= a.rr_q_raw_d &&
                                       !a.max_inout
                                     : a.rr_q != nullptr) &&
         a.K > 0 && a.K <= kMaxKInt && a.n_cols > 0 && a.l_chunks > 0 && a.l_np > 0 && a.l_period > 0 &&
         L <= kLsMaxLists && 2 * a.l_chunks <= 2 * kSelectThreads && a.l_tiles * 32 >= a.n_cols &&
         (a.l_tiles + a.l_chunks - 1) / a.l_chunks <= 2047 && !(a.slab_start & 31) && !a.carry_in &&
         (!a.max_inout || a.r0lists) && (a.out_scores ? (a.out_ids && a.k_final > 0 && a.k_final <= kMaxKInt)
                                                      : a.keys_out != nullptr);
}

hipError_t launch_select_list(const SelectArgs& a0, const SelectArgs* a1, int B, hipStream_t s) {
  if (B <= 0 || !list_args_ok(a0) || (a1 && !list_args_ok(*a1))) return hipErrorInvalidValue;
  if (a1)
    bb_launch(select_list_dual_kernel, dim3(2 * B), dim3(kSelectThreads), 0, s, a0, *a1, B);
  else
    bb_launch(select_list_kernel, dim3(B), dim3(kSelectThreads), 0, s, a0, B);
  return hipGetLastError();
}

}  // namespace bb
