// select_list.hip — exact per-query top-K from the bounded candidate lists of a kScanList scan.
//
// Replaces the score-image select + rerank pair of the exact re-rank path (one slab, f32
// index) — np.argsort(sim)[::-1] + the filter walk of get_similar_sets
// (recommendation_system.py:214-247), the CF loop + sort (:438-461) and pgvector's
// ORDER BY <=> LIMIT k — for the 25K-row configs.  One workgroup (4 waves) per query row:
//
//   lists   every lane's top-4 keys per period (list_epi.h): key = (u16 code, chunk position)
//   bound   T0 = the K-th largest list head: K distinct items have codes >= T0, so the exact
//           K-th score is >= dec(T0) − ε', and every exact top-K member has code >= Tg =
//           T0 − Δ (Δ = the re-rank margin 2ε'(1+2^-10)+2^-20 in codes, + 2 codes of slack)
//   gather  keys >= Tg of the lists whose 4th key is below Tg (they dropped nothing that
//           matters); lists whose 4th key reaches Tg may have dropped candidates, so all
//           eligible items of their period are enumerated instead ("segments")
//   rank 0  (similar / hybrid content side) the present half tiles whose maximum is within
//           Δ of the largest; a lane whose 2nd-best half tile is also within Δ contributes its
//           whole chunk half.  Their present items are rescored exactly; the exact maximum is
//           the unmasked arg-max key that the similar-sets path drops (:217)
//   rescore every candidate from the f32 rows (f64 sums in rescore_rows' fixed order, rounded
//           to f32: the same bits as every other path), sort by (score desc, id asc), emit
// Common case (no segments, <= 512 candidates): one rescore round + a register sort by one
// wave.  Otherwise an exact running top-K: candidates and enumerated items are rescored in
// batches and merged by a bitonic sort in LDS (masses of near-duplicates, all-equal scores).
#include "common.h"
#include "list_epi.h"
#include "select_util.h"

namespace bb {

constexpr int kLsCand = 2048;   // candidate / batch buffer (u64 keys)
constexpr int kLsFlush = 1024;  // batch size that triggers a merge of the running top-K
constexpr int kLsSeg = 512;     // content segments (overflowing lists)
constexpr int kLsR0Seg = 64;    // rank-0 segments
constexpr int kLsMaxLists = 1024;
constexpr int kLsOffCand = 0;
constexpr int kLsOffSel = kLsOffCand + kLsCand * 8;          // u64 [kMaxKInt] running top-K
constexpr int kLsOffHd = kLsOffSel + kMaxKInt * 8;           // u32 [kLsMaxLists] head codes
constexpr int kLsOffSeg = kLsOffHd + kLsMaxLists * 4;        // u32 [kLsSeg][2] (t0, nt << 1 | h)
constexpr int kLsOffPre = kLsOffSeg + kLsSeg * 8;            // u32 [kLsSeg + 1] item prefix
constexpr int kLsOffR0 = kLsOffPre + (kLsSeg + 1) * 4 + 12;  // u32 [kLsR0Seg][2]
constexpr int kLsOffQs = kLsOffR0 + kLsR0Seg * 8;            // f32 [kRrMaxD]
constexpr int kLsOffMisc = kLsOffQs + kRrMaxD * 4;           // u32 [16]
constexpr int kLsOffAll = kLsOffMisc + 64;                   // u32 [4] + [3]: every item of the row
constexpr int kLsLds = kLsOffAll + 32;
static_assert(kLsOffQs % 16 == 0, "query row must be 16-B aligned");
// misc words; M_GMAX is a u64 (8-byte aligned: misc starts 8-aligned)
enum { M_CAND = 0, M_SEG, M_R0SEG, M_BUF, M_PM, M_GMAX = 8 };
static_assert(kLsOffMisc % 8 == 0, "u64 misc word must be 8-byte aligned");

// Exhaustive enumeration of segments (tile ranges of one lane half) in rounds of 256 items:
// item i of the concatenation -> (segment, tile, register) by binary search over the item
// prefix; items passing `keep` are appended to buf as placeholder keys; a batch reaching
// `flush` items is reduced (merge or max); at most flush - 1 + 256 items are buffered.  Every thread returns holding the same buffer count.
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

__device__ __forceinline__ void select_list_body(const SelectArgs& a, int row) {
  __shared__ __attribute__((aligned(16))) char dsm[kLsLds];
  uint64_t* cand = (uint64_t*)(dsm + kLsOffCand);
  uint64_t* sel = (uint64_t*)(dsm + kLsOffSel);
  uint32_t* hd = (uint32_t*)(dsm + kLsOffHd);
  uint32_t* seg = (uint32_t*)(dsm + kLsOffSeg);
  uint32_t* pre = (uint32_t*)(dsm + kLsOffPre);
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

  if (tid < 16) misc[tid] = 0u;
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
  if (tid < nq4) ((float4*)qs)[tid] = ((const float4*)(a.rr_q + (size_t)row * a.rr_ld))[tid];

  // Δ: the re-rank margin in codes (h = 0: a zero query row, every code equal -> take all)
  const float hq = a.s_h[row];
  const uint32_t delta = hq > 0.f ? (uint32_t)fminf(ceilf(rr_margin(a.rr_eps[row]) / hq), 60000.f) + 2u : 0x10000u;

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
#pragma unroll
  for (int i = 0; i < kLPT; ++i) {
    const int j = tid + i * kSelectThreads;
    if (j < kLsMaxLists) hd[j] = v[i].x >> 16;
  }
  __syncthreads();

  // ---- bound: T0 = K-th largest head code (every wave on its own, ballot counts) ----
  uint32_t Tg = 1u;
  {
    uint32_t hv[kLsMaxLists / 64];
#pragma unroll
    for (int i = 0; i < kLsMaxLists / 64; ++i) hv[i] = lane + 64 * i < L ? hd[lane + 64 * i] : 0u;
    auto cnt_ge = [&](uint32_t c) -> uint32_t {
      uint32_t s = 0;
#pragma unroll
      for (int i = 0; i < kLsMaxLists / 64; ++i) s += (uint32_t)__popcll(__ballot(hv[i] >= c));
      return s;
    };
    if (cnt_ge(1u) >= (uint32_t)K) {
      uint32_t hi = 0, lo = 0xFFFFu;
#pragma unroll
      for (int i = 0; i < kLsMaxLists / 64; ++i) {
        hi = max(hi, hv[i]);
        lo = min(lo, hv[i] ? hv[i] : 0xFFFFu);
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
      uint32_t P = top < 0 ? hi : hi & ~((2u << top) - 1u);
      for (int b = top; b >= 0; --b) {
        const uint32_t c = P | (1u << b);
        if (cnt_ge(c) >= (uint32_t)K) P = c;
      }
      Tg = P > delta ? P - delta : 1u;
    }
  }

  // ---- classify: candidates of complete lists, segments for the overflowing ones ----
#pragma unroll
  for (int i = 0; i < kLPT; ++i) {
    if (vt0[i] < 0 || v[i].x == 0u) continue;
    const int j = tid + i * kSelectThreads, hh = j & 1;
    const int c = (j >> 1) / NP, tlo = chunk_tile_lo(c, T, NC);
    if ((v[i].w >> 16) >= Tg) {  // all four within the margin: the period may hold more
      const uint32_t s = atomicAdd(&misc[M_SEG], 1u);
      const int thi = chunk_tile_lo(c + 1, T, NC), nt = min(G, thi - vt0[i]);
      if (s < (uint32_t)kLsSeg) {
        seg[2 * s] = (uint32_t)vt0[i];
        seg[2 * s + 1] = ((uint32_t)nt << 1) | (uint32_t)hh;
      }
      continue;
    }
    // keys are sorted: the ones at or above Tg form a prefix
    const uint32_t m = (uint32_t)((v[i].x >> 16) >= Tg) + (uint32_t)((v[i].y >> 16) >= Tg) +
                       (uint32_t)((v[i].z >> 16) >= Tg);
    if (!m) continue;
    const uint32_t p0 = atomicAdd(&misc[M_CAND], m);
    const uint32_t gb = a.gid0 + (uint32_t)(tlo * 32);
    if (p0 < (uint32_t)kLsCand) cand[p0] = make_key(1u, gb + (v[i].x & 0xFFFFu));
    if (m > 1 && p0 + 1 < (uint32_t)kLsCand) cand[p0 + 1] = make_key(1u, gb + (v[i].y & 0xFFFFu));
    if (m > 2 && p0 + 2 < (uint32_t)kLsCand) cand[p0 + 2] = make_key(1u, gb + (v[i].z & 0xFFFFu));
  }

  // ---- rank 0: present half tiles within Δ of the largest present maximum ----
  constexpr int kRPT = 2;  // (chunk, half) entries per thread: 2·NC <= 512
  uint2 rv[kRPT];
  if (want_r0) {
    uint32_t pm = 0;
#pragma unroll
    for (int i = 0; i < kRPT; ++i) {
      const int e = tid + i * kSelectThreads, c = e >> 1, hh = e & 1;
      rv[i] = make_uint2(0u, 0u);
      if (c < NC && chunk_tile_lo(c + 1, T, NC) > chunk_tile_lo(c, T, NC))
        rv[i] = *(const uint2*)(a.r0lists + 2 * list_slot(c, 0, 1, a.l_nb, blk, hh * 32 + r));
      pm = max(pm, rv[i].x >> 16);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) pm = max(pm, (uint32_t)__shfl_xor((int)pm, o));
    if (lane == 0) atomicMax(&misc[M_PM], pm);
  }
  __syncthreads();
  const uint32_t ncand0 = misc[M_CAND], nseg = misc[M_SEG];
  // (the rank-0 phase buffers in the upper half of cand: more candidates -> enumerate all)
  const bool full_scan = ncand0 > (uint32_t)(kLsCand / 2) || nseg > (uint32_t)kLsSeg;
  if (want_r0) {
    const uint32_t Pm = misc[M_PM];
    const uint32_t thr0 = Pm > delta ? Pm - delta : 1u;
    if (Pm) {
#pragma unroll
      for (int i = 0; i < kRPT; ++i) {
        const int e = tid + i * kSelectThreads, c = e >> 1, hh = e & 1;
        if (c >= NC || (rv[i].x >> 16) < thr0) continue;
        const int tlo = chunk_tile_lo(c, T, NC), thi = chunk_tile_lo(c + 1, T, NC);
        const bool whole = (rv[i].y >> 16) >= thr0;  // a 2nd half tile within Δ: the whole chunk half
        const uint32_t s = atomicAdd(&misc[M_R0SEG], 1u);
        if (s < (uint32_t)kLsR0Seg) {
          r0s[2 * s] = whole ? (uint32_t)tlo : (uint32_t)(tlo + (rv[i].x & 0xFFFFu));
          r0s[2 * s + 1] = ((uint32_t)(whole ? thi - tlo : 1) << 1) | (uint32_t)hh;
        }
      }
    }
  }
  __syncthreads();
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

  // ---- exact rank 0 (into misc[M_GMAX*]) ----
  uint64_t gmax = 0;
  if (want_r0) {
    const uint32_t nr0 = misc[M_R0SEG];
    const bool r0_all = nr0 > (uint32_t)kLsR0Seg;  // masses at the top: every present item
    if (!r0_all && tid == 0) {
      uint32_t acc = 0;
      for (uint32_t s = 0; s < nr0; ++s) {
        pre[s] = acc;
        acc += (r0s[2 * s + 1] >> 1) * 16;
      }
      pre[nr0] = acc;
    }
    __syncthreads();
    const int nsg = r0_all ? 2 : (int)nr0;
    // the rank-0 items go to the upper half of the candidate buffer (the lower half holds
    // the content candidates of the complete lists)
    uint64_t* rb = cand + kLsCand / 2;
    if (tid == 0) misc[M_BUF] = 0u;
    __syncthreads();
    uint64_t best = 0;
    auto r0_reduce = [&](int nb) {
      rr_rescore_any(rb, nb, a, qs);
      __syncthreads();
      for (int i = tid; i < nb; i += kSelectThreads) best = rb[i] > best ? rb[i] : best;
      __syncthreads();
      if (tid == 0) misc[M_BUF] = 0u;
      __syncthreads();
    };
    // flush at 512: at most 767 < kLsCand / 2 items are buffered at once
    ls_stream(r0_all ? allseg : r0s, r0_all ? allpre : pre, nsg, rb, misc, a.gid0, n, 512, present_bit, r0_reduce);
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

  // ---- common case: every list complete, few candidates: one rescore, one register sort ----
  if (!full_scan && nseg == 0 && ncand0 <= 512u) {
    rr_rescore_any(cand, (int)ncand0, a, qs);
    __syncthreads();
    if (wave != 0) return;
    if (ncand0 <= 64) wave_sort_emit<1>(cand, (int)ncand0, a, row, gmax);
    else if (ncand0 <= 128) wave_sort_emit<2>(cand, (int)ncand0, a, row, gmax);
    else if (ncand0 <= 256) wave_sort_emit<4>(cand, (int)ncand0, a, row, gmax);
    else wave_sort_emit<8>(cand, (int)ncand0, a, row, gmax);
    return;
  }

  // ---- exact running top-K over the candidates and the enumerated segments ----
  for (int i = tid; i < K; i += kSelectThreads) sel[i] = 0ull;
  __syncthreads();
  auto merge = [&](int nb) {
    rr_rescore_any(cand, nb, a, qs);
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
  if (tid == 0) misc[M_BUF] = 0u;
  __syncthreads();
  if (full_scan) {  // too many candidates or segments: enumerate every eligible item of the row
    ls_stream(allseg, allpre, 2, cand, misc, a.gid0, n, kLsFlush, elig_bit, merge);
  } else {
    if (ncand0) merge((int)ncand0);  // the complete lists' candidates (<= kLsCand / 2) first
    if (nseg) {
      if (tid == 0) {
        uint32_t acc = 0;
        for (uint32_t s = 0; s < nseg; ++s) {
          pre[s] = acc;
          acc += (seg[2 * s + 1] >> 1) * 16;
        }
        pre[nseg] = acc;
        misc[M_BUF] = 0u;
      }
      __syncthreads();
      ls_stream(seg, pre, (int)nseg, cand, misc, a.gid0, n, kLsFlush, elig_bit, merge);
    }
  }
  // ---- emit the running list (rank 0 dropped when it heads it) ----
  int cnt = 0;
  for (int i = 0; i < K; ++i) cnt += sel[i] != 0ull;  // uniform: every thread counts
  if (a.out_scores) {
    const int start = (gmax && cnt && sel[0] == gmax) ? 1 : 0;
    const int c = min(a.k_final, cnt - start);
    float* sc = a.out_scores + (size_t)row * a.k_final;
    int64_t* id = a.out_ids + (size_t)row * a.k_final;
    for (int i = tid; i < a.k_final; i += kSelectThreads) {
      sc[i] = i < c ? float_of_ord(ordk_of(sel[start + i])) : 0.f;
      id[i] = i < c ? (int64_t)gid_of(sel[start + i]) : (int64_t)-1;
    }
    if (a.out_counts && tid == 0) a.out_counts[row] = c;
    return;
  }
  uint64_t* out = a.keys_out + (size_t)row * K;
  for (int i = tid; i < K; i += kSelectThreads) out[i] = sel[i];
}

__global__ __launch_bounds__(kSelectThreads) void select_list_kernel(SelectArgs a, int B) {
  select_list_body(a, xcd_row(blockIdx.x, B));
}
// both sides of a hybrid search: workgroups [0, B) side 0, the rest side 1
__global__ __launch_bounds__(kSelectThreads) void select_list_dual_kernel(SelectArgs a0, SelectArgs a1, int B) {
  if ((int)blockIdx.x < B)
    select_list_body(a0, xcd_row(blockIdx.x, B));
  else
    select_list_body(a1, xcd_row(blockIdx.x - B, B));
}

static bool list_args_ok(const SelectArgs& a) {
  const int L = 2 * a.l_chunks * a.l_np;
  return a.lists && a.rr_eps && a.s_h && a.rr_x && a.rr_q && a.rr_d > 0 && a.rr_d <= kRrMaxD && !(a.rr_d & 3) &&
         a.K > 0 && a.K <= kMaxKInt && a.n_cols > 0 && a.l_chunks > 0 && a.l_np > 0 && a.l_period > 0 &&
         L <= kLsMaxLists && 2 * a.l_chunks <= 2 * kSelectThreads && a.l_tiles * 32 >= a.n_cols &&
         (a.l_tiles + a.l_chunks - 1) / a.l_chunks <= 2047 && !(a.slab_start & 31) && !a.carry_in &&
         (!a.max_inout || a.r0lists) && (a.out_scores ? (a.out_ids && a.k_final > 0 && a.k_final <= kMaxKInt)
                                                      : a.keys_out != nullptr);
}

hipError_t launch_select_list(const SelectArgs& a0, const SelectArgs* a1, int B, hipStream_t s) {
  if (B <= 0 || !list_args_ok(a0) || (a1 && !list_args_ok(*a1))) return hipErrorInvalidValue;
  if (a1)
    hipLaunchKernelGGL(select_list_dual_kernel, dim3(2 * B), dim3(kSelectThreads), 0, s, a0, *a1, B);
  else
    hipLaunchKernelGGL(select_list_kernel, dim3(B), dim3(kSelectThreads), 0, s, a0, B);
  return hipGetLastError();
}

}  // namespace bb
