// compact.hip — constraint-first search: the allowed rows of a selective mask gathered into a
// compact shadow index, so the scans and the list select touch only them.
//
// The reference applies the hard constraints FIRST and scores inside the valid set:
// HybridRecommender.get_recommendations step 1 (recommendation_system.py:628-640) turns the
// constraints into valid_set_nums, then both sides walk only those sets (:648-656, the filter
// walks at :229 and :454).  With the mask's count known on the host (the length of
// valid_set_nums), bb_search does the same on the device: this kernel packs the allowed rows
// — position p = the p-th allowed item, ascending, so (score desc, position asc) is exactly
// (score desc, id asc) — and the per-query bits that refer to them, and the unchanged search
// pipeline runs over the packed rows.  Scores are computed from bit-identical operands, so the
// results are identical to the full scan's.
//
// One launch, four kinds of workgroup (all but the prep ones first build the popcount prefix of
// the mask words in LDS — ≤ 2,048 words, L2-resident — so no workgroup waits for another):
//   word workgroups      32 positions each: the id map and the present words of both item
//                        spaces
//   copy workgroups      one 16-B piece per thread of the packed rows (f32 + f16 content, f32 +
//                        f16 CF; zeros for the padding): every load independent, one memory
//                        round trip (64 positions per workgroup walked in turn took ~44 us at
//                        configs[2], r06c)
// Allowed item p sits in slot p·stride.  With stride 4 each lane half of a 32-row MFMA tile
// (items {0-3, 8-11, 16-19, 24-27} or the other four groups) holds at most four allowed
// items, so a per-lane top-5 list of one tile never overflows: when the top-K is a large
// share of the allowed rows (configs[2]: 101 of ~440), dense packing overflowed most lists
// and the list select rescored most rows (48 us, r06d).
//   exclusion workgroups four query rows each, one wave per row: the content exclusion of the
//                        liked set's rank-0 item (the arg-max of the UNMASKED ranking, :217 —
//                        known per item from the rank-0 table, so the packed search drops it as
//                        the full one does) and the query's CF exclusions (rated items,
//                        :441-451) re-indexed to slots
//   prep workgroups      four query rows of one side each (no mask prefix): prep_kernel's body
//                        (prep_body.h — the liked set's stored row gathered by id from the FULL
//                        index, the CF user row; the f16 operand in the scan's lane order, the
//                        f32 row and bound), so the packed search launches no prep
// Short, independent latency chains in one occupancy round: the content prep and the
// exclusions in one workgroup made the launch 11.5 -> 13.2 us (r06o).
#include "common.h"
#include "prep_body.h"

namespace bb {

constexpr int kCompactThreads = 256;
constexpr int kCompactPieces = 4;  // 16-B row pieces per copy thread

// p-th set bit of w (0-based; p < popcount(w))
__device__ __forceinline__ int select_bit(uint32_t w, int p) {
  for (int i = 0; i < p; ++i) w &= w - 1u;
  return __builtin_ctz(w);
}

// (four workgroups per CU: 128 VGPRs — every role in one round at configs[2])
__global__ __launch_bounds__(kCompactThreads) __attribute__((amdgpu_waves_per_eu(4))) void compact_kernel(CompactArgs a) {
  __shared__ uint32_t mw[kCompactMaxWords];
  __shared__ uint32_t pre[kCompactMaxWords + 1];
  __shared__ uint32_t rowbits[kCompactThreads / 64][kCompactMaxSlots / 32];  // exclusion rows: one per wave
  __shared__ uint32_t scan[kCompactThreads / 64];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int nw = a.nw;
  const int g = blockIdx.x;
  const int gq0 = a.n_word_wg + a.n_copy_wg;  // first exclusion workgroup
  // ---- prep workgroups (no mask prefix needed): four rows of one side each, one wave per row
  // — prep_kernel's body (prep_body.h), so the packed search launches no prep ----
  {
    const int g0 = gq0 + a.n_query_wg, nc = a.prep_c.Bpad / 4;
    if (g >= g0) {
      if (g < g0 + nc) prep_rows(a.prep_c, g - g0);
      else prep_rows(a.prep_f, g - g0 - nc);
      return;
    }
  }
  // ---- mask words (bits past n cleared) and their exclusive popcount prefix ----
  constexpr int kWpt = kCompactMaxWords / kCompactThreads;
  uint32_t cnt[kWpt];
  uint32_t mine = 0;
#pragma unroll
  for (int j = 0; j < kWpt; ++j) {
    const int w = tid * kWpt + j;
    uint32_t v = 0;
    if (w < nw) {
      v = a.mask[w];
      if ((int64_t)(w + 1) * 32 > a.n) v &= (1u << (a.n & 31)) - 1u;
      mw[w] = v;
    }
    cnt[j] = (uint32_t)__popc(v);
    mine += cnt[j];
  }
  // block exclusive scan of the per-thread sums
  uint32_t incl = mine;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = (uint32_t)__shfl_up((int)incl, o);
    if (lane >= o) incl += y;
  }
  if (lane == 63) scan[wave] = incl;
  __syncthreads();
  uint32_t base = incl - mine;
  for (int w = 0; w < wave; ++w) base += scan[w];
  const uint32_t total = scan[0] + scan[1] + scan[2] + scan[3];
#pragma unroll
  for (int j = 0; j < kWpt; ++j) {
    const int w = tid * kWpt + j;
    if (w < nw) pre[w] = base;
    base += cnt[j];
  }
  if (tid == 0) pre[nw] = total;
  __syncthreads();
  // more allowed items than the caller's count: the packed search would miss items, so it
  // finds none (every present bit 0 -> empty results) instead of a silently wrong list
  const uint32_t E = total <= (uint32_t)a.cap_pos ? total : 0u;
  const int S = a.stride;

  // the p-th allowed item (p < E): binary search over the prefix, then the bit inside the word
  auto item_of = [&](int p) -> int64_t {
    if ((uint32_t)p >= E) return -1;
    int lo = 0, hi = nw;  // pre[lo] <= p < pre[hi]
    while (hi - lo > 1) {
      const int mid = (lo + hi) >> 1;
      if (pre[mid] <= (uint32_t)p) lo = mid;
      else hi = mid;
    }
    return (int64_t)lo * 32 + select_bit(mw[lo], p - (int)pre[lo]);
  };

  if (g < a.n_word_wg) {
    // ---- slots [32g, 32g + 32): the id map and one present word per item space ----
    if (wave == 0) {
      const int sl = g * 32 + (lane & 31);
      const int64_t item = sl % S ? -1 : item_of(sl / S);
      if (lane < 32) a.idmap[sl] = item >= 0 ? (uint32_t)(item + a.id_offset) : 0xFFFFFFFFu;
      const bool pc = a.items && item >= 0 && ((a.items_present[item >> 5] >> (item & 31)) & 1u);
      const bool pf = a.cf && item >= 0 && ((a.cf_present[item >> 5] >> (item & 31)) & 1u);
      const uint64_t bc = __ballot(pc && lane < 32), bf = __ballot(pf && lane < 32);
      if (lane == 0 && a.items) a.c_present[g] = (uint32_t)bc;
      if (lane == 0 && a.cf) a.c_cf_present[g] = (uint32_t)bf;
    }
    return;
  }
  if (g < a.n_word_wg + a.n_copy_wg) {
    // ---- rows: kCompactPieces 16-B pieces per thread (all loads before any store) over
    // [allowed positions] x [the f32 content and CF pieces of a row] then [every slot] x [the
    // f16 pieces the scans read] (zeros for the padding slots; the f32 rows of padding slots are
    // never read: nothing there is present) ----
    const int per32 = a.ch_items + a.ch_cf, per16 = a.ch_items_b + a.ch_cf_b;
    const int64_t n32 = (int64_t)E * per32;
    const int64_t total_pieces = n32 + (int64_t)a.cap * per16;
    uint4 v[kCompactPieces];
    uint4* dst[kCompactPieces];
#pragma unroll
    for (int u = 0; u < kCompactPieces; ++u) {
      const int64_t i = ((int64_t)(g - a.n_word_wg) * kCompactPieces + u) * kCompactThreads + tid;
      v[u] = make_uint4(0u, 0u, 0u, 0u);
      dst[u] = nullptr;
      if (i >= total_pieces) continue;
      if (i < n32) {
        const int p = (int)(i / per32);
        int c = (int)(i - (int64_t)p * per32);
        const int64_t item = item_of(p), sl = (int64_t)p * S;
        if (c < a.ch_items) {
          v[u] = ((const uint4*)(a.items + item * a.ld))[c];
          dst[u] = (uint4*)(a.c_items + sl * a.ld) + c;
        } else {
          c -= a.ch_items;
          v[u] = ((const uint4*)(a.cf + item * a.ldc))[c];
          dst[u] = (uint4*)(a.c_cf + sl * a.ldc) + c;
        }
      } else {
        const int64_t j = i - n32;
        const int sl = (int)(j / per16);
        int c = (int)(j - (int64_t)sl * per16);
        const int64_t item = sl % S ? -1 : item_of(sl / S);
        const int64_t it = item >= 0 ? item : 0;
        if (c < a.ch_items_b) {
          if (item >= 0) v[u] = ((const uint4*)(a.items_bf + it * a.ld_b))[c];
          dst[u] = (uint4*)(a.c_items_bf + (int64_t)sl * a.ld_b) + c;
        } else {
          c -= a.ch_items_b;
          if (item >= 0) v[u] = ((const uint4*)(a.cf_bf + it * a.ldc_b))[c];
          dst[u] = (uint4*)(a.c_cf_bf + (int64_t)sl * a.ldc_b) + c;
        }
      }
    }
#pragma unroll
    for (int u = 0; u < kCompactPieces; ++u)
      if (dst[u]) *dst[u] = v[u];
    return;
  }

  if (g >= gq0 && !a.B) return;  // (no exclusion rows)
  // ---- exclusion rows [4q, 4q + 4), one wave each ----
  const int gq = g - gq0;
  const int b = gq * 4 + wave;
  if (b >= a.B) return;  // (per wave: no block barrier below)
  uint32_t* rb = rowbits[wave];
  // the exclusion row's words, all in flight at once and before the rank-0 lookups (a loop
  // loading one word per step waited a memory round trip per step: ~13 at configs[2])
  constexpr int kEx = kCompactMaxWords / 64;
  uint32_t exw[kEx];
  if (a.c_excl1) {
    const uint32_t* ex = a.excl + (int64_t)b * a.excl_ld;
#pragma unroll
    for (int j = 0; j < kEx; ++j) {
      const int w = lane + 64 * j;
      exw[j] = w < nw ? ex[w] : 0u;
    }
  }
  auto wave_sync = []() __attribute__((always_inline)) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  };
  if (a.c_excl0) {  // the liked set's rank-0 item (its unmasked arg-max), where it is allowed
    for (int w = lane; w < a.xnw; w += 64) rb[w] = 0u;
    wave_sync();
    if (lane == 0) {
      const int64_t lid = a.q_items[b] - (int64_t)a.id_offset;
      const bool ok = lid >= 0 && lid < a.n;  // (outside the index: a zero row, as prep's gather)
      const uint64_t key = a.r0key[ok ? lid : a.n];  // [n]: a zero row's rank 0
      const int64_t r = key ? (int64_t)gid_of(key) - (int64_t)a.id_offset : -1;
      if (r >= 0 && r < a.n && ((mw[r >> 5] >> (r & 31)) & 1u)) {
        const uint32_t p = pre[r >> 5] + (uint32_t)__popc(mw[r >> 5] & ((1u << (r & 31)) - 1u));
        if (p < E) rb[(p * S) >> 5] |= 1u << ((p * S) & 31);
      }
    }
    wave_sync();
    uint32_t* out = a.c_excl0 + (int64_t)b * a.xnw;
    for (int w = lane; w < a.xnw; w += 64) out[w] = rb[w];
    wave_sync();
  }
  if (a.c_excl1) {  // the query's exclusions (rated items), re-indexed to slots
    for (int w = lane; w < a.xnw; w += 64) rb[w] = 0u;
    wave_sync();
#pragma unroll
    for (int j = 0; j < kEx; ++j) {
      const int w = lane + 64 * j;
      if (w >= nw) continue;
      uint32_t hit = mw[w] & exw[j];
      while (hit) {
        const int bit = __builtin_ctz(hit);
        hit &= hit - 1u;
        const uint32_t p = pre[w] + (uint32_t)__popc(mw[w] & ((1u << bit) - 1u));
        if (p < E) atomicOr(&rb[(p * S) >> 5], 1u << ((p * S) & 31));
      }
    }
    wave_sync();
    uint32_t* out = a.c_excl1 + (int64_t)b * a.xnw;
    for (int w = lane; w < a.xnw; w += 64) out[w] = rb[w];
  }
}

hipError_t launch_compact(const CompactArgs& a, hipStream_t s) {
  const int per = a.ch_items + a.ch_items_b + a.ch_cf + a.ch_cf_b;
  if (a.nw <= 0 || a.nw > kCompactMaxWords || a.cap <= 0 || a.cap % 32 || a.cnw * 32 != a.cap ||
      a.cap > kCompactMaxSlots || a.xnw <= 0 || a.xnw > a.cnw || a.n_word_wg != a.cnw || a.B < 0 || per <= 0 ||
      a.stride < 1 || a.cap_pos * a.stride != a.cap ||
      (int64_t)a.n_copy_wg * kCompactThreads * kCompactPieces <
          (int64_t)a.cap_pos * (a.ch_items + a.ch_cf) + (int64_t)a.cap * (a.ch_items_b + a.ch_cf_b) ||
      (a.items && (!a.items_bf || !a.c_items || !a.c_items_bf || !a.c_present || a.ld % 4 || a.ld_b % 8 ||
                   a.ch_items != a.ld / 4 || a.ch_items_b != a.ld_b / 8)) ||
      (!a.items && (a.ch_items || a.ch_items_b)) ||
      (a.cf && (!a.cf_bf || !a.c_cf || !a.c_cf_bf || !a.c_cf_present || a.ldc % 4 || a.ldc_b % 8 ||
                a.ch_cf != a.ldc / 4 || a.ch_cf_b != a.ldc_b / 8)) ||
      (!a.cf && (a.ch_cf || a.ch_cf_b)) ||
      (a.c_excl0 && (!a.q_items || !a.r0key)) || (a.c_excl1 && (!a.excl || a.excl_ld < a.nw)) ||
      a.n_query_wg * 4 < a.B || (a.B && !a.c_excl0 && !a.c_excl1) ||
      a.prep_c.Bpad % 4 || a.prep_f.Bpad % 4)
    return hipErrorInvalidValue;
  bb_launch(compact_kernel, dim3(a.n_word_wg + a.n_copy_wg + a.n_query_wg + (a.prep_c.Bpad + a.prep_f.Bpad) / 4),
            dim3(kCompactThreads), 0, s, a);
  return hipGetLastError();
}

}  // namespace bb
