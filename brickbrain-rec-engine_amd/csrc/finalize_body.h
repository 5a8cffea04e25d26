// finalize_body.h — the single-shard finalize of one query row (finalize1): rank-0 drop,
// truncation and the hybrid union blend of _combine_recommendations
// (recommendation_system.py:789-843) over two sorted, unique side lists, templated on the
// list capacity; finalize1_kernel runs it on lists read from global memory.  (A hybrid list
// select running both sides and this blend in one workgroup per row measured slower than
// two side workgroups + finalize1: 100.7 vs 50.3 + 19.4 us at configs[2])
#pragma once
#include "common.h"

namespace bb {

constexpr int kFinThreads = 256;

// h = wc·c + wcf·cf exactly as the reference's Python evaluates it (:812-818): two rounded
// products, one rounded sum.  Without the pragma the compiler contracts it to fma(wc, c, wcf·cf),
// which can differ in the last bit of h and so reorder near-tied blends (v_fma_f64 in the r05
// finalize kernels).
__device__ __forceinline__ double blend_h(double wc, double c, double wf, double f) {
#pragma clang fp contract(off)
  return wc * c + wf * f;
}

// Order image of a blended h.  -0.0 is folded into +0.0 first (the Python sort compares them
// equal; a -0.0 blend needs negative weights and two zero scores)
__device__ __forceinline__ uint64_t ord64_of(double d) {
  const uint64_t u = __builtin_bit_cast(uint64_t, d + 0.0);
  return (u & 0x8000000000000000ull) ? ~u : (u | 0x8000000000000000ull);
}

// Single-shard fast path (P == 1: each side's key list is already sorted and unique): no
// serial list walk and no sort network.  Each side's list is sliced in parallel (rank-0
// drop = skip the head when it is the unmasked arg-max maxk), the union blend looks each id
// up in the other list, and every blended entry finds its output position as its rank
// under (h desc, id asc) — O(n²) independent comparisons, n <= 2·k_side, no barriers inside.
// k0 / k1: the side lists (a.K_int keys each, generic pointers: global or LDS).
template <int KC, int NT = kFinThreads>
__device__ __forceinline__ void finalize1_body(const FinalizeArgs& a, int q, const uint64_t* k0, const uint64_t* k1,
                                               uint64_t maxk) {
  __shared__ uint64_t lst[2][KC];
  __shared__ double eh[2 * KC];
  __shared__ uint64_t ek[2 * KC];  // order image of eh (the legacy kernel's sort key)
  __shared__ uint32_t eg[2 * KC];
  __shared__ __attribute__((aligned(16))) uint32_t ehi[2 * KC];  // order image of (float)eh
  __shared__ int nnz[2], n_ent;
  constexpr int kSamp = 64;  // pruning sample (hybrid ranking, below)
  __shared__ uint32_t samp[kSamp];
  __shared__ int n_samp_cf, n_surv;
  __shared__ uint32_t prune_t;
  __shared__ int claim[2 * KC];         // survivors per strictly-greater count (ties, below)
  __shared__ uint16_t rk[2 * KC];       // each survivor's strictly-greater count
  const int tid = threadIdx.x;
  auto stamp = [&](int slot) {  // probe-only phase timeline (s_memrealtime, 100 MHz)
    if (a.trace && tid == 0) a.trace[q * 8 + slot] = __builtin_amdgcn_s_memrealtime();
  };
  stamp(0);
  // both side lists into registers first: a barrier waits for every outstanding load, so
  // loads issued after the setup barrier would add a second memory round trip (r04r trace:
  // 5.9 us until the lists were in LDS)
  constexpr int KR = (KC + NT - 1) / NT;
  uint64_t kv[2][KR];
#pragma unroll
  for (int side = 0; side < 2; ++side)
#pragma unroll
    for (int j = 0; j < KR; ++j) {
      const int i = tid + j * NT;
      kv[side][j] = side < a.sides && i < a.K_int ? (side ? k1 : k0)[i] : 0ull;
    }
  if (tid < 2) nnz[tid] = 0;
  if (tid == 0) {
    n_ent = 0;
    n_samp_cf = 0;
  }
  __syncthreads();
  int cnt_local[2] = {0, 0};
#pragma unroll
  for (int side = 0; side < 2; ++side)
#pragma unroll
    for (int j = 0; j < KR; ++j) {
      const int i = tid + j * NT;
      if (side < a.sides && i < a.K_int) {
        lst[side][i] = kv[side][j];
        cnt_local[side] += kv[side][j] != 0ull;
      }
    }
  // (side loops unrolled with constant indices: a loop bounded by a.sides indexed these
  // arrays dynamically and put them in scratch — a memory round trip per access)
#pragma unroll
  for (int side = 0; side < 2; ++side)
    if (side < a.sides && cnt_local[side]) atomicAdd(&nnz[side], cnt_local[side]);
  __syncthreads();
  stamp(1);
  int start[2] = {0, 0}, c[2] = {0, 0};
#pragma unroll
  for (int side = 0; side < 2; ++side) {
    if (side >= a.sides) continue;
    const uint64_t head = lst[side][0];
    if (side == 0 && a.drop_rank0 && maxk && head && head == maxk) start[side] = 1;
    const int target = a.hybrid ? a.k_side : a.k;
    const int avail = nnz[side] - start[side];
    c[side] = avail < target ? (avail > 0 ? avail : 0) : target;
  }
  float* sc = a.scores + (size_t)q * a.k;
  int64_t* id = a.ids + (size_t)q * a.k;
  if (!a.hybrid || c[0] == 0 || c[1] == 0) {
    const bool s1 = a.hybrid && c[0] == 0;
    const int cs = s1 ? c[1] : c[0];
    const uint64_t* L = s1 ? lst[1] + start[1] : lst[0] + start[0];
    const int n = cs < a.k ? cs : a.k;
    for (int i = tid; i < a.k; i += NT) {
      if (i < n) {
        const uint64_t key = L[i];
        sc[i] = float_of_ord(ordk_of(key));
        id[i] = out_id(a.idmap, gid_of(key));
      } else {
        sc[i] = 0.f;
        id[i] = -1;
      }
    }
    if (a.counts && tid == 0) a.counts[q] = n;
    return;
  }
  // union blend (recommendation_system.py:789-843): content entries, then CF-only entries.
  // CF ids go into an LDS hash table (open addressing, 2·KC slots: load <= 1/2); each
  // content entry looks its id up there and marks the CF entry it consumed.
  const uint64_t* L0 = lst[0] + start[0];
  const uint64_t* L1 = lst[1] + start[1];
  constexpr int kTab = 2 * KC;
  __shared__ __attribute__((aligned(16))) uint32_t tab_g[kTab];  // gid + 1 (0 = empty); later the survivors' images
  __shared__ uint16_t tab_j[kTab];
  __shared__ uint8_t used[KC];
  for (int i = tid; i < kTab; i += NT) tab_g[i] = 0u;
  for (int j = tid; j < c[1]; j += NT) used[j] = 0;
  __syncthreads();
  stamp(2);
  auto slot0 = [](uint32_t g) { return (int)((g * 2654435761u) >> 22) & (kTab - 1); };
  for (int j = tid; j < c[1]; j += NT) {
    const uint32_t g = gid_of(L1[j]);
    for (int sl = slot0(g);; sl = (sl + 1) & (kTab - 1))
      if (atomicCAS(&tab_g[sl], 0u, g + 1u) == 0u) {
        tab_j[sl] = (uint16_t)j;
        break;
      }
  }
  __syncthreads();
  for (int i = tid; i < c[0]; i += NT) {
    const uint32_t g = gid_of(L0[i]);
    int hit = -1;
    for (int sl = slot0(g);; sl = (sl + 1) & (kTab - 1)) {
      const uint32_t t = tab_g[sl];
      if (t == 0u) break;
      if (t == g + 1u) {
        hit = tab_j[sl];
        break;
      }
    }
    if (hit >= 0) used[hit] = 1;
    const double cs = (double)float_of_ord(ordk_of(L0[i]));
    const double fs = hit >= 0 ? (double)float_of_ord(ordk_of(L1[hit])) : 0.0;
    eh[i] = blend_h(a.w_content, cs, a.w_cf, fs);
    ek[i] = ord64_of(eh[i]);
    ehi[i] = ord_of((float)eh[i] + 0.0f);
    eg[i] = g;
  }
  __syncthreads();
  stamp(3);
  // sample S for the pruning bound below: the first content entries (L0 order: the best
  // content scores, blended), topped up with the best CF-only entries (L1 order) when the
  // content list is short — at most kSamp together.  (The two side lists of a selective
  // mask overlap heavily, so few CF-only entries come from the head of L1.)
  const int c0s = c[0] < kSamp ? c[0] : kSamp;
  for (int i = tid; i < c0s; i += NT) samp[i] = ehi[i];
  for (int j = tid; j < c[1]; j += NT) {
    const uint32_t g = gid_of(L1[j]);
    if (!used[j]) {
      const int pos = c[0] + atomicAdd(&n_ent, 1);
      eh[pos] = blend_h(a.w_content, 0.0, a.w_cf, (double)float_of_ord(ordk_of(L1[j])));
      ek[pos] = ord64_of(eh[pos]);
      ehi[pos] = ord_of((float)eh[pos] + 0.0f);
      eg[pos] = g;
      if (j < kSamp - c0s) samp[c0s + atomicAdd(&n_samp_cf, 1)] = ehi[pos];
    }
  }
  __syncthreads();
  stamp(4);
  const int ne = c[0] + n_ent;
  const int n = ne < a.k ? ne : a.k;
  // Pruning bound (exact): T = the k-th largest f32 image in the sample S.  At least k
  // entries reach T, so an entry below it ranks >= k and is dropped; an entry at or above
  // T has every entry that outranks it at or above T too, so its rank among the survivors
  // is its rank among all entries.  The O(n²) rank count then runs over the survivors
  // only (configs[2]: ~200 entries, the count was 9 of the kernel's 16.7 us).
  const int ns = c0s + n_samp_cf;
  if (tid < 64) {
    uint32_t t = 0u;  // fewer than k samples: no bound
    if (ns >= a.k && tid < ns) {
      const uint32_t v = samp[tid];
      int gt = 0, ge = 0;
      for (int f = 0; f < ns; ++f) {
        const uint32_t u = samp[f];
        gt += u > v;
        ge += u >= v;
      }
      t = (gt < a.k && ge >= a.k) ? v : 0u;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) t = max(t, (uint32_t)__shfl_xor((int)t, o));
    if (tid == 0) {
      prune_t = t;
      n_surv = 0;
    }
  }
  __syncthreads();
  // survivors, compacted: their images (reusing the hash table's words) and entry indices
  uint32_t* sv_h = tab_g;
  uint16_t* sv_e = tab_j;
  const uint32_t T = prune_t;
  for (int i = tid; i < ne; i += NT) claim[i] = 0;
  for (int e = tid; e < ne; e += NT)
    if (ehi[e] >= T) {
      const int si = atomicAdd(&n_surv, 1);
      sv_h[si] = ehi[e];
      sv_e[si] = (uint16_t)e;
    }
  __syncthreads();
  const int nsv = n_surv, nsp = (nsv + 15) & ~15;
  for (int i = nsv + tid; i < nsp; i += NT) sv_h[i] = 0u;  // pad to whole blocks: image 0 ranks below every entry
  __syncthreads();
  // output position = rank under (h desc, id asc).  First the count of survivors with a
  // strictly larger f32 image of h (monotonic in h; 16 per round from four ds_read_b128
  // broadcasts).  Survivors sharing an image get the same count — and only they do (a larger
  // image is counted by the smaller one's count) — so a claim table on the counts finds the
  // ties and near-ties (rare), which then take the full (h, id) comparison among themselves.
  // (One survivor per thread: a second round of the count doubled the phase, rank_probe.)
  int64_t oid_pf = 0;  // the output id of survivor tid (an idmap gather), loaded ahead of the count
  for (int si = tid; si < nsv; si += NT) {
    const uint32_t hh = sv_h[si];
    if (si == tid) oid_pf = out_id(a.idmap, eg[sv_e[si]]);
    int gt = 0;
    for (int f = 0; f < nsp; f += 16) {
      uint32_t kk[16];
#pragma unroll
      for (int j = 0; j < 4; ++j) *(uint4*)(kk + 4 * j) = *(const uint4*)(sv_h + f + 4 * j);
#pragma unroll
      for (int j = 0; j < 16; ++j) gt += kk[j] > hh;
    }
    rk[si] = (uint16_t)gt;
    atomicAdd(&claim[gt], 1);
  }
  __syncthreads();
  for (int si = tid; si < nsv; si += NT) {
    const int e = sv_e[si];
    const int gt = rk[si];
    int rank = gt;
    if (claim[gt] > 1) {
      const uint64_t hk = ek[e];
      const uint32_t g = eg[e], hh = ehi[e];
      for (int f = 0; f < nsv; ++f) {
        const int x = sv_e[f];
        rank += sv_h[f] == hh && ((ek[x] > hk) || (ek[x] == hk && eg[x] < g));
      }
    }
    if (rank < a.k) {
      sc[rank] = (float)eh[e];
      id[rank] = si == tid ? oid_pf : out_id(a.idmap, eg[e]);
    }
  }
  for (int i = n + tid; i < a.k; i += NT) {
    sc[i] = 0.f;
    id[i] = -1;
  }
  if (a.counts && tid == 0) a.counts[q] = n;
  __syncthreads();
  stamp(5);
}


}  // namespace bb
