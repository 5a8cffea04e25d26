// select.hip — exact per-query top-K over a score slab (gfx950).
//
// Replaces np.argsort(sim)[::-1] + the Python filter walk of get_similar_sets
// (recommendation_system.py:217-247), the rated/valid filter loop + list.sort of the CF
// path (:441-461) and pgvector's ORDER BY <=> LIMIT k.  One workgroup (4 waves) per query
// row.  Eligible = in the slab ∧ present bit (structural: the side's item space) ∧ mask
// bit (valid_set_filter, :229/:454) ∧ ¬exclusion bit (items the user rated, :441-451).
//
// Fast path (bound + filter + sort):
//   pass 1  stage the row's order-images in LDS (0 = ineligible), track each thread's max
//           and the unmasked arg-max key (rank 0 of the reference's argsort, :217)
//   bound   T0 = the K-th largest per-thread max (and the carried list's K-th key): at
//           least K eligible elements are >= T0, so every member of the top K is too
//   pass 2  append every element with order-image >= T0 (typically ~K..2K of them)
//   sort    bitonic sort of the candidates by the full key (score desc, id asc) -> top K
// Exact fallback (candidates overflow the LDS buffer, e.g. masses of equal scores):
//   3-level radix select (12/12/8 bits) for the K-th score T, take everything above T and
//   the ties at T in ascending global id (carried keys first: earlier slabs = smaller ids).
#include "common.h"

namespace bb {

constexpr int kCandCap = 2048;                  // fast-path candidate capacity
constexpr int kOffHist = kMaxKInt * 8;          // radix path: cand[0..kMaxKInt) then hist
constexpr int kRegionA = kOffHist + 4096 * 4;   // 20 KiB, reused by both paths
static_assert(kCandCap * 8 <= kRegionA, "candidate buffer must fit region A");
constexpr int kOffTmax = kRegionA;              // u32[256] per-thread maxima
constexpr int kOffMisc = kOffTmax + kSelectThreads * 4;
constexpr int kOffOrds = kOffMisc + 256;        // staged row
constexpr size_t kSelectFixedLds = kOffOrds;

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

// Exact radix fallback over the staged row (+ carried keys).  Leaves cnt (<= K) keys in
// cand[0..cnt) and returns cnt.
__device__ uint32_t radix_select(const uint32_t* ords, int n, uint32_t gid0, const uint64_t* carry, int K,
                                 uint64_t* cand, uint32_t* hist, uint32_t* misc, uint32_t* scan_sh) {
  const int tid = threadIdx.x;
  for (int i = tid; i < 4096; i += kSelectThreads) hist[i] = 0;
  __syncthreads();
  for (int j = tid; j < n; j += kSelectThreads) {
    const uint32_t o = ords[j];
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
      const uint32_t o = ords[j];
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
      const uint32_t o = ords[j];
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
    const uint32_t o = ords[j];
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
      const uint32_t o = j < n ? ords[j] : 0u;
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

__global__ __launch_bounds__(kSelectThreads) void select_kernel(SelectArgs a) {
  extern __shared__ __attribute__((aligned(16))) char dsm[];
  uint64_t* cand = (uint64_t*)dsm;
  uint32_t* hist = (uint32_t*)(dsm + kOffHist);
  uint32_t* tmax = (uint32_t*)(dsm + kOffTmax);
  uint32_t* misc = (uint32_t*)(dsm + kOffMisc);  // [0..15] scalars
  uint32_t* scan_sh = misc + 16;                  // 8 words
  uint64_t* red = (uint64_t*)(misc + 32);         // 4 u64
  uint32_t* ords = (uint32_t*)(dsm + kOffOrds);

  const int row = blockIdx.x, tid = threadIdx.x;
  const int n = a.n_cols, K = a.K;
  const float* Srow = a.S + (size_t)row * a.lds;
  const uint32_t* excl = a.excl ? a.excl + (size_t)row * a.excl_ld : nullptr;
  const uint64_t* carry = a.carry_in ? a.carry_in + (size_t)row * K : nullptr;

  // ---- pass 1: stage order-images, per-thread max, unmasked arg-max ----
  uint64_t lmax = 0;
  uint32_t tm = 0;
  for (int j = tid; j < n; j += kSelectThreads) {
    const int64_t li = a.slab_start + j;
    const int64_t w = li >> 5;
    const uint32_t bit = 1u << (li & 31);
    const uint32_t o = ord_of(Srow[j]);
    const bool pr = !a.present || (a.present[w] & bit);
    if (pr) {
      const uint64_t key = make_key(o, a.gid0 + (uint32_t)j);
      lmax = key > lmax ? key : lmax;
    }
    const bool e = pr && (!a.mask || (a.mask[w] & bit)) && !(excl && (excl[w] & bit));
    const uint32_t oe = e ? o : 0u;
    ords[j] = oe;
    tm = oe > tm ? oe : tm;
  }
  tmax[tid] = tm;
  if (a.max_inout) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const uint64_t y = __shfl_xor(lmax, o);
      lmax = y > lmax ? y : lmax;
    }
    if ((tid & 63) == 0) red[tid >> 6] = lmax;
  }
  if (tid == 0) {
    misc[6] = 0;  // T0 (atomicMax)
    misc[7] = 0;  // candidate count
  }
  __syncthreads();
  if (a.max_inout && tid == 0) {
    uint64_t m = a.first_slab ? 0ull : a.max_inout[row];
    for (int i = 0; i < kSelectThreads / 64; ++i) m = red[i] > m ? red[i] : m;
    a.max_inout[row] = m;
  }

  // ---- bound: T0 = K-th largest per-thread max (ties: count of values >= mine) ----
  if (tm) {
    uint32_t ge = 0;
    for (int t = 0; t < kSelectThreads; ++t) ge += tmax[t] >= tm ? 1u : 0u;
    if (ge >= (uint32_t)K) atomicMax(&misc[6], tm);
  }
  __syncthreads();
  uint32_t T0 = misc[6];
  if (carry && K > 0) {
    const uint32_t ck = ordk_of(carry[K - 1]);  // K carried keys >= ck
    T0 = ck > T0 ? ck : T0;
  }
  if (T0 == 0) T0 = 1;  // fewer than K threads hold eligible items: take every eligible one

  // ---- pass 2: candidates >= T0 ----
  for (int j = tid; j < n; j += kSelectThreads) {
    const uint32_t o = ords[j];
    if (o >= T0) {
      const uint32_t p = atomicAdd(&misc[7], 1u);
      if (p < kCandCap) cand[p] = make_key(o, a.gid0 + (uint32_t)j);
    }
  }
  if (carry)
    for (int c = tid; c < K; c += kSelectThreads) {
      const uint64_t key = carry[c];
      if (key && ordk_of(key) >= T0) {
        const uint32_t p = atomicAdd(&misc[7], 1u);
        if (p < kCandCap) cand[p] = key;
      }
    }
  __syncthreads();
  uint32_t cnt = misc[7];
  if (cnt > (uint32_t)kCandCap) {
    __syncthreads();
    cnt = radix_select(ords, n, a.gid0, carry, K, cand, hist, misc, scan_sh);
  }

  // ---- sort candidates by full key, emit the top K ----
  int P = 1;
  while (P < (int)cnt) P <<= 1;
  for (int i = (int)cnt + tid; i < P; i += kSelectThreads) cand[i] = 0ull;
  __syncthreads();
  bitonic_desc_u64(cand, P);
  uint64_t* out = a.keys_out + (size_t)row * K;
  for (int i = tid; i < K; i += kSelectThreads) out[i] = i < (int)cnt ? cand[i] : 0ull;
}

static int g_select_attr_dev = -1;

hipError_t launch_select(const SelectArgs& a, int B, hipStream_t s) {
  if (a.K <= 0 || a.K > kMaxKInt || B <= 0 || a.n_cols <= 0 || a.n_cols > kSelectStageMax)
    return hipErrorInvalidValue;
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  if (g_select_attr_dev != dev) {
    e = hipFuncSetAttribute((const void*)select_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)(kSelectFixedLds + (size_t)kSelectStageMax * 4));
    if (e != hipSuccess) return e;
    g_select_attr_dev = dev;
  }
  const size_t bytes = kSelectFixedLds + (size_t)((a.n_cols + 3) & ~3) * 4;
  hipLaunchKernelGGL(select_kernel, dim3(B), dim3(kSelectThreads), bytes, s, a);
  return hipGetLastError();
}

}  // namespace bb
