// misc.hip — query preparation, cross-slab/shard finalize (rank-0 drop, hybrid
// union-blend), hard-constraint predicate masks and item-row conversion (gfx950).
#include "common.h"
#include "finalize_body.h"
#include "prep_body.h"
#include "qnorm.h"

#include <cstdlib>

namespace bb {


// ---------------------------------------------------------------------------------------
// rows -> (optionally L2-normalised) rows of the index dtype, padded to Dpad.
// Normalisation follows sklearn.preprocessing.normalize, which cosine_similarity applies
// to both arguments (recommendation_system.py:214): norm = sqrt(Σx²) (accumulated in f64
// here), zero norms -> 1, then a true division.  One wave per row.
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void convert_rows_kernel(const void* src, int src_dtype, int64_t n, int d,
                                                           int normalize, void* dst, int dst_dtype,
                                                           int64_t Dpad) {
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= n) return;
  const size_t sb = (size_t)row * d, db = (size_t)row * Dpad;
  double norm = 1.0;
  if (normalize) {
    double ss = 0.0;
    for (int i = lane; i < d; i += 64) {
      const double x = load_elem_d(src, src_dtype, sb + i);
      ss += x * x;
    }
    ss = wave_sum(ss);
    norm = sqrt(ss);
    if (norm == 0.0) norm = 1.0;
  }
  for (int i = lane; i < Dpad; i += 64) {
    float v = 0.f;
    if (i < d) v = (float)(load_elem_d(src, src_dtype, sb + i) / norm);
    store_elem(dst, dst_dtype, db + i, v);
  }
}

hipError_t launch_convert_rows(const void* src, int src_dtype, int64_t n, int d, int normalize, void* dst,
                               int dst_dtype, int64_t Dpad, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  const int64_t blocks = (n + 3) / 4;
  bb_launch(convert_rows_kernel, dim3((unsigned)blocks), dim3(256), 0, s, src, src_dtype, n, d,
                     normalize, dst, dst_dtype, Dpad);
  return hipGetLastError();
}


// f32 rows -> three bf16 planes (x = xh + xm + xl exactly) in the scan3 tile image
// (t3_chunk_offset, common.h).  One thread per 8-element chunk of a row: 32 B read, three
// 16-B plane chunks written.
__global__ __launch_bounds__(256) void split_planes_kernel(const float* src, int64_t n, int64_t ld, uint16_t* dst) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t cpr = ld >> 3;
  if (i >= n * cpr) return;
  const int64_t row = i / cpr;
  const int c = (int)(i - row * cpr);
  const float4 v0 = *(const float4*)(src + row * ld + 8 * c);
  const float4 v1 = *(const float4*)(src + row * ld + 8 * c + 4);
  const float v[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
  uint32_t hw[4], mw[4], lw[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    uint16_t h0, m0, l0, h1, m1, l1;
    split3_bits(v[2 * k], h0, m0, l0);
    split3_bits(v[2 * k + 1], h1, m1, l1);
    hw[k] = h0 | ((uint32_t)h1 << 16);
    mw[k] = m0 | ((uint32_t)m1 << 16);
    lw[k] = l0 | ((uint32_t)l1 << 16);
  }
  char* o = (char*)dst;
  *(uint4*)(o + t3_chunk_offset(row, c, 0, (int)ld)) = make_uint4(hw[0], hw[1], hw[2], hw[3]);
  *(uint4*)(o + t3_chunk_offset(row, c, 1, (int)ld)) = make_uint4(mw[0], mw[1], mw[2], mw[3]);
  *(uint4*)(o + t3_chunk_offset(row, c, 2, (int)ld)) = make_uint4(lw[0], lw[1], lw[2], lw[3]);
}

hipError_t launch_split_planes(const float* src, int64_t n, int64_t ld, uint16_t* dst, hipStream_t s) {
  if (n % 32 || ld % 8) return hipErrorInvalidValue;  // whole tiles, whole chunks
  const int64_t total = n * (ld >> 3);
  if (total <= 0) return hipSuccess;
  bb_launch(split_planes_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, src, n, ld, dst);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// Re-rank operands of an f32 index: the one-product f16 copy of every row (RNE, saturating)
// for the approximate MFMA scan — 11 significant bits, so its error, and every bound and
// candidate window built on it, is 1/8 of a bf16 copy's — and the statistics that bound that
// error (prep_kernel turns them into the per-query ε): max over rows of ||x̃−x||, ||x||, ||x̃|| (f64 sums, rounded up to
// f32, merged by integer atomicMax — non-negative floats order like their bit patterns).
// One wave per row.
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void rr_prepare_kernel(const float* src, int64_t npad, int64_t ld_f, uint16_t* dst,
                                                         int64_t ld_b, float* stats) {
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= npad) return;
  double e2 = 0.0, n2 = 0.0, b2 = 0.0;
  for (int64_t i = lane; i < ld_b; i += 64) {
    const float v = i < ld_f ? src[row * ld_f + i] : 0.f;
    const uint16_t hb = to_f16(v);
    const float bv = f16_val(hb);
    dst[row * ld_b + i] = hb;
    const double dv = (double)v, db = (double)bv;
    e2 += (dv - db) * (dv - db);
    n2 += dv * dv;
    b2 += db * db;
  }
  e2 = wave_sum(e2);
  n2 = wave_sum(n2);
  b2 = wave_sum(b2);
  if (lane == 0) {
    atomicMax((unsigned int*)&stats[0], __float_as_uint(__double2float_ru(sqrt(e2))));
    atomicMax((unsigned int*)&stats[1], __float_as_uint(__double2float_ru(sqrt(n2))));
    atomicMax((unsigned int*)&stats[2], __float_as_uint(__double2float_ru(sqrt(b2))));
  }
}

hipError_t launch_rr_prepare(const float* src, int64_t npad, int64_t ld_f, uint16_t* dst, int64_t ld_b, float* stats,
                             hipStream_t s) {
  if (npad <= 0) return hipSuccess;
  if (ld_b < ld_f) return hipErrorInvalidValue;
  bb_launch(rr_prepare_kernel, dim3((unsigned)((npad + 3) / 4)), dim3(256), 0, s, src, npad, ld_f, dst, ld_b,
                     stats);
  return hipGetLastError();
}

__global__ __launch_bounds__(256) void prep_kernel(PrepArgs a) { prep_rows(a, blockIdx.x); }

// both sides of a hybrid search in one launch: blocks [0, nb0) prep a0, the rest a1
__global__ __launch_bounds__(256) void prep2_kernel(PrepArgs a0, PrepArgs a1, int nb0) {
  if ((int)blockIdx.x < nb0)
    prep_rows(a0, blockIdx.x);
  else
    prep_rows(a1, blockIdx.x - nb0);
}

hipError_t launch_prep(const PrepArgs& a, hipStream_t s) {
  if (a.Bpad <= 0) return hipSuccess;
  bb_launch(prep_kernel, dim3((a.Bpad + 3) / 4), dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_prep2(const PrepArgs& a0, const PrepArgs& a1, hipStream_t s) {
  if (a0.Bpad <= 0 || a1.Bpad <= 0) return hipErrorInvalidValue;
  const int nb0 = (a0.Bpad + 3) / 4, nb1 = (a1.Bpad + 3) / 4;
  bb_launch(prep2_kernel, dim3(nb0 + nb1), dim3(256), 0, s, a0, a1, nb0);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// finalize: merge P shard lists per side, drop rank 0 (similar side), truncate, and for
// the hybrid run _combine_recommendations (recommendation_system.py:789-843): union of the
// two lists, h = wc·c + wcf·cf with a missing side = 0 (:812-818, in f64 like the Python
// floats), sort by (h desc, id asc), top k.  One side empty -> the other side's top k
// with its raw scores (:659-662).  One workgroup per query.
// ---------------------------------------------------------------------------------------
constexpr int kFinMerge = 4096;  // P * K_int capacity

template <typename T, typename Better>
__device__ void bitonic_desc(T* v, int P, Better better) {
  for (int k = 2; k <= P; k <<= 1)
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = threadIdx.x; i < P; i += kFinThreads) {
        const int ixj = i ^ j;
        if (ixj > i) {
          const T x = v[i], y = v[ixj];
          const bool desc = (i & k) == 0;
          if (desc ? better(y, x) : better(x, y)) {
            v[i] = y;
            v[ixj] = x;
          }
        }
      }
      __syncthreads();
    }
}

struct Blend {
  uint64_t h;   // order image of the f64 blended score
  uint32_t gid;
  uint32_t pad;
  double hv;
};

__global__ __launch_bounds__(kFinThreads) void finalize1_kernel(FinalizeArgs a) {
  const int q = blockIdx.x;
  finalize1_body<kMaxKInt>(a, q, a.keys + (size_t)q * a.K_int, a.keys + ((size_t)a.B + q) * a.K_int,
                           a.drop_rank0 && a.max_keys ? a.max_keys[q] : 0ull);
}

// Side lists of <= 64 keys (k <= 63: every configs[2]-shaped hybrid): one wave per row, the
// tables sized to the lists (≈5 KiB of LDS instead of ≈38 KiB), so a CU holds many rows and
// the barriers are one wave's.
constexpr int kFinSmallK = 64;
__global__ __launch_bounds__(64) void finalize1_small_kernel(FinalizeArgs a) {
  const int q = blockIdx.x;
  finalize1_body<kFinSmallK, 64>(a, q, a.keys + (size_t)q * a.K_int, a.keys + ((size_t)a.B + q) * a.K_int,
                                 a.drop_rank0 && a.max_keys ? a.max_keys[q] : 0ull);
}

// Side lists of <= 128 keys (k_side = 2k up to k = 63: the configs[2] hybrid's 101): ≈13 KiB
// of LDS per row instead of the 512-key instance's ≈41 KiB, so the other in-flight batches'
// kernels keep room on every CU (configs[2] 22.7 -> 24.5-25.3 M q/s), and four waves, so
// the rank count takes each of its <= 256 survivors in one round.
constexpr int kFinMidK = 128;
__global__ __launch_bounds__(256) void finalize1_mid_kernel(FinalizeArgs a) {
  const int q = blockIdx.x;
  finalize1_body<kFinMidK, 256>(a, q, a.keys + (size_t)q * a.K_int, a.keys + ((size_t)a.B + q) * a.K_int,
                                a.drop_rank0 && a.max_keys ? a.max_keys[q] : 0ull);
}

__global__ __launch_bounds__(kFinThreads) void finalize_kernel(FinalizeArgs a) {
  __shared__ uint64_t buf[kFinMerge];
  __shared__ uint64_t lists[2][kMaxKInt];
  __shared__ int counts[2];
  const int q = blockIdx.x, tid = threadIdx.x;

  for (int side = 0; side < a.sides; ++side) {
    const int m = a.P * a.K_int;
    int P2 = 1;
    while (P2 < m) P2 <<= 1;
    for (int i = tid; i < P2; i += kFinThreads) {
      uint64_t key = 0ull;
      if (i < m) {
        const int p = i / a.K_int, j = i % a.K_int;
        key = a.keys[(((size_t)p * a.sides + side) * a.B + q) * a.K_int + j];
      }
      buf[i] = key;
    }
    __syncthreads();
    if (a.P > 1) bitonic_desc(buf, P2, [](uint64_t x, uint64_t y) { return x > y; });
    const bool drop = side == 0 && a.drop_rank0;
    const int target = a.hybrid ? a.k_side : a.k;
    if (tid == 0) {
      int start = 0;
      if (drop && a.max_keys) {
        uint64_t gmax = 0;
        for (int p = 0; p < a.P; ++p) {
          const uint64_t v = a.max_keys[(size_t)p * a.B + q];
          gmax = v > gmax ? v : gmax;
        }
        if (buf[0] == gmax && gmax) start = 1;
      }
      int c = 0;
      for (int i = start; i < a.K_int && c < target; ++i) {
        if (!buf[i]) break;
        lists[side][c++] = buf[i];
      }
      counts[side] = c;
    }
    __syncthreads();
  }

  float* sc = a.scores + (size_t)q * a.k;
  int64_t* id = a.ids + (size_t)q * a.k;
  if (!a.hybrid || counts[0] == 0 || counts[1] == 0) {
    const int side = (!a.hybrid || counts[0] > 0) ? 0 : 1;
    const int c = counts[side] < a.k ? counts[side] : a.k;
    for (int i = tid; i < a.k; i += kFinThreads) {
      if (i < c) {
        sc[i] = float_of_ord(ordk_of(lists[side][i]));
        id[i] = out_id(a.idmap, gid_of(lists[side][i]));
      } else {
        sc[i] = 0.f;
        id[i] = -1;
      }
    }
    if (a.counts && tid == 0) a.counts[q] = c;
    return;
  }
  // hybrid union blend
  Blend* ent = (Blend*)buf;  // 2 * kMaxKInt entries of 24 B fit in buf (32 KB)
  const int c0 = counts[0], c1 = counts[1];
  __shared__ int n_ent;
  if (tid == 0) n_ent = 0;
  __syncthreads();
  for (int i = tid; i < c0; i += kFinThreads) {
    const uint32_t g = gid_of(lists[0][i]);
    const double cs = (double)float_of_ord(ordk_of(lists[0][i]));
    double fs = 0.0;
    for (int j = 0; j < c1; ++j)
      if (gid_of(lists[1][j]) == g) {
        fs = (double)float_of_ord(ordk_of(lists[1][j]));
        break;
      }
    const double h = blend_h(a.w_content, cs, a.w_cf, fs);
    const int pos = atomicAdd(&n_ent, 1);
    ent[pos] = Blend{ord64_of(h), g, 0u, h};
  }
  for (int j = tid; j < c1; j += kFinThreads) {
    const uint32_t g = gid_of(lists[1][j]);
    bool in_c = false;
    for (int i = 0; i < c0; ++i)
      if (gid_of(lists[0][i]) == g) {
        in_c = true;
        break;
      }
    if (in_c) continue;
    const double h = blend_h(a.w_content, 0.0, a.w_cf, (double)float_of_ord(ordk_of(lists[1][j])));
    const int pos = atomicAdd(&n_ent, 1);
    ent[pos] = Blend{ord64_of(h), g, 0u, h};
  }
  __syncthreads();
  const int ne = n_ent;
  int P2 = 1;
  while (P2 < ne) P2 <<= 1;
  for (int i = ne + tid; i < P2; i += kFinThreads) ent[i] = Blend{0ull, 0xFFFFFFFFu, 0u, 0.0};
  __syncthreads();
  bitonic_desc(ent, P2, [](const Blend& x, const Blend& y) {
    return x.h > y.h || (x.h == y.h && x.gid < y.gid);
  });
  const int c = ne < a.k ? ne : a.k;
  for (int i = tid; i < a.k; i += kFinThreads) {
    if (i < c) {
      sc[i] = (float)ent[i].hv;
      id[i] = out_id(a.idmap, ent[i].gid);
    } else {
      sc[i] = 0.f;
      id[i] = -1;
    }
  }
  if (a.counts && tid == 0) a.counts[q] = c;
}

// ---------------------------------------------------------------------------------------
// Streaming bound from a kScanPilot scan (scan4_kernel.h): each query row's K-th largest
// eligible half-tile maximum over the pilot rows.  The values come from K distinct half
// tiles, so K distinct eligible items score at least that much: it bounds the K-th score
// of the pilot sample — and of the whole index — from below, as the exact pilot list's
// K-th key did (the stream then appends every eligible score reaching it).  One workgroup
// per row: up to 16 values per thread, bitwise search of the K-th largest with ballot
// counts and one LDS exchange per bit.
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void pilot_bound_kernel(const uint32_t* top, int n_chunks, int m, int nb, int K,
                                                          uint64_t* thr_out) {
  constexpr int kPer = 16;  // values per thread: 2·n_chunks·m <= 4096
  __shared__ uint32_t xch[16];
  const int row = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int blk = row >> 5, r = row & 31;
  const int nv = 2 * n_chunks * m;  // (chunk, half, i) -> ((chunk·nb + blk)·64 + half·32 + r)·m + i
  uint32_t v[kPer];
#pragma unroll
  for (int e = 0; e < kPer; ++e) {
    const int j = tid + e * 256;
    uint32_t x = 0;
    if (j < nv) {
      const int i = j % m, ch = j / m, c = ch >> 1, hh = ch & 1;
      x = top[((size_t)(c * nb + blk) * 64 + hh * 32 + r) * m + i];
    }
    v[e] = x;
  }
  auto wave_count_ge = [&](uint32_t c) -> uint32_t {
    uint32_t n = 0;
#pragma unroll
    for (int e = 0; e < kPer; ++e) n += (uint32_t)__popcll(__ballot(v[e] >= c));
    return n;
  };
  uint32_t hi = 0, lo = 0xFFFFFFFFu;
#pragma unroll
  for (int e = 0; e < kPer; ++e) {
    hi = max(hi, v[e]);
    lo = v[e] ? min(lo, v[e]) : lo;
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
  __syncthreads();
  const uint32_t H = max(max(xch[8], xch[9]), max(xch[10], xch[11]));
  const uint32_t Lo = min(min(xch[12], xch[13]), min(xch[14], xch[15]));
  uint32_t P = 0;  // 0 = fewer than K values: take every eligible item
  if (xch[0] + xch[1] + xch[2] + xch[3] >= (uint32_t)K) {
    const uint32_t d = H ^ Lo;
    const int top_bit = d ? 31 - __builtin_clz(d) : -1;
    P = top_bit < 0 ? H : H & ~((2u << top_bit) - 1u);
    for (int bit = top_bit, st = 1; bit >= 0; --bit, ++st) {
      const uint32_t c = P | (1u << bit);
      const uint32_t wc = wave_count_ge(c);
      uint32_t* slot = xch + 4 * (st & 1);
      if (lane == 0) slot[wave] = wc;
      __syncthreads();
      if (slot[0] + slot[1] + slot[2] + slot[3] >= (uint32_t)K) P = c;
    }
  }
  if (tid == 0) thr_out[row] = (uint64_t)P << 32;
}

// The same bound with one wave per row (four rows per workgroup) when a row has at most
// 1,024 values (every configs[3]/[4] geometry: 2·chunks·m = 128): the search needs no
// barrier at all (the workgroup version paid one per bit for 4,096 short workgroups).
__global__ __launch_bounds__(256) void pilot_bound_wave_kernel(const uint32_t* top, int n_chunks, int m, int nb, int K,
                                                               int B, uint64_t* thr_out) {
  constexpr int kPer = 16;  // values per lane: 2·n_chunks·m <= 1024
  const int lane = threadIdx.x & 63, row = (int)blockIdx.x * 4 + (int)(threadIdx.x >> 6);
  if (row >= B) return;  // (whole waves)
  const int blk = row >> 5, r = row & 31;
  const int nv = 2 * n_chunks * m;
  uint32_t v[kPer];
  uint32_t hi = 0, lo = 0xFFFFFFFFu, cnt = 0;
#pragma unroll
  for (int e = 0; e < kPer; ++e) {
    const int j = lane + e * 64;
    uint32_t x = 0;
    if (j < nv) {
      const int i = j % m, ch = j / m, c = ch >> 1, hh = ch & 1;
      x = top[((size_t)(c * nb + blk) * 64 + hh * 32 + r) * m + i];
    }
    v[e] = x;
    hi = max(hi, x);
    lo = x ? min(lo, x) : lo;
  }
  auto count_ge = [&](uint32_t c) -> uint32_t {
    uint32_t n = 0;
#pragma unroll
    for (int e = 0; e < kPer; ++e) n += (uint32_t)__popcll(__ballot(v[e] >= c));
    return n;
  };
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    hi = max(hi, (uint32_t)__shfl_xor((int)hi, o));
    lo = min(lo, (uint32_t)__shfl_xor((int)lo, o));
  }
  cnt = count_ge(1u);
  uint32_t P = 0;  // 0 = fewer than K values: take every eligible item
  if (cnt >= (uint32_t)K) {
    const uint32_t d = hi ^ lo;
    const int top_bit = d ? 31 - __builtin_clz(d) : -1;
    P = top_bit < 0 ? hi : hi & ~((2u << top_bit) - 1u);
    for (int bit = top_bit; bit >= 0; --bit) {
      const uint32_t c = P | (1u << bit);
      if (count_ge(c) >= (uint32_t)K) P = c;
    }
  }
  if (lane == 0) thr_out[row] = (uint64_t)P << 32;
}

hipError_t launch_pilot_bound(const uint32_t* top, int n_chunks, int m, int nb, int K, int B, uint64_t* thr_out,
                              hipStream_t s) {
  if (B <= 0) return hipSuccess;
  if (!top || !thr_out || n_chunks <= 0 || m <= 0 || 2 * n_chunks * m > 16 * 256 || K <= 0 || B > 32 * nb)
    return hipErrorInvalidValue;
  if (2 * n_chunks * m <= 16 * 64)
    bb_launch(pilot_bound_wave_kernel, dim3((B + 3) / 4), dim3(256), 0, s, top, n_chunks, m, nb, K, B, thr_out);
  else
    bb_launch(pilot_bound_kernel, dim3(B), dim3(256), 0, s, top, n_chunks, m, nb, K, thr_out);
  return hipGetLastError();
}

hipError_t launch_finalize(const FinalizeArgs& a, hipStream_t s) {
  if (a.n_rows <= 0) return hipSuccess;
  if (a.n_rows > a.B || a.P * a.K_int > kFinMerge || a.K_int > kMaxKInt || a.sides < 1 || a.sides > 2) return hipErrorInvalidValue;
  static const bool legacy = ab_env("BB_FINALIZE_LEGACY") != nullptr;
  static const bool wide = ab_env("BB_FIN_WIDE") != nullptr;
  if (a.P == 1 && !legacy && a.K_int <= kFinSmallK && !wide)
    bb_launch(finalize1_small_kernel, dim3(a.n_rows), dim3(64), 0, s, a);
  else if (a.P == 1 && !legacy && a.K_int <= kFinMidK && !wide)
    bb_launch(finalize1_mid_kernel, dim3(a.n_rows), dim3(256), 0, s, a);
  else if (a.P == 1 && !legacy)
    bb_launch(finalize1_kernel, dim3(a.n_rows), dim3(kFinThreads), 0, s, a);
  else
    bb_launch(finalize_kernel, dim3(a.n_rows), dim3(kFinThreads), 0, s, a);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// hard-constraint predicates -> mask bitset (hard_constraint_filter.py:318-480).  One item
// per lane, one 64-bit ballot per wave -> two mask words.
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void mask_kernel(MaskArgs a) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  bool ok = false;
  if (i < a.n) {
    const int32_t p = a.parts[i];
    const int32_t y = a.year[i];
    const int32_t t = a.theme[i];
    ok = p > 0 && p >= a.parts_min && p <= a.parts_max && y >= a.year_min && y <= a.year_max;
    if (a.theme_mode) {
      const bool in_set = t >= 0 && t < a.n_theme_bits && ((a.theme_bits[t >> 5] >> (t & 31)) & 1u);
      ok = ok && t >= 0 && (a.theme_mode == 1 ? in_set : !in_set);
    }
  }
  const uint64_t b = __ballot(ok);
  const int lane = threadIdx.x & 63;
  const int64_t w0 = ((int64_t)blockIdx.x * 256 + (threadIdx.x & ~63)) >> 5;
  const int64_t nw = (a.n + 31) >> 5;
  if (lane == 0 && w0 < nw) a.out[w0] = (uint32_t)b;
  if (lane == 32 && w0 + 1 < nw) a.out[w0 + 1] = (uint32_t)(b >> 32);
}

hipError_t launch_mask(const MaskArgs& a, hipStream_t s) {
  if (a.n <= 0) return hipSuccess;
  bb_launch(mask_kernel, dim3((unsigned)((a.n + 255) / 256)), dim3(256), 0, s, a);
  return hipGetLastError();
}

__global__ void clear_bits_kernel(uint32_t* bits, const int64_t* ids, int64_t n_ids, int64_t n_items) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_ids) return;
  const int64_t id = ids[i];
  if (id < 0 || id >= n_items) return;
  atomicAnd(&bits[id >> 5], ~(1u << (id & 31)));
}

hipError_t launch_clear_bits(uint32_t* bits, const int64_t* ids, int64_t n_ids, int64_t n_items, hipStream_t s) {
  if (n_ids <= 0) return hipSuccess;
  bb_launch(clear_bits_kernel, dim3((unsigned)((n_ids + 255) / 256)), dim3(256), 0, s, bits, ids, n_ids,
                     n_items);
  return hipGetLastError();
}

}  // namespace bb
