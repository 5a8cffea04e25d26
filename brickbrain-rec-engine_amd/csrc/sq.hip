// sq.hip — small-batch exact search: B <= 16 query rows of one side against an f32 index.
//
// The reference's own request shape is one query: get_similar_sets scores ONE target row
// (recommendation_system.py:213-217), the CF path one user row (:438), the pgvector retriever
// one embedding with k = 20 (lego_nlp_recommeder.py:305, 1394), HybridRecommender one user and
// one liked set (:612-677).  For such batches the MFMA scan + per-lane lists + list select of
// the large-batch path is mostly latency; here (sq.h):
//
//   pass   workgroup blk stages rows [blk·rpw, +rpw) of the f16 copy into LDS by LDS-DMA
//          (the whole block in flight at once) and scores them on the matrix cores against the
//          query rows split into f16 hi + lo (16 queries per MFMA column block, f32
//          accumulation): a = Σ x̃_j (h_j + l_j).  |a − s| <= δ (sq_margin) for the exact score s
//          (E_x, N_x, Ñ_x = rr_stats).  Per query it leaves its top kSqM eligible (and present)
//          approximate keys and every row's approximate order image.
//   merge  one workgroup per query: L = a lower bound of the K-th largest workgroup maximum
//          (16-bit prefix search: K distinct items reach it, so the exact K-th score is
//          >= L − δ and every exact top-K member has a >= L − 2δ); the candidates are the list
//          keys >= L − 2δ, plus every such row of a workgroup whose kSqM-th key reaches it
//          (the list may have dropped some); for the rank-0 drop the present items within 2δ
//          of the largest present approximate score (the exact arg-max is among them).  The
//          candidates are rescored exactly (rescore_rows: f32 products summed in f64 in one
//          fixed order, rounded to f32 — the bits of every other path), sorted, rank 0
//          dropped, emitted.  More candidates than the buffers hold (masses of equal scores):
//          the same bounds over every row, rescored in batches into a running top-K.
#include "sq.h"
#include "qnorm.h"
#include "select_util.h"

namespace bb {
namespace {

constexpr int kSqThreads = 256;
constexpr int kSqWaves = kSqThreads / 64;
typedef uint32_t u4v __attribute__((ext_vector_type(4)));

// 16 B of LDS as four u32 (16-bit pairs).  (Read as a float vector, __builtin_bit_cast of its
// .y/.z/.w elements compiled to a single ds_read_b32 whose .x stood in for all four on ROCm
// 7.2 — wrong operands, not a fault.)
__device__ __forceinline__ u4v lds_u4(const void* p, int c) {
  return *(const __attribute__((address_space(3))) u4v*)((const __attribute__((address_space(3))) char*)((size_t)p) +
                                                         c * 16);
}


__device__ __forceinline__ uint64_t wave_max_u64(uint64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const uint64_t y = __shfl_xor(v, o);
    v = v > y ? v : y;
  }
  return v;
}

// ballot compaction of `take` lanes' keys into cb[base..cap): returns the new base (uniform;
// it keeps counting past cap)
__device__ __forceinline__ uint32_t wave_append(bool take, uint64_t key, uint64_t* cb, uint32_t base, uint32_t cap) {
  const uint64_t m = __ballot(take);
  const uint32_t pos = base + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
  if (take && pos < cap) cb[pos] = key;
  return base + (uint32_t)__popcll(m);
}

// Sort the first C (<= 64·E) exact keys of cb descending in registers and write query b's
// result: the K best, rank 0 dropped when it is the head (wave_sort_emit's rule), k_final of
// them; or the key list + the present maximum (BB_Q_OUT_KEYS / hybrid sides).
template <int E>
__device__ __forceinline__ void sq_emit(const SqArgs& a, int b, const uint64_t* cb, int C, uint64_t gmax) {
  const int lane = threadIdx.x & 63;
  uint64_t v[E];
#pragma unroll
  for (int s = 0; s < E; ++s) {
    const int e = s * 64 + lane;
    v[s] = e < C ? cb[e] : 0ull;
  }
  wave_bitonic_desc<E>(v, lane);
  const int cnt = C < a.K ? C : a.K;
  if (a.out_scores) {
    const uint64_t head = __shfl(v[0], 0);
    const int start = (gmax && cnt && head == gmax) ? 1 : 0;
    const int c = min(a.k_final, cnt - start);
    float* sc = a.out_scores + (size_t)b * a.k_final;
    int64_t* id = a.out_ids + (size_t)b * a.k_final;
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
    if (a.out_counts && lane == 0) a.out_counts[b] = c;
    return;
  }
  uint64_t* out = a.keys_out + (size_t)b * a.K;
#pragma unroll
  for (int s = 0; s < E; ++s) {
    const int e = s * 64 + lane;
    if (e < a.K) out[e] = e < cnt ? v[s] : 0ull;
  }
  for (int e = 64 * E + lane; e < a.K; e += 64) out[e] = 0ull;
  if (lane == 0 && a.max_out) a.max_out[b] = a.drop ? gmax : 0ull;
}

// The same result for C <= 64 keys without a sorting network: the keys are distinct (ids), so
// lane l's rank is the number of larger keys, counted against each key broadcast in turn.
__device__ __forceinline__ void sq_emit_rank(const SqArgs& a, int b, const uint64_t* cb, int C, uint64_t gmax) {
  const int lane = threadIdx.x & 63;
  const uint64_t v = lane < C ? cb[lane] : 0ull;
  const uint32_t vlo = (uint32_t)v, vhi = (uint32_t)(v >> 32);
  int r = 0;
  for (int j = 0; j < C; ++j) {  // uniform
    // (readlane returns int: each half goes through uint32_t, or the low one sign-extends)
    const uint64_t y = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane(vhi, j) << 32) |
                       (uint64_t)(uint32_t)__builtin_amdgcn_readlane(vlo, j);
    r += y > v;
  }
  const bool on = lane < C;
  const int cnt = C < a.K ? C : a.K;
  if (a.out_scores) {
    const uint64_t h = __ballot(on && r == 0);
    const uint64_t head = h ? __shfl(v, __ffsll((unsigned long long)h) - 1) : 0ull;
    const int start = (gmax && cnt && head == gmax) ? 1 : 0;
    const int c = min(a.k_final, cnt - start);
    float* sc = a.out_scores + (size_t)b * a.k_final;
    int64_t* id = a.out_ids + (size_t)b * a.k_final;
    const int i = r - start;
    if (on && i >= 0 && i < c) {
      sc[i] = float_of_ord(ordk_of(v));
      id[i] = (int64_t)gid_of(v);
    }
    for (int e = max(c, 0) + lane; e < a.k_final; e += 64) {
      sc[e] = 0.f;
      id[e] = -1;
    }
    if (a.out_counts && lane == 0) a.out_counts[b] = c;
    return;
  }
  uint64_t* out = a.keys_out + (size_t)b * a.K;
  if (on && r < cnt) out[r] = v;
  for (int e = cnt + lane; e < a.K; e += 64) out[e] = 0ull;
  if (lane == 0 && a.max_out) a.max_out[b] = a.drop ? gmax : 0ull;
}

__device__ __forceinline__ void sq_emit_any(const SqArgs& a, int b, const uint64_t* cb, int C, uint64_t gmax) {
  if (C <= 64 && (a.mopt & 2)) sq_emit_rank(a, b, cb, C, gmax);
  else if (C <= 64) sq_emit<1>(a, b, cb, C, gmax);
  else if (C <= 128) sq_emit<2>(a, b, cb, C, gmax);
  else sq_emit<4>(a, b, cb, C, gmax);  // C <= kSqCand
}

// LDS-DMA of one 1-KiB piece (the wave's 64 lanes x 16 B, lane-linear at dst), M0 saved and
// restored in the same statement (the compiler does not preserve it around inline asm)
__device__ __forceinline__ void glds16(const void* src, uint32_t dst) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(src), "s"(dst) : "memory");
}

template <int CTRL>
__device__ __forceinline__ uint32_t dpp_u32(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xF, 0xF, false);
}
// wave maximum of a u32 (uniform result): DPP within each 16-lane row, readlane across rows
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
  v = max(v, dpp_u32<0xB1>(v));
  v = max(v, dpp_u32<0x4E>(v));
  v = max(v, dpp_u32<0x141>(v));
  v = max(v, dpp_u32<0x140>(v));
  const uint32_t a = __builtin_amdgcn_readlane(v, 0), b = __builtin_amdgcn_readlane(v, 16),
                 c = __builtin_amdgcn_readlane(v, 32), d = __builtin_amdgcn_readlane(v, 48);
  return max(max(a, b), max(c, d));
}

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
// the query split of one 8-element k-group: hi = f16(v) and lo = f16(v − hi) (RNE,
// saturating: to_f16), packed as the MFMA's B operands.  The merge recomputes both from the
// f32 row for the bound (sq_margin), so nothing here is assumed about their accuracy.
__device__ __forceinline__ void split_f16x8(const float (&v)[8], u4v& hi, u4v& lo) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const uint16_t h0 = to_f16(v[2 * i]), h1 = to_f16(v[2 * i + 1]);
    hi[i] = (uint32_t)h0 | ((uint32_t)h1 << 16);
    lo[i] = (uint32_t)to_f16(v[2 * i] - f16_val(h0)) | ((uint32_t)to_f16(v[2 * i + 1] - f16_val(h1)) << 16);
  }
}

// Approximate pass on the matrix cores.  The workgroup's rows are staged into LDS by LDS-DMA
// (the whole block in flight at once, one wait) in a chunk-major image: 16-row chunks, and in
// a chunk the 16-B column cc of row r at slot cc·16 + r — one 1-KiB LDS-DMA piece (64 slots) per
// four columns, and the MFMA operand of a 32-wide k-step is one contiguous, conflict-free
// 1-KiB wave read.  Each wave scores whole chunks: per k-step two v_mfma_f32_16x16x32_f16 —
// the f16 rows (A: 16 rows x 32) against the query rows split into f16 hi + lo (B: 32 x 16
// queries, up to 16 per launch; |q − hi − lo| <= 2^-22·|q|), f32 accumulation.  KS = ldb / 32.
template <int KS>
__global__ __launch_bounds__(kSqThreads) void sq_scan_kernel(SqArgs a) {
  extern __shared__ __attribute__((aligned(16))) char sq_smem[];
  const int B = a.B;
  const int ldb = (int)a.ldb, ldx = (int)a.ldx;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int blk = blockIdx.x;
  const int r0 = blk * a.rpw, r1 = min(a.n, r0 + a.rpw), nr = r1 - r0;
  const int nck = (nr + 15) >> 4;
  constexpr int CHB = 32 * 32 * KS;                   // bytes of a 16-row chunk (16 · ldb · 2)
  char* rows = sq_smem;                               // [nck][CHB]
  float* qs = (float*)(sq_smem + (size_t)nck * CHB);  // [B][ldx] f32 query rows
  uint32_t* sel = (uint32_t*)(qs + B * ldx);          // [B][rpw] approximate order images
  auto stamp = [&](int slot) {  // BB_SQ_TRACE probe runs: phase timeline (100 MHz), 8 words per workgroup
    if (a.trace && tid == 0) a.trace[(size_t)blk * 8 + slot] = __builtin_amdgcn_s_memrealtime();
  };
  stamp(0);
  {
    const uint32_t rows_lds = (uint32_t)(size_t)((__attribute__((address_space(3))) char*)rows);
    const int r = lane & 15;
    for (int c = 0; c < nck; ++c) {
      const int row = 16 * c + r < nr ? r0 + 16 * c + r : r0;  // rows past the block: any valid row
      const char* src_row = (const char*)a.Xb + (size_t)row * ldb * 2;
      for (int P = w; P < KS; P += kSqWaves) {  // wave-uniform
        const int cc = 4 * P + (lane >> 4);
        glds16(src_row + cc * 16, __builtin_amdgcn_readfirstlane(rows_lds + (uint32_t)(c * CHB + P * 1024)));
      }
    }
  }

  // query rows, as prep_kernel writes its f32 operand: normalised raw rows (qnorm.h), the
  // stored rows of item ids, or CF rows as they are; zero past the row.  A wave's rows
  // (b = w, w + 4, ...) are all loaded before any is used: one round trip, not one per row.
  // Workgroup 0 also hands them to the merge (q_out).
  constexpr int QT = kSqMaxB / kSqWaves;
  double xq[QT][kQnC];
#pragma unroll
  for (int t = 0; t < QT; ++t) {
    const int b = w + kSqWaves * t;
    if (b >= B) break;  // wave-uniform
    if (a.q_kind == 1) {
      const int64_t id = a.q_ids[b] - a.q_id_offset;
      const bool ok = id >= 0 && id < a.n;
      const float* src = a.X + (size_t)(ok ? id : 0) * ldx;
      float v[kQnC];
#pragma unroll
      for (int c = 0; c < kQnC; ++c) v[c] = src[min(lane + 64 * c, ldx - 1)];
#pragma unroll
      for (int c = 0; c < kQnC; ++c) xq[t][c] = ok && lane + 64 * c < ldx ? (double)v[c] : 0.0;
    } else {
      load_chunk<kQnC>(a.q_src, a.q_dtype, (size_t)b * a.q_ld, 0, a.q_d, lane, xq[t]);
    }
  }
  stamp(1);
#pragma unroll
  for (int t = 0; t < QT; ++t) {
    const int b = w + kSqWaves * t;
    if (b >= B) break;
    const double nrm = a.q_kind == 0 ? qn_norm(xq[t]) : 1.0;
#pragma unroll
    for (int c = 0; c < kQnC; ++c) {
      const int i = lane + 64 * c;
      if (i < ldx) {
        const float v = qn_elem(xq[t][c], nrm);
        qs[b * ldx + i] = v;
        if (blk == 0) a.q_out[(size_t)b * ldx + i] = v;
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the rows' LDS-DMA has landed
  __syncthreads();
  stamp(2);
  // the B operand: lane l holds query n = l & 15, k = 32·ks + 8·(l >> 4) + j, as f16 hi + lo
  u4v qhi[KS], qlo[KS];
  {
    const int n = lane & 15;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int k0 = 32 * ks + 8 * (lane >> 4);
      const bool on = n < B && k0 < ldx;
      const f4v v0 = on ? lds_f4(qs + n * ldx, k0 >> 2) : f4v{0.f, 0.f, 0.f, 0.f};
      const f4v v1 = on ? lds_f4(qs + n * ldx, (k0 >> 2) + 1) : f4v{0.f, 0.f, 0.f, 0.f};
      const float v[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
      split_f16x8(v, qhi[ks], qlo[ks]);
    }
  }
  for (int c = w; c < nck; c += kSqWaves) {  // wave-uniform
    const char* chunk = rows + c * CHB;
    u4v af[KS];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) af[ks] = lds_u4(chunk, ks * 64 + lane);
    f4v acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, af[ks]), __builtin_bit_cast(f16x8, qhi[ks]),
                                                   acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, af[ks]), __builtin_bit_cast(f16x8, qlo[ks]),
                                                   acc, 0, 0, 0);
    }
    const int n = lane & 15, rb = 16 * c + 4 * (lane >> 4);  // D: query n, rows rb .. rb + 3
    if (n < B) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (rb + i < nr) sel[n * a.rpw + rb + i] = ord_of(acc[i] + 0.0f);
    }
  }
  __syncthreads();
  stamp(3);

  // per query: eligibility, the order images of the rows, the top kSqM eligible (and present)
  // approximate keys.  The item-space and mask words are the same for every query: loaded once;
  // a wave's exclusion words for all its queries in one round.
  constexpr int NE = kSqMaxRows / 64;
  uint32_t wp[NE], wm[NE], wx[QT][NE];
#pragma unroll
  for (int e = 0; e < NE; ++e) {
    const int row = min(r0 + lane + 64 * e, a.n - 1);
    wp[e] = a.present[row >> 5];
    wm[e] = a.mask ? a.mask[row >> 5] : 0xFFFFFFFFu;
  }
#pragma unroll
  for (int t = 0; t < QT; ++t) {
    const int b = w + kSqWaves * t;
#pragma unroll
    for (int e = 0; e < NE; ++e) {
      const int row = min(r0 + lane + 64 * e, a.n - 1);
      wx[t][e] = a.excl && b < B ? a.excl[(size_t)b * a.excl_ld + (row >> 5)] : 0u;
    }
  }
#pragma unroll
  for (int t = 0; t < QT; ++t) {
    const int b = w + kSqWaves * t;
    if (b >= B) break;  // wave-uniform
    uint32_t o[NE], op[NE];
#pragma unroll
    for (int e = 0; e < NE; ++e) {
      const int i = lane + 64 * e, row = r0 + i;
      const uint32_t raw = i < nr ? sel[b * a.rpw + i] : 0u;
      const uint32_t bit = 1u << (row & 31);
      const bool pres = i < nr && (wp[e] & bit);
      const bool elig = pres && (wm[e] & bit) && !(wx[t][e] & bit);
      o[e] = elig ? raw : 0u;
      op[e] = a.drop && pres ? raw : 0u;
      if (i < nr) {
        a.ords[(size_t)b * a.ords_ld + row] = o[e];
        if (a.drop) a.ords_p[(size_t)b * a.ords_ld + row] = op[e];
      }
    }
    for (int set = 0; set < (a.drop ? 2 : 1); ++set) {  // wave-uniform
      uint32_t(&oo)[NE] = set ? op : o;
      uint64_t mine = 0;
#pragma unroll
      for (int tt = 0; tt < kSqM; ++tt) {
        // the largest remaining order image; among equal ones the lowest row (largest key)
        uint32_t lm = 0;
#pragma unroll
        for (int e = 0; e < NE; ++e) lm = max(lm, oo[e]);
        const uint32_t m = wave_max_u32(lm);
        uint64_t key = 0;
        if (m) {
#pragma unroll
          for (int e = 0; e < NE; ++e) {
            const uint64_t hit = __ballot(oo[e] == m);
            if (hit && !key) {
              const int src = __ffsll((unsigned long long)hit) - 1;
              key = make_key(m, a.gid0 + (uint32_t)(r0 + src + 64 * e));
              if (lane == src) oo[e] = 0u;
            }
          }
        }
        if (lane == tt) mine = key;
      }
      if (lane < kSqM) (set ? a.wg_ptop : a.wg_top)[((size_t)b * a.nwg + blk) * kSqM + lane] = mine;
    }
  }
  stamp(4);
}

// the re-rank margin 2δ (rr_margin) of a query row, every lane of the wave (qrow: the f32 row,
// ldx wide), with h, l the pass's f16 split of q and r = q − h − l (recomputed here in f64):
//   δ = E_x·‖q‖ + Ñ_x·‖r‖ + γ·Ñ_x·(‖h‖ + ‖l‖) + 2^-23·N_x·‖q‖
// — Σ(x̃_j − x_j)q_j by Cauchy–Schwarz (E_x); Σ x̃_j r_j (the split's residual); the f32
// accumulation of the 2·ldb exact f16 products, Σ|x̃_j|(|h_j| + |l_j|) <= Ñ_x(‖h‖ + ‖l‖), over
// 2·ldb/32 chained MFMAs of 32 products + the accumulator each, every one of the 33 values
// rounded or truncated by at most 2^-23 of the largest partial sum whatever the matrix core's
// order (γ = 33·(2·ldb/32)·2^-23); and the f32 rounding of s (2^-23·N_x).  E_x, N_x, Ñ_x =
// rr_stats of the side.
__device__ __forceinline__ float sq_margin(const SqArgs& a, const float* qrow) {
  const int lane = threadIdx.x & 63, ldx = (int)a.ldx;
  float v[kQnC];
#pragma unroll
  for (int c = 0; c < kQnC; ++c) v[c] = qrow[min(lane + 64 * c, ldx - 1)];
  double qq = 0.0, rr = 0.0, hh = 0.0, ll = 0.0;
#pragma unroll
  for (int c = 0; c < kQnC; ++c) {
    const float x = lane + 64 * c < ldx ? v[c] : 0.f;
    const double h = (double)f16_val(to_f16(x));
    const double l = (double)f16_val(to_f16(x - (float)h));
    const double r = (double)x - h - l;
    qq = fma((double)x, (double)x, qq);
    rr = fma(r, r, rr);
    hh = fma(h, h, hh);
    ll = fma(l, l, ll);
  }
  qq = qn_wave_sum(qq);
  rr = qn_wave_sum(rr);
  hh = qn_wave_sum(hh);
  ll = qn_wave_sum(ll);
  const double up = 1.0 + 0x1p-40;
  const double qn = sqrt(qq) * up, rn = sqrt(rr) * up, sn = (sqrt(hh) + sqrt(ll)) * up;
  const double gam = 33.0 * (2.0 * (double)a.ldb / 32.0) * 0x1p-23;
  const double ex = (double)a.stats[0], nx = (double)a.stats[1], nxb = (double)a.stats[2];
  const double d = ex * qn + nxb * rn + gam * nxb * sn + 0x1p-23 * nx * qn;
  return rr_margin(__double2float_ru(d * (1.0 + 0x1p-20)));
}

// Candidates of one query by one wave from the workgroups' lists of kSqM approximate keys
// (tops: [nwg][kSqM]): the bound is the K-th largest list maximum's 16-bit prefix (kth) or
// the largest maximum (rank 0), minus the margin (computed here from qrow while the list loads
// are in flight); the candidates are the list keys at or above it, plus every row of a
// workgroup whose kSqM-th key reaches it that its list did not hold.  Returns the count (it
// may exceed cap: the caller's slow path) and the bound.
template <int NL>  // nwg <= 64·NL
__device__ __forceinline__ uint32_t sq_gather(const SqArgs& a, const uint64_t* tops, const uint32_t* ords, int K, const float* qrow,
                              bool kth, uint64_t* cb, uint32_t cap, uint32_t* T_out) {
  const int lane = threadIdx.x & 63;
  const int nwg = a.nwg;
  uint64_t ent[NL][kSqM];
#pragma unroll
  for (int i = 0; i < NL; ++i) {
    const int t = lane + 64 * i;
#pragma unroll
    for (int j = 0; j < kSqM; ++j) ent[i][j] = t < nwg ? tops[(size_t)t * kSqM + j] : 0ull;
  }
  const float margin = sq_margin(a, qrow);
  uint32_t top;
  if (kth) {  // the largest multiple of 2^16 with >= K workgroup maxima at or above it
    uint32_t prefix = 0;
    for (int bit = 31; bit >= 16; --bit) {
      const uint32_t c = prefix | (1u << bit);
      int cnt = 0;
#pragma unroll
      for (int i = 0; i < NL; ++i) cnt += __popcll(__ballot(ordk_of(ent[i][0]) >= c));
      if (cnt >= K) prefix = c;
    }
    top = prefix;
  } else {  // the largest maximum (rank 0)
    uint64_t m = 0;
#pragma unroll
    for (int i = 0; i < NL; ++i) m = m > ent[i][0] ? m : ent[i][0];
    top = ordk_of(wave_max_u64(m));
  }
  const uint32_t T = top ? ord_sub(top, margin) : 1u;
  *T_out = T;
  uint32_t base = 0;
#pragma unroll
  for (int i = 0; i < NL; ++i)
#pragma unroll
    for (int j = 0; j < kSqM; ++j) {
      const bool take = ordk_of(ent[i][j]) >= T;
      if ((a.mopt & 1) && !__ballot(take)) break;  // each list is descending
      base = wave_append(take, ent[i][j], cb, base, cap);
    }
#pragma unroll
  for (int i = 0; i < NL; ++i) {
    uint64_t ovm = __ballot(ordk_of(ent[i][kSqM - 1]) >= T);
    while (ovm) {
      const int src = __ffsll((unsigned long long)ovm) - 1;
      ovm &= ovm - 1;
      const uint64_t last = __shfl(ent[i][kSqM - 1], src);
      const int q0 = (src + 64 * i) * a.rpw, q1 = min(a.n, q0 + a.rpw);
      for (int rb = q0; rb < q1; rb += 64) {
        const int row = rb + lane;
        const uint32_t o = row < q1 ? ords[row] : 0u;
        const uint64_t key = make_key(o, a.gid0 + (uint32_t)row);
        base = wave_append(o && o >= T && key < last, key, cb, base, cap);
      }
    }
  }
  return base;
}

// rescore keys[0..m) in place: exact keys (rescore_rows: the f32 rows, f64 sums in one fixed
// order, rounded to f32); all kSqThreads threads, 4 rows in flight per 16-lane group at d = 384
// (the merge's ~K candidates in one round of gathers)
__device__ __forceinline__ void sq_rescore(const SqArgs& a, uint64_t* keys, int m, const float* qs) {
  SelectArgs sa{};
  sa.rr_x = a.X;
  sa.rr_ld = a.ldx;
  sa.rr_d = (int)a.ldx;
  sa.rr_gid_base = a.gid0;
  const int cpl = (((int)a.ldx >> 2) + 15) >> 4;
  const int t = threadIdx.x;
  if (cpl <= 1) rescore_rows<1, 12, 16>(keys, m, sa, qs, t);
  else if (cpl <= 2) rescore_rows<2, 8, 16>(keys, m, sa, qs, t);
  else if (cpl <= 4) rescore_rows<4, 4, 16>(keys, m, sa, qs, t);
  else if (cpl <= 6) rescore_rows<6, 4, 16>(keys, m, sa, qs, t);
  else rescore_rows<8, 2, 16>(keys, m, sa, qs, t);
}

// Slow exact path (more candidates than the buffers hold: masses of equal scores): every
// eligible row with order image >= Te and every present row >= Tp, rescored in batches of 256
// into a running exact top-K (and running present maximum).
__device__ __forceinline__ void sq_slow(const SqArgs& a, int b, uint32_t Te, uint32_t Tp, const float* qs, uint64_t* eb,
                        uint64_t* pb, uint64_t* run, uint32_t* scan_sh, uint32_t* misc) {
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  const uint32_t* oe = a.ords + (size_t)b * a.ords_ld;
  const uint32_t* opr = a.drop ? a.ords_p + (size_t)b * a.ords_ld : nullptr;
  int rc = 0;       // running list length (uniform)
  uint64_t gm = 0;  // running present maximum (wave 0)
  for (int base = 0; base < a.n; base += kSqThreads) {
    const int row = base + tid;
    const uint32_t o = row < a.n ? oe[row] : 0u;
    const uint32_t op = opr && row < a.n ? opr[row] : 0u;
    const bool te = o && o >= Te, tp = op && op >= Tp;
    uint32_t ne, np;
    const uint32_t pe = block_excl_scan(te ? 1u : 0u, scan_sh, ne);
    if (te) eb[pe] = make_key(o, a.gid0 + (uint32_t)row);
    const uint32_t pp = block_excl_scan(tp ? 1u : 0u, scan_sh, np);
    if (tp) pb[pp] = make_key(op, a.gid0 + (uint32_t)row);
    __syncthreads();
    if (ne) sq_rescore(a, eb, (int)ne, qs);
    if (np) sq_rescore(a, pb, (int)np, qs);
    __syncthreads();
    if (w == 0) {
      uint64_t pm = 0;
      for (int i = lane; i < (int)np; i += 64) pm = pm > pb[i] ? pm : pb[i];
      pm = wave_max_u64(pm);
      gm = gm > pm ? gm : pm;
      if (ne) {  // merge the batch into the running list: sort run[0..rc) + eb[0..ne) (<= 384)
        uint64_t v[8];
#pragma unroll
        for (int s = 0; s < 8; ++s) {
          const int e = s * 64 + lane;
          v[s] = e < rc ? run[e] : e - rc < (int)ne ? eb[e - rc] : 0ull;
        }
        wave_bitonic_desc<8>(v, lane);
        rc = min(a.K, rc + (int)ne);
#pragma unroll
        for (int s = 0; s < 8; ++s)
          if (s * 64 + lane < rc) run[s * 64 + lane] = v[s];
      }
      if (lane == 0) misc[0] = (uint32_t)rc;
    }
    __syncthreads();
    rc = (int)misc[0];
    __syncthreads();
  }
  if (w == 0) sq_emit_any(a, b, run, rc, gm);
}

struct SqMergeLds {
  __attribute__((aligned(16))) float qs[kRrMaxD];
  uint64_t cand[kSqCand + kSqPCand];
  uint64_t ptmp[kSqCand];
  uint64_t run[kSqMaxK];
  uint32_t scan_sh[kSelectThreads / 64];
  uint32_t misc[8];
};

// Merge of query b of one side (a: a kernel argument itself, so its fields stay scalar loads)
__device__ __forceinline__ void sq_merge_row(const SqArgs& a, int b, SqMergeLds& L) {
  float* qs = L.qs;
  uint64_t* cand = L.cand;
  uint64_t* ptmp = L.ptmp;
  uint64_t* run = L.run;
  uint32_t* scan_sh = L.scan_sh;
  uint32_t* misc = L.misc;
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  const int ldx = (int)a.ldx;
  const float* qrow = a.q_out + (size_t)b * ldx;
  auto stamp = [&](int slot) {  // BB_SQ_TRACE probe runs: phase timeline (100 MHz)
    if (a.mtrace && tid == 0) a.mtrace[(size_t)b * 8 + slot] = __builtin_amdgcn_s_memrealtime();
  };
  stamp(0);
  for (int i = tid; i < ldx; i += kSqThreads) qs[i] = qrow[i];
  if (w == 0) {
    uint32_t T;
    const uint64_t* tops = a.wg_top + (size_t)b * a.nwg * kSqM;
    const uint32_t* ords = a.ords + (size_t)b * a.ords_ld;
    const uint32_t ce = (a.mopt & 1) && a.nwg <= 256 ? sq_gather<4>(a, tops, ords, a.K, qrow, true, cand, kSqCand, &T)
                                                      : sq_gather<8>(a, tops, ords, a.K, qrow, true, cand, kSqCand, &T);
    if (lane == 0) misc[0] = ce, misc[2] = T;
  } else if (w == 1) {
    uint32_t T = 0xFFFFFFFFu, cp = 0;
    if (a.drop) {
      const uint64_t* tops = a.wg_ptop + (size_t)b * a.nwg * kSqM;
      const uint32_t* ords = a.ords_p + (size_t)b * a.ords_ld;
      cp = (a.mopt & 1) && a.nwg <= 256 ? sq_gather<4>(a, tops, ords, 1, qrow, false, ptmp, kSqPCand, &T)
                                        : sq_gather<8>(a, tops, ords, 1, qrow, false, ptmp, kSqPCand, &T);
    }
    if (lane == 0) misc[1] = cp, misc[3] = T;
  }
  __syncthreads();
  stamp(1);
  const uint32_t ce = misc[0], cp = misc[1];
  if (ce > (uint32_t)kSqCand || cp > (uint32_t)kSqPCand) {
    const uint32_t Te = misc[2], Tp = misc[3];
    __syncthreads();
    sq_slow(a, b, Te, Tp, qs, cand, ptmp, run, scan_sh, misc);
    return;
  }
  for (int i = tid; i < (int)cp; i += kSqThreads) cand[ce + i] = ptmp[i];
  __syncthreads();
  sq_rescore(a, cand, (int)(ce + cp), qs);
  __syncthreads();
  stamp(2);
  if (w == 0) {
    uint64_t gm = 0;
    for (int i = lane; i < (int)cp; i += 64) gm = gm > cand[ce + i] ? gm : cand[ce + i];
    gm = wave_max_u64(gm);
    sq_emit_any(a, b, cand, (int)ce, gm);
    if (a.mtrace && lane == 0) a.mtrace[(size_t)b * 8 + 4] = ce | ((uint64_t)cp << 32);
  }
  stamp(3);
}

// Merge: one workgroup per (side, query); each side's body reads its own argument directly
// (a reference selected between the two would copy both to the stack).
__global__ __launch_bounds__(kSqThreads) void sq_merge_kernel(SqArgs a0, SqArgs a1) {
  __shared__ SqMergeLds L;
  if ((int)blockIdx.x < a0.B) sq_merge_row(a0, (int)blockIdx.x, L);
  else sq_merge_row(a1, (int)blockIdx.x - a0.B, L);
}

template <int KS>
hipError_t launch_sq_ks(const SqArgs& a, hipStream_t s) {
  const int nck = (a.rpw + 15) / 16;
  const size_t lds = (size_t)nck * 32 * 32 * KS + (size_t)a.B * a.ldx * 4 + (size_t)a.B * a.rpw * 4;
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  // dynamic LDS beyond 64 KiB needs the per-kernel opt-in, at the size launched (grows only)
  static size_t allowed = 64 * 1024;
  if (lds > allowed) {
    const hipError_t e = hipFuncSetAttribute((const void*)sq_scan_kernel<KS>,
                                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    allowed = lds;
  }
  hipLaunchKernelGGL(sq_scan_kernel<KS>, dim3(a.nwg), dim3(kSqThreads), lds, s, a);
  return hipGetLastError();
}

}  // namespace

int sq_rows_cap(int64_t ldb, int B, int64_t ldx) {
  const int64_t avail = 160 * 1024 - (int64_t)B * ldx * 4;
  int rows = kSqMaxRows;
  while (rows > 16 && (int64_t)(rows / 16) * 32 * ldb + (int64_t)B * rows * 4 > avail) rows -= 16;
  return rows;
}

hipError_t launch_sq_scan(const SqArgs& a, hipStream_t s) {
  if (a.B < 1 || a.B > kSqMaxB || a.ldx > kRrMaxD || (a.ldx & 31) || a.ldb < a.ldx || (a.ldb & 63) || a.ldb > 512 ||
      a.K < 1 || a.K > kSqMaxK || a.rpw < 4 || (a.rpw & 3) || a.rpw > kSqMaxRows || a.nwg < 1 || a.nwg > kSqMaxWg ||
      (int64_t)a.nwg * a.rpw < a.n || (int64_t)(a.nwg - 1) * a.rpw >= a.n || a.n < 1 || a.ords_ld < a.n ||
      !a.present || !a.Xb || !a.X || !a.stats || !a.q_out || (a.drop && (!a.ords_p || !a.wg_ptop)))
    return hipErrorInvalidValue;
  switch (a.ldb / 32) {
    case 2: return launch_sq_ks<2>(a, s);
    case 4: return launch_sq_ks<4>(a, s);
    case 6: return launch_sq_ks<6>(a, s);
    case 8: return launch_sq_ks<8>(a, s);
    case 10: return launch_sq_ks<10>(a, s);
    case 12: return launch_sq_ks<12>(a, s);
    case 14: return launch_sq_ks<14>(a, s);
    case 16: return launch_sq_ks<16>(a, s);
    default: return hipErrorInvalidValue;
  }
}

hipError_t launch_sq_merge(const SqArgs& a0, const SqArgs* a1, hipStream_t s) {
  if (a0.B < 1 || a0.B > kSqMaxB || (a1 && a1->B != a0.B) ||
      (a0.out_scores ? (!a0.out_ids || a0.k_final < 1 || a0.k_final > a0.K) : !a0.keys_out) ||
      (a1 && !a1->keys_out))
    return hipErrorInvalidValue;
  hipLaunchKernelGGL(sq_merge_kernel, dim3(a1 ? 2 * a0.B : a0.B), dim3(kSqThreads), 0, s, a0, a1 ? *a1 : a0);
  return hipGetLastError();
}

}  // namespace bb
