// sq.hip — small-batch exact search: B <= 16 query rows of one side against an f32 index.
//
// The reference's own request shape is one query: get_similar_sets scores ONE target row
// (recommendation_system.py:213-217), the CF path one user row (:438), the pgvector retriever
// one embedding with k = 20 (lego_nlp_recommeder.py:305, 1394), HybridRecommender one user and
// one liked set (:612-677).  For such batches the MFMA scan + per-lane lists + list select of
// the large-batch path is mostly latency; here (sq.h):
//
//   pass   workgroup blk loads rows [blk·rpw, +rpw) of the f16 copy straight into registers
//          (every load in flight at once) and scores them on the matrix cores against the
//          query rows split into f16 hi + lo (16 queries per MFMA column block, f32
//          accumulation): a = Σ x̃_j (h_j + l_j).  |a − s| <= δ (sq_margin_of) for the exact
//          score s (E_x, N_x, Ñ_x = rr_stats).  Per query it leaves its top kSqM eligible (and present)
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
// write the C <= 64 keys v (lane < C) at their ranks r
__device__ __forceinline__ void sq_emit_ranked(const SqArgs& a, int b, uint64_t v, int r, int C, uint64_t gmax) {
  const int lane = threadIdx.x & 63;
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

__device__ __forceinline__ void sq_emit_rank(const SqArgs& a, int b, const uint64_t* cb, int C, uint64_t gmax) {
  const int lane = threadIdx.x & 63;
  const uint64_t v = lane < C ? cb[lane] : 0ull;
  int r = 0;
  for (int j = 0; j < C; ++j) r += cb[j] > v;  // (uniform; one broadcast LDS read per key)
  sq_emit_ranked(a, b, v, r, C, gmax);
}

__device__ __forceinline__ void sq_emit_any(const SqArgs& a, int b, const uint64_t* cb, int C, uint64_t gmax) {
  if (C <= 64 && (a.mopt & 2)) sq_emit_rank(a, b, cb, C, gmax);
  else if (C <= 64) sq_emit<1>(a, b, cb, C, gmax);
  else if (C <= 128) sq_emit<2>(a, b, cb, C, gmax);
  else sq_emit<4>(a, b, cb, C, gmax);  // C <= kSqCand
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
// wave maximum of a u64: the high words, then the low words of the lanes holding that high word
__device__ __forceinline__ uint64_t wave_max_u64(uint64_t v) {
  const uint32_t hi = wave_max_u32((uint32_t)(v >> 32));
  const uint32_t lo = wave_max_u32((uint32_t)(v >> 32) == hi ? (uint32_t)v : 0u);
  return ((uint64_t)hi << 32) | lo;
}

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
// The query split of one 8-element k-group as the MFMA's B operands: hi = f16(v) and lo =
// f16(v − hi), both rounded toward zero (v_cvt_pkrtz_f16_f32: one instruction per pair, and
// |hi| <= |v|, finite for finite v).  v − hi is exact in f32.  sq_margin_of bounds what the
// split leaves out.
__device__ __forceinline__ void split_f16x8(const float (&v)[8], u4v& hi, u4v& lo) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const auto h = __builtin_amdgcn_cvt_pkrtz(v[2 * i], v[2 * i + 1]);
    hi[i] = __builtin_bit_cast(uint32_t, h);
    lo[i] = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_pkrtz(v[2 * i] - (float)h[0], v[2 * i + 1] - (float)h[1]));
  }
}

// The re-rank margin 2δ (rr_margin) of one query row q (ldx wide; qn >= ‖q‖, qmax = max |q_j|),
// with h, l the split above and r = q − h − l:
//   δ = E_x·‖q‖ + Ñ_x·‖r‖ + γ·Ñ_x·(‖h‖ + ‖l‖) + 2^-23·N_x·‖q‖
// — Σ(x̃_j − x_j)q_j by Cauchy–Schwarz (E_x); Σ x̃_j r_j, the split's residual; the f32
// accumulation of the 2·ldb exact f16 products, Σ|x̃_j|(|h_j| + |l_j|) <= Ñ_x(‖h‖ + ‖l‖), over
// 2·ldb/32 chained MFMAs of 32 products + the accumulator each, every one of the 33 values
// rounded or truncated by at most 2^-23 of the largest partial sum whatever the matrix core's
// order (γ = 33·(2·ldb/32)·2^-23); and, the pass scoring the row as given (times its scale c)
// where the exact score s uses prep's normalised f32 row, |c·s − x·q| <= 2^-22·N_x·‖q‖ (the
// f32 rounding of every normalised element, of the raw f64 / bf16 input, and of s itself, in
// the units of the scaled row).  Toward-zero f16
// rounding is off by < 2^-10·|v| + 2^-24 (the subnormal spacing), so
//   ‖h‖ <= ‖q‖,  ‖l‖ <= ‖q − h‖ <= 2^-10·‖q‖ + 2^-24·√ldx,  ‖r‖ <= 2^-20·‖q‖ + 2^-23·√ldx.
// A row reaching the f16 range (|q_j| >= 2^15) gets an infinite margin: every item is then a
// candidate (the merge's exact slow path).  E_x, N_x, Ñ_x = rr_stats of the side.
__device__ __forceinline__ float sq_margin_of(const SqArgs& a, double qn, float qmax) {
  if (!(qmax < 32768.f)) return __builtin_huge_valf();
  const double rt = sqrt((double)a.ldx);
  const double hl = qn * (1.0 + 0x1p-10) + 0x1p-24 * rt, rn = 0x1p-20 * qn + 0x1p-23 * rt;
  const double gam = 33.0 * (2.0 * (double)a.ldb / 32.0) * 0x1p-23;
  const double ex = (double)a.stats[0], nx = (double)a.stats[1], nxb = (double)a.stats[2];
  const double d = ex * qn + nxb * rn + gam * nxb * hl + 0x1p-22 * nx * qn;
  return rr_margin(__double2float_ru(d * (1.0 + 0x1p-20)));
}

// the margin of one query row as the pass scored it (v: the row before its scale; the whole
// wave): ‖c·q‖ and max |c·q| of the scaled row, then sq_margin_of
__device__ __forceinline__ float sq_margin_row(const SqArgs& a, const float (&v)[kQnC]);

// The query rows of a wave as the pass and the merge see them: element lane + 64c of row
// b = min(w0 + step·t, B − 1) of the query source, as f32 — raw rows (q_kind 0, rounded to
// f32 when given as f64 / bf16) or CF rows (2) as they are, the stored f32 rows of item ids
// (1); zero past the row.  All loads are issued before any is used; `then` runs between the
// issue and the first use (the pass issues its item rows there).
template <int QT, typename Then>
__device__ __forceinline__ void sq_query_rows(const SqArgs& a, int w0, int step, int lane, float (&qv)[QT][kQnC],
                                              Then&& then) {
  const int B = a.B, ldx = (int)a.ldx;
  if (a.q_kind != 1 && a.q_dtype != F32) {  // (uniform) bf16 / f64 rows: the generic loader
    double xq[QT][kQnC];
#pragma unroll
    for (int t = 0; t < QT; ++t)
      load_chunk<kQnC>(a.q_src, a.q_dtype, (size_t)min(w0 + step * t, B - 1) * a.q_ld, 0, a.q_d, lane, xq[t]);
    then();
#pragma unroll
    for (int t = 0; t < QT; ++t)
#pragma unroll
      for (int c = 0; c < kQnC; ++c) qv[t][c] = (float)xq[t][c];
    return;
  }
  int64_t qid[QT];
  if (a.q_kind == 1) {
#pragma unroll
    for (int t = 0; t < QT; ++t) qid[t] = a.q_ids[min(w0 + step * t, B - 1)] - a.q_id_offset;
  }
  bool qok[QT];
  const int qlen = a.q_kind == 1 ? ldx : a.q_d;
#pragma unroll
  for (int t = 0; t < QT; ++t) {
    const int b = min(w0 + step * t, B - 1);
    qok[t] = a.q_kind != 1 || (qid[t] >= 0 && qid[t] < a.n);
    const float* src = a.q_kind == 1 ? a.X + (size_t)(qok[t] ? qid[t] : 0) * ldx : (const float*)a.q_src + (size_t)b * a.q_ld;
#pragma unroll
    for (int c = 0; c < kQnC; ++c) qv[t][c] = src[min(lane + 64 * c, qlen - 1)];
  }
  then();
#pragma unroll
  for (int t = 0; t < QT; ++t)
#pragma unroll
    for (int c = 0; c < kQnC; ++c) qv[t][c] = qok[t] && lane + 64 * c < qlen ? qv[t][c] : 0.f;
}

// The power-of-two scale 2^k of a query row (the wave's lanes: elements lane + 64c) that puts
// its largest element in [2^13, 2^14): exact, so the scaled row is the row times a positive
// constant, and well inside the f16 range of the split (an all-zero or non-finite row: 1).
__device__ __forceinline__ float sq_row_scale(const float (&v)[kQnC]) {
  float m = 0.f;
#pragma unroll
  for (int c = 0; c < kQnC; ++c) m = fmaxf(m, fabsf(v[c]));
  m = __int_as_float((int)wave_max_u32((uint32_t)__float_as_int(m)));  // non-negative: bits order
  if (!(m > 0.f) || !(m <= 3.4e38f)) return 1.f;
  int e;
  (void)frexpf(m, &e);  // m = f·2^e, f in [0.5, 1)
  // at most 2^126 (finite): a row whose largest |q| is below ~2^-112 scales to below 2^14,
  // still exact (a power of two), its small elements covered by the split's 2^-24 term
  return ldexpf(1.f, min(14 - e, 126));
}

__device__ __forceinline__ float sq_margin_row(const SqArgs& a, const float (&v)[kQnC]) {
  const float sc = sq_row_scale(v);
  double ss = 0.0;
  float mx = 0.f;
#pragma unroll
  for (int c = 0; c < kQnC; ++c) {
    const float x = v[c] * sc;
    ss = fma((double)x, (double)x, ss);
    mx = fmaxf(mx, fabsf(x));
  }
  ss = qn_wave_sum(ss);
  mx = __int_as_float((int)wave_max_u32((uint32_t)__float_as_int(mx)));
  return sq_margin_of(a, sqrt(ss) * (1.0 + 0x1p-40), mx);
}

// Approximate pass on the matrix cores.  Each wave scores whole 16-row chunks of the
// workgroup's rows (chunks w, w + 4): it loads their f16 rows straight into registers as the
// MFMA's A operands (lane l: row l & 15, bytes 64·ks + 16·(l >> 4) of k-step ks — two k-steps
// read whole 128-B lines), so the rows never pass through LDS; per k-step two
// v_mfma_f32_16x16x32_f16 against the query rows split into f16 hi + lo (B: 32 x 16 queries,
// up to 16 per launch), f32 accumulation.  KS = ldb / 32.
template <int KS>
__global__ __launch_bounds__(kSqThreads) void sq_scan_kernel(SqArgs a) {
  extern __shared__ __attribute__((aligned(16))) char sq_smem[];
  const int B = a.B;
  const int ldb = (int)a.ldb, ldx = (int)a.ldx;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int blk = blockIdx.x;
  const int r0 = blk * a.rpw, r1 = min(a.n, r0 + a.rpw), nr = r1 - r0;
  const int nck = (nr + 15) >> 4;
  float* qs = (float*)sq_smem;               // [B][ldx] f32 query rows
  uint32_t* sel = (uint32_t*)(qs + B * ldx);  // [B][rpw] approximate order images
  auto stamp = [&](int slot) {  // BB_SQ_TRACE probe runs: phase timeline (100 MHz), 8 words per workgroup
    if (a.trace && tid == 0) a.trace[(size_t)blk * 8 + slot] = __builtin_amdgcn_s_memrealtime();
  };
  stamp(0);
  // query rows as the pass scores them (sq_query_row): raw rows as given (rounded to f32), the
  // stored rows of item ids, CF rows — each times its power-of-two scale (sq_row_scale), so the
  // approximate scores are a positive multiple of the exact ones and no workgroup normalises
  // (the merge does, once per query, for the rescore).  Every query load of the wave (rows
  // b = w, w + 4, ...) is issued before any is used, then this wave's chunks of item rows —
  // unconditionally (a chunk past the block reloads row r0), so that the first use of a query
  // element waits for the query loads only and leaves the chunks in flight (a branch between
  // them would make the compiler drain everything).
  constexpr int QT = kSqMaxB / kSqWaves;
  constexpr int NCW = kSqMaxRows / 16 / kSqWaves;  // chunks per wave
  u4v af[NCW][KS];
  // the summary's eligibility words (item space, mask, per-query exclusions: every pointer
  // valid, the host passes all-ones / all-zeros words for an absent mask / exclusion set)
  constexpr int NE = kSqMaxRows / 64;
  uint32_t wp[NE], wm[NE], wx[QT][NE];
  auto load_rows = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < NCW; ++i) {
      const int rr = 16 * (w + kSqWaves * i) + (lane & 15);
      const int row = r0 + (rr < nr ? rr : 0);
      const u4v* src = (const u4v*)((const char*)a.Xb + (size_t)row * ldb * 2 + 16 * (lane >> 4));
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) af[i][ks] = src[4 * ks];
    }
#pragma unroll
    for (int e = 0; e < NE; ++e) {
      const int row = min(r0 + lane + 64 * e, a.n - 1);
      wp[e] = a.present[row >> 5];
      wm[e] = a.mask[row >> 5];
#pragma unroll
      for (int t = 0; t < QT; ++t) wx[t][e] = a.excl[(size_t)min(w + kSqWaves * t, B - 1) * a.excl_ld + (row >> 5)];
    }
    asm volatile("" ::: "memory");  // the scheduler would sink these loads below the query's first use
  };
  float qv[QT][kQnC];
  sq_query_rows<QT>(a, w, kSqWaves, lane, qv, load_rows);
  stamp(1);
  // this wave's queries (b = w + 4t, t < nq): scaled into LDS, the rows' maxima interleaved
  const int nq = B > w ? (B - w + kSqWaves - 1) / kSqWaves : 0;  // (wave-uniform)
  auto scale_rows = [&](auto NQC) __attribute__((always_inline)) {
    constexpr int NQ = decltype(NQC)::value;
    float sc[NQ];
#pragma unroll
    for (int t = 0; t < NQ; ++t) sc[t] = sq_row_scale(qv[t]);
#pragma unroll
    for (int t = 0; t < NQ; ++t) {
      const int b = w + kSqWaves * t;
#pragma unroll
      for (int c = 0; c < kQnC; ++c) {
        const int i = lane + 64 * c;
        if (i < ldx) qs[b * ldx + i] = qv[t][c] * sc[t];
      }
    }
  };
  switch (nq) {
    case 1: scale_rows(std::integral_constant<int, 1>{}); break;
    case 2: scale_rows(std::integral_constant<int, 2>{}); break;
    case 3: scale_rows(std::integral_constant<int, 3>{}); break;
    case 4: scale_rows(std::integral_constant<int, 4>{}); break;
    default: break;
  }
  __syncthreads();
  stamp(2);
  f4v acc[NCW];
#pragma unroll
  for (int i = 0; i < NCW; ++i) acc[i] = f4v{0.f, 0.f, 0.f, 0.f};
  {
    const int n = lane & 15;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      // the B operand of k-step ks: lane l holds query n = l & 15, k = 32·ks + 8·(l >> 4) + j
      const int k0 = 32 * ks + 8 * (lane >> 4);
      const bool on = n < B && k0 < ldx;
      const f4v v0 = on ? lds_f4(qs + n * ldx, k0 >> 2) : f4v{0.f, 0.f, 0.f, 0.f};
      const f4v v1 = on ? lds_f4(qs + n * ldx, (k0 >> 2) + 1) : f4v{0.f, 0.f, 0.f, 0.f};
      const float v[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
      u4v hi, lo;
      split_f16x8(v, hi, lo);
#pragma unroll
      for (int i = 0; i < NCW; ++i) {
        if (w + kSqWaves * i < nck) {  // wave-uniform
          acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, af[i][ks]),
                                                          __builtin_bit_cast(f16x8, hi), acc[i], 0, 0, 0);
          acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, af[i][ks]),
                                                          __builtin_bit_cast(f16x8, lo), acc[i], 0, 0, 0);
        }
      }
    }
  }
#pragma unroll
  for (int i = 0; i < NCW; ++i) {
    const int c = w + kSqWaves * i;
    const int n = lane & 15, rb = 16 * c + 4 * (lane >> 4);  // D: query n, rows rb .. rb + 3
    if (c < nck && n < B) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (rb + j < nr) sel[n * a.rpw + rb + j] = ord_of(acc[i][j] + 0.0f);
    }
  }
  __syncthreads();
  stamp(3);

  // per query: eligibility, the order images of the rows, the top kSqM eligible (and present)
  // approximate keys — the wave's queries side by side, so their wave-maximum chains (DPP +
  // readlane) interleave instead of running one after another
  auto summary = [&](auto NQC) __attribute__((always_inline)) {
    constexpr int NQ = decltype(NQC)::value;
    uint32_t o[NQ][NE], op[NQ][NE];
#pragma unroll
    for (int t = 0; t < NQ; ++t) {
      const int b = w + kSqWaves * t;
#pragma unroll
      for (int e = 0; e < NE; ++e) {
        const int i = lane + 64 * e, row = r0 + i;
        const uint32_t raw = i < nr ? sel[b * a.rpw + i] : 0u;
        const uint32_t bit = 1u << (row & 31);
        const bool pres = i < nr && (wp[e] & bit);
        const bool elig = pres && (wm[e] & bit) && !(wx[t][e] & bit);
        o[t][e] = elig ? raw : 0u;
        op[t][e] = a.drop && pres ? raw : 0u;
        if (i < nr) {
          a.ords[(size_t)b * a.ords_ld + row] = o[t][e];
          if (a.drop) a.ords_p[(size_t)b * a.ords_ld + row] = op[t][e];
        }
      }
    }
    stamp(5);
    for (int set = 0; set < (a.drop ? 2 : 1); ++set) {  // wave-uniform
      uint64_t mine[NQ];
#pragma unroll
      for (int t = 0; t < NQ; ++t) mine[t] = 0;
#pragma unroll
      for (int tt = 0; tt < kSqM; ++tt) {
        // the largest remaining order image; among equal ones the lowest row (largest key)
        uint32_t m[NQ];
#pragma unroll
        for (int t = 0; t < NQ; ++t) {
          uint32_t lm = 0;
#pragma unroll
          for (int e = 0; e < NE; ++e) lm = max(lm, set ? op[t][e] : o[t][e]);
          m[t] = wave_max_u32(lm);
        }
#pragma unroll
        for (int t = 0; t < NQ; ++t) {
          uint32_t(&oo)[NE] = set ? op[t] : o[t];
          uint64_t key = 0;
          if (m[t]) {
#pragma unroll
            for (int e = 0; e < NE; ++e) {
              const uint64_t hit = __ballot(oo[e] == m[t]);
              if (hit && !key) {
                const int src = __ffsll((unsigned long long)hit) - 1;
                key = make_key(m[t], a.gid0 + (uint32_t)(r0 + src + 64 * e));
                if (lane == src) oo[e] = 0u;
              }
            }
          }
          if (lane == tt) mine[t] = key;
        }
      }
#pragma unroll
      for (int t = 0; t < NQ; ++t)
        if (lane < kSqM)
          (set ? a.wg_ptop : a.wg_top)[((size_t)(w + kSqWaves * t) * a.nwg + blk) * kSqM + lane] = mine[t];
    }
  };
  switch (nq) {
    case 1: summary(std::integral_constant<int, 1>{}); break;
    case 2: summary(std::integral_constant<int, 2>{}); break;
    case 3: summary(std::integral_constant<int, 3>{}); break;
    case 4: summary(std::integral_constant<int, 4>{}); break;
    default: break;
  }
  stamp(4);
}

// Candidates of one query by one wave from the workgroups' lists of kSqM approximate keys
// (tops: [nwg][kSqM]): the bound is the K-th largest list maximum's 16-bit prefix (kth) or
// the largest maximum (rank 0), minus the margin (computed here from qrow while the list loads
// are in flight); the candidates are the list keys at or above it, plus every row of a
// workgroup whose kSqM-th key reaches it that its list did not hold.  Returns the count (it
// may exceed cap: the caller's slow path) and the bound.
template <int NL>  // nwg <= 64·NL
__device__ __forceinline__ uint32_t sq_gather(const SqArgs& a, const uint64_t* tops, const uint32_t* ords, int K,
                                              const float (&qv)[kQnC],
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
  const float margin = sq_margin_row(a, qv);
  uint32_t top;
  if (kth) {  // the largest multiple of 2^16 with >= K list keys at or above it (every key of
              // every list is a distinct item, so K of them reach it).  The workgroup maxima
              // alone are counted while at least 2K workgroups hold an eligible item (a quarter of
              // the ballots on the merge's latency chain); below that, every key (the maxima
              // alone left the bound at 0 when fewer than K workgroups hold one: ADVICE r04)
    int nz = 0;  // workgroups holding an eligible item (a selective mask can leave few)
#pragma unroll
    for (int i = 0; i < NL; ++i) nz += __popcll(__ballot(ent[i][0] != 0ull));
    const bool all_keys = nwg < 2 * K || nz < 2 * K;  // (uniform)
    uint32_t prefix = 0;
    for (int bit = 31; bit >= 16; --bit) {
      const uint32_t c = prefix | (1u << bit);
      int cnt = 0;
#pragma unroll
      for (int i = 0; i < NL; ++i) {
        cnt += __popcll(__ballot(ordk_of(ent[i][0]) >= c));
        if (all_keys)
#pragma unroll
          for (int j = 1; j < kSqM; ++j) cnt += __popcll(__ballot(ordk_of(ent[i][j]) >= c));
      }
      if (cnt >= K) prefix = c;
    }
    top = prefix;
  } else {  // the largest maximum (rank 0)
    uint32_t m = 0;
#pragma unroll
    for (int i = 0; i < NL; ++i) m = max(m, ordk_of(ent[i][0]));
    top = wave_max_u32(m);
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
  int32_t rank[kSqWaves][64];
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
  auto stamp = [&](int slot) {  // BB_SQ_TRACE probe runs: phase timeline (100 MHz)
    if (a.mtrace && tid == 0) a.mtrace[(size_t)b * 8 + slot] = __builtin_amdgcn_s_memrealtime();
  };
  stamp(0);
  // every wave: the query row as the pass scored it (before its scale); wave 2 writes the
  // rescore's f32 row into LDS — normalised with prep's arithmetic (qnorm.h: the same bits as
  // every other path) for raw rows, as it is otherwise — while waves 0 and 1 gather
  float qv[1][kQnC];
  sq_query_rows<1>(a, b, 0, lane, qv, [] {});
  if (w == 2) {
    if (a.q_kind == 0) {
      double x[kQnC];
      if (a.q_dtype == F32) {
#pragma unroll
        for (int c = 0; c < kQnC; ++c) x[c] = (double)qv[0][c];
      } else {
        load_chunk<kQnC>(a.q_src, a.q_dtype, (size_t)b * a.q_ld, 0, a.q_d, lane, x);
      }
      const double nrm = qn_norm(x), rinv = 1.0 / nrm;
#pragma unroll
      for (int c = 0; c < kQnC; ++c)
        if (lane + 64 * c < ldx) qs[lane + 64 * c] = qn_elem(x[c], nrm, rinv);
    } else {
#pragma unroll
      for (int c = 0; c < kQnC; ++c)
        if (lane + 64 * c < ldx) qs[lane + 64 * c] = qv[0][c];
    }
  }
  if (w == 0) {
    uint32_t T;
    const uint64_t* tops = a.wg_top + (size_t)b * a.nwg * kSqM;
    const uint32_t* ords = a.ords + (size_t)b * a.ords_ld;
    const uint32_t ce = (a.mopt & 1) && a.nwg <= 256 ? sq_gather<4>(a, tops, ords, a.K, qv[0], true, cand, kSqCand, &T)
                                                      : sq_gather<8>(a, tops, ords, a.K, qv[0], true, cand, kSqCand, &T);
    if (lane == 0) misc[0] = ce, misc[2] = T;
  } else if (w == 1) {
    uint32_t T = 0xFFFFFFFFu, cp = 0;
    if (a.drop) {
      const uint64_t* tops = a.wg_ptop + (size_t)b * a.nwg * kSqM;
      const uint32_t* ords = a.ords_p + (size_t)b * a.ords_ld;
      cp = (a.mopt & 1) && a.nwg <= 256 ? sq_gather<4>(a, tops, ords, 1, qv[0], false, ptmp, kSqPCand, &T)
                                        : sq_gather<8>(a, tops, ords, 1, qv[0], false, ptmp, kSqPCand, &T);
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
  const int C = (int)ce;
  if (C <= 64 && (a.mopt & 2)) {
    // rank counting on all four waves: wave w compares against keys [16w, 16w + 16)
    const uint64_t v = lane < C ? cand[lane] : 0ull;
    int r = 0;
    for (int j = 16 * w; j < min(C, 16 * w + 16); ++j) r += cand[j] > v;  // (uniform)
    L.rank[w][lane] = r;
    __syncthreads();
    if (w == 0) {
      uint64_t gm = lane < (int)cp ? cand[C + lane] : 0ull;  // cp <= kSqPCand = 64
      gm = wave_max_u64(gm);
      sq_emit_ranked(a, b, v, L.rank[0][lane] + L.rank[1][lane] + L.rank[2][lane] + L.rank[3][lane], C, gm);
    }
  } else if (w == 0) {
    uint64_t gm = 0;
    for (int i = lane; i < (int)cp; i += 64) gm = gm > cand[ce + i] ? gm : cand[ce + i];
    gm = wave_max_u64(gm);
    sq_emit_any(a, b, cand, C, gm);
  }
  if (a.mtrace && tid == 0) a.mtrace[(size_t)b * 8 + 4] = ce | ((uint64_t)cp << 32);
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
  const size_t lds = (size_t)a.B * a.ldx * 4 + (size_t)a.B * a.rpw * 4;  // <= 40 KiB
  bb_launch(sq_scan_kernel<KS>, dim3(a.nwg), dim3(kSqThreads), lds, s, a);
  return hipGetLastError();
}

}  // namespace

hipError_t launch_sq_scan(const SqArgs& a, hipStream_t s) {
  if (a.B < 1 || a.B > kSqMaxB || a.ldx > kRrMaxD || (a.ldx & 31) || a.ldb < a.ldx || (a.ldb & 63) || a.ldb > 512 ||
      a.K < 1 || a.K > kSqMaxK || a.rpw < 4 || (a.rpw & 3) || a.rpw > kSqMaxRows || a.nwg < 1 || a.nwg > kSqMaxWg ||
      (int64_t)a.nwg * a.rpw < a.n || (int64_t)(a.nwg - 1) * a.rpw >= a.n || a.n < 1 || a.ords_ld < a.n ||
      !a.present || !a.mask || !a.excl || a.excl_ld < 0 || !a.Xb || !a.X || !a.stats ||
      (a.q_kind == 1 ? !a.q_ids : !a.q_src) || (a.drop && (!a.ords_p || !a.wg_ptop)))
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
  bb_launch(sq_merge_kernel, dim3(a1 ? 2 * a0.B : a0.B), dim3(kSqThreads), 0, s, a0, a1 ? *a1 : a0);
  return hipGetLastError();
}

}  // namespace bb
