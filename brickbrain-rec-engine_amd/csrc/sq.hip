// sq.hip — small-batch exact search: B <= 16 query rows of one side against an f32 index.
//
// The reference's own request shape is one query: get_similar_sets scores ONE target row
// (recommendation_system.py:213-217), the CF path one user row (:438), the pgvector retriever
// one embedding with k = 20 (lego_nlp_recommeder.py:305, 1394), HybridRecommender one user and
// one liked set (:612-677).  For such batches the MFMA scan + per-lane lists + list select of
// the large-batch path is mostly latency; here (sq.h):
//
//   pass   workgroup blk streams rows [blk·rpw, +rpw) of the bf16 copy through an LDS ring by
//          LDS-DMA (all of a 25K-row index's block in flight at once) and scores them in f32
//          against the f32 query rows (packed FMAs, 16 lanes per row): a = Σ x̃_j q_j.  With
//          q unrounded, |a − s| <= δ = ‖q‖·(E_x + γ·Ñ_x + 2^-23·N_x) for the exact score s
//          (Cauchy–Schwarz on Σ(x̃_j − x_j)q_j, the f32 summation bound γ = 2·ldb·2^-24, the f32
//          rounding of s; E_x, N_x, Ñ_x = rr_stats).  Per query it leaves its top kSqM
//          eligible (and present) approximate keys and every row's approximate order image.
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
typedef float f2v __attribute__((ext_vector_type(2)));
typedef uint32_t u4v __attribute__((ext_vector_type(4)));

// 16 B of LDS as four u32 (bf16 pairs).  (Read as a float vector, __builtin_bit_cast of its
// .y/.z/.w elements compiled to a single ds_read_b32 whose .x stood in for all four on ROCm
// 7.2 — wrong operands, not a fault.)
__device__ __forceinline__ u4v lds_u4(const void* p, int c) {
  return *(const __attribute__((address_space(3))) u4v*)((const __attribute__((address_space(3))) char*)((size_t)p) +
                                                         c * 16);
}

__device__ __forceinline__ bool bit_of(const uint32_t* w, int i) { return (w[i >> 5] >> (i & 31)) & 1u; }

__device__ __forceinline__ uint64_t wave_max_u64(uint64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const uint64_t y = __shfl_xor(v, o);
    v = v > y ? v : y;
  }
  return v;
}

template <int CTRL>
__device__ __forceinline__ float dpp_f32(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}
// sum over the 16 lanes of a DPP row (the approximate score: any order)
__device__ __forceinline__ float sum16_f32(float v) {
  v += dpp_f32<0xB1>(v);
  v += dpp_f32<0x4E>(v);
  v += dpp_f32<0x141>(v);
  v += dpp_f32<0x140>(v);
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

__device__ __forceinline__ void sq_emit_any(const SqArgs& a, int b, const uint64_t* cb, int C, uint64_t gmax) {
  if (C <= 64) sq_emit<1>(a, b, cb, C, gmax);
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
// this wave's LDS-DMA of the chunk to read has landed when at most N of its pieces are
// outstanding; then every wave's (one statement with the barrier: no memory access moves
// across it)
template <int N>
__device__ __forceinline__ void wait_barrier() {
  asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"i"(N) : "memory");
}

// Ring chunks of the pass (16 bf16 rows of up to 128·CPB elements = 4·CPB KiB each): the
// prologue puts NBUF-1 of them in flight (a 25,216 x 384 index's 99-row block is 7 chunks)
template <int CPB, int RS>
constexpr int sq_nbuf() { return CPB >= 4 ? 6 : CPB == 3 ? (RS >= 2 ? 10 : 8) : 10; }

// Approximate pass.  Lane (g, p): 16-lane group g = 4 slots per wave, p its chunk lane (16-B
// chunks of 8 bf16 elements p, p+16, ...).  Slot g takes row slot g % RS of the wave's RS rows
// and query set g / RS (QPW queries); a wave covers QW = (4/RS)·QPW queries, and with more
// queries than that the waves split into nqg query groups (kSqWaves / nqg row phases each).
// The only vector-memory operations of the row loop are the ring's DMAs (counted by vmcnt);
// eligibility is applied after the loop.
template <int CPB, int RS, int QPW>
__global__ __launch_bounds__(kSqThreads) void sq_scan_kernel(SqArgs a) {
  constexpr int QW = (4 / RS) * QPW;
  constexpr int NBUF = sq_nbuf<CPB, RS>();
  constexpr int CHB = 4096 * CPB;
  extern __shared__ __attribute__((aligned(16))) char sq_smem[];
  const int B = a.B;
  const int ldb = (int)a.ldb, nchb = ldb >> 3, ldx = (int)a.ldx;
  char* ring = sq_smem;
  float* qs = (float*)(sq_smem + NBUF * CHB);  // [B][ldx] f32 query rows
  uint32_t* sel = (uint32_t*)(qs + B * ldx);   // [B][rpw] approximate order images
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int p = lane & 15, g = lane >> 4;
  const int rs = g % RS, qsub = g / RS;
  const int nqg = (B + QW - 1) / QW;
  const int qg = w % nqg, ph = w / nqg, nph = kSqWaves / nqg;
  const int blk = blockIdx.x;
  const int r0 = blk * a.rpw, r1 = min(a.n, r0 + a.rpw), nr = r1 - r0;
  const int nck = (nr + 15) >> 4;
  const char* Xb = (const char*)a.Xb + (size_t)r0 * ldb * 2;  // the block
  const int blk_bytes = nr * ldb * 2;
  const uint32_t ring_lds = (uint32_t)(size_t)((__attribute__((address_space(3))) char*)ring);
  auto stage = [&](int c) __attribute__((always_inline)) {
    const uint32_t dst0 = ring_lds + (uint32_t)((c % NBUF) * CHB);
#pragma unroll
    for (int i = 0; i < CPB; ++i) {
      const int piece = w + 4 * i;
      const int off = c * 32 * ldb + piece * 1024 + lane * 16;  // byte offset in the block
      glds16(Xb + (off < blk_bytes ? off : 0), __builtin_amdgcn_readfirstlane(dst0 + piece * 1024));
    }
  };
#pragma unroll
  for (int c = 0; c < NBUF - 1; ++c)
    if (c < nck) stage(c);

  // query rows, as prep_kernel writes its f32 operand: normalised raw rows (qnorm.h), the
  // stored rows of item ids, or CF rows as they are; zero past the row.  Workgroup 0 also
  // hands them to the merge (q_out).
  for (int b = w; b < B; b += kSqWaves) {
    float v[kQnC];
    if (a.q_kind == 1) {  // (all loads of the row in flight together, as load_chunk)
      const int64_t id = a.q_ids[b] - a.q_id_offset;
      const bool ok = id >= 0 && id < a.n;
      const float* src = a.X + (size_t)(ok ? id : 0) * ldx;
#pragma unroll
      for (int c = 0; c < kQnC; ++c) v[c] = src[min(lane + 64 * c, ldx - 1)];
#pragma unroll
      for (int c = 0; c < kQnC; ++c) v[c] = ok ? v[c] : 0.f;
    } else {
      double xq[kQnC];
      load_chunk<kQnC>(a.q_src, a.q_dtype, (size_t)b * a.q_ld, 0, a.q_d, lane, xq);
      const double nrm = a.q_kind == 0 ? qn_norm(xq) : 1.0;
#pragma unroll
      for (int c = 0; c < kQnC; ++c) v[c] = qn_elem(xq[c], nrm);
    }
#pragma unroll
    for (int c = 0; c < kQnC; ++c) {
      const int i = lane + 64 * c;
      if (i < ldx) {
        qs[b * ldx + i] = v[c];
        if (blk == 0) a.q_out[(size_t)b * ldx + i] = v[c];
      }
    }
  }
  __syncthreads();  // (its vmcnt(0) also lands the prologue's chunks)
  f2v qf[QPW][CPB][4];
  int qb[QPW];
#pragma unroll
  for (int i = 0; i < QPW; ++i) {
    qb[i] = qg * QW + qsub * QPW + i;
#pragma unroll
    for (int j = 0; j < CPB; ++j) {
      const int c = p + 16 * j;
      const bool on = qb[i] < B && c < nchb && 8 * c < ldx;
      const f4v v0 = on ? lds_f4(qs + qb[i] * ldx, 2 * c) : f4v{0.f, 0.f, 0.f, 0.f};
      const f4v v1 = on ? lds_f4(qs + qb[i] * ldx, 2 * c + 1) : f4v{0.f, 0.f, 0.f, 0.f};
      qf[i][j][0] = f2v{v0.x, v0.y};
      qf[i][j][1] = f2v{v0.z, v0.w};
      qf[i][j][2] = f2v{v1.x, v1.y};
      qf[i][j][3] = f2v{v1.z, v1.w};
    }
  }

  for (int c = 0; c < nck; ++c) {
    const int ahead = min(nck - 1 - c, NBUF - 2);
    switch (ahead) {
      case 0: wait_barrier<0>(); break;
      case 1: wait_barrier<CPB>(); break;
      case 2: wait_barrier<2 * CPB>(); break;
      case 3: wait_barrier<3 * CPB>(); break;
      case 4: wait_barrier<4 * CPB>(); break;
      case 5: wait_barrier<5 * CPB>(); break;
      case 6: wait_barrier<6 * CPB>(); break;
      case 7: wait_barrier<7 * CPB>(); break;
      default: wait_barrier<8 * CPB>(); break;
    }
    // refill the buffer read in the previous phase (every wave has passed this barrier, its
    // reads consumed)
    if (c + NBUF - 1 < nck) stage(c + NBUF - 1);
    const char* buf = ring + (c % NBUF) * CHB;
    const int rows_c = min(16, nr - 16 * c);
    for (int s0 = ph * RS; s0 < 16; s0 += nph * RS) {  // wave-uniform
      const int ri = s0 + rs;
      const char* xr = buf + (ri < rows_c ? ri : 0) * ldb * 2;
      f2v acc[QPW];
#pragma unroll
      for (int i = 0; i < QPW; ++i) acc[i] = f2v{0.f, 0.f};
#pragma unroll
      for (int j = 0; j < CPB; ++j) {
        const u4v raw = lds_u4(xr, min(p + 16 * j, nchb - 1));
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const uint32_t u = raw[k];
          const f2v xv = f2v{__uint_as_float(u << 16), __uint_as_float(u & 0xFFFF0000u)};
#pragma unroll
          for (int i = 0; i < QPW; ++i) acc[i] = __builtin_elementwise_fma(xv, qf[i][j][k], acc[i]);
        }
      }
#pragma unroll
      for (int i = 0; i < QPW; ++i) {
        const float s = sum16_f32(acc[i].x + acc[i].y);
        if (p == 0 && ri < rows_c && qb[i] < B) sel[qb[i] * a.rpw + 16 * c + ri] = ord_of(s + 0.0f);
      }
    }
  }
  __syncthreads();

  // per query: eligibility, the order images of the rows, the top kSqM eligible (and present)
  // approximate keys
  for (int b = w; b < B; b += kSqWaves) {
    uint32_t o[kSqMaxRows / 64], op[kSqMaxRows / 64];
    const uint32_t* exb = a.excl ? a.excl + (size_t)b * a.excl_ld : nullptr;
#pragma unroll
    for (int e = 0; e < kSqMaxRows / 64; ++e) {
      const int i = lane + 64 * e, row = r0 + i;
      const uint32_t raw = i < nr ? sel[b * a.rpw + i] : 0u;
      const bool pres = i < nr && bit_of(a.present, row);
      const bool elig = pres && (!a.mask || bit_of(a.mask, row)) && (!exb || !bit_of(exb, row));
      o[e] = elig ? raw : 0u;
      op[e] = a.drop && pres ? raw : 0u;
      if (i < nr) {
        a.ords[(size_t)b * a.ords_ld + row] = o[e];
        if (a.drop) a.ords_p[(size_t)b * a.ords_ld + row] = op[e];
      }
    }
    for (int set = 0; set < (a.drop ? 2 : 1); ++set) {  // wave-uniform
      uint32_t(&oo)[kSqMaxRows / 64] = set ? op : o;
      uint64_t mine = 0;
#pragma unroll
      for (int t = 0; t < kSqM; ++t) {
        uint64_t best = 0;
#pragma unroll
        for (int e = 0; e < kSqMaxRows / 64; ++e) {
          const uint64_t k = oo[e] ? make_key(oo[e], a.gid0 + (uint32_t)(r0 + lane + 64 * e)) : 0ull;
          best = best > k ? best : k;
        }
        best = wave_max_u64(best);
#pragma unroll
        for (int e = 0; e < kSqMaxRows / 64; ++e)
          if (oo[e] && make_key(oo[e], a.gid0 + (uint32_t)(r0 + lane + 64 * e)) == best) oo[e] = 0u;
        if (lane == t) mine = best;
      }
      if (lane < kSqM) (set ? a.wg_ptop : a.wg_top)[((size_t)b * a.nwg + blk) * kSqM + lane] = mine;
    }
  }
}

template <int CPB, int RS>
size_t sq_lds_bytes(const SqArgs& a) {
  return (size_t)sq_nbuf<CPB, RS>() * 4096 * CPB + (size_t)a.B * a.ldx * 4 + (size_t)a.B * a.rpw * 4;
}

// Candidates of one query by one wave from the workgroups' lists of kSqM approximate keys
// (tops: [nwg][kSqM]): the bound is the K-th largest list maximum's 16-bit prefix (kth) or
// the largest maximum (rank 0), minus the margin; the candidates are the list keys at or
// above it, plus every row of a workgroup whose kSqM-th key reaches it that its list did not
// hold.  Returns the count (it may exceed cap: the caller's slow path) and the bound.
__device__ uint32_t sq_gather(const SqArgs& a, const uint64_t* tops, const uint32_t* ords, int K, float margin,
                              bool kth, uint64_t* cb, uint32_t cap, uint32_t* T_out) {
  const int lane = threadIdx.x & 63;
  const int nwg = a.nwg;
  constexpr int NL = kSqMaxWg / 64;
  uint64_t ent[NL][kSqM];
#pragma unroll
  for (int i = 0; i < NL; ++i) {
    const int t = lane + 64 * i;
#pragma unroll
    for (int j = 0; j < kSqM; ++j) ent[i][j] = t < nwg ? tops[(size_t)t * kSqM + j] : 0ull;
  }
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
    for (int j = 0; j < kSqM; ++j) base = wave_append(ordk_of(ent[i][j]) >= T, ent[i][j], cb, base, cap);
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
// order, rounded to f32); all kSqThreads threads
__device__ __forceinline__ void sq_rescore(const SqArgs& a, uint64_t* keys, int m, const float* qs) {
  SelectArgs sa{};
  sa.rr_x = a.X;
  sa.rr_ld = a.ldx;
  sa.rr_d = (int)a.ldx;
  sa.rr_gid_base = a.gid0;
  rr_rescore_any(keys, m, sa, qs);
}

// Slow exact path (more candidates than the buffers hold: masses of equal scores): every
// eligible row with order image >= Te and every present row >= Tp, rescored in batches of 256
// into a running exact top-K (and running present maximum).
__device__ void sq_slow(const SqArgs& a, int b, uint32_t Te, uint32_t Tp, const float* qs, uint64_t* eb,
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

// Merge: one workgroup per (side, query).
__global__ __launch_bounds__(kSqThreads) void sq_merge_kernel(SqArgs a0, SqArgs a1) {
  __shared__ __attribute__((aligned(16))) float qs[kRrMaxD];
  __shared__ uint64_t cand[kSqCand + kSqPCand];
  __shared__ uint64_t ptmp[kSqCand];
  __shared__ uint64_t run[kSqMaxK];
  __shared__ uint32_t scan_sh[kSelectThreads / 64];
  __shared__ uint32_t misc[8];
  __shared__ float margin_sh;
  const int side = (int)blockIdx.x >= a0.B ? 1 : 0;
  const SqArgs& a = side ? a1 : a0;
  const int b = (int)blockIdx.x - side * a0.B;
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  const int ldx = (int)a.ldx;
  const float* qrow = a.q_out + (size_t)b * ldx;
  for (int i = tid; i < ldx; i += kSqThreads) qs[i] = qrow[i];
  if (w == 0) {  // the bound δ of |approximate − exact| from the query's norm and the row statistics
    double ss = 0.0;
#pragma unroll
    for (int c = 0; c < kQnC; ++c) {
      const int i = lane + 64 * c;
      const double v = (double)qrow[min(i, ldx - 1)];
      ss = fma(i < ldx ? v : 0.0, v, ss);
    }
    ss = qn_wave_sum(ss);
    if (lane == 0) {
      const double qn = sqrt(ss) * (1.0 + 0x1p-40);
      const double gam = 2.0 * (double)a.ldb * 0x1p-24;
      const double d = qn * ((double)a.stats[0] + gam * (double)a.stats[2] + 0x1p-23 * (double)a.stats[1]);
      margin_sh = rr_margin(__double2float_ru(d * (1.0 + 0x1p-20)));
    }
  }
  __syncthreads();
  const float margin = margin_sh;
  if (w == 0) {
    uint32_t T;
    const uint32_t ce = sq_gather(a, a.wg_top + (size_t)b * a.nwg * kSqM, a.ords + (size_t)b * a.ords_ld, a.K, margin,
                                  true, cand, kSqCand, &T);
    if (lane == 0) misc[0] = ce, misc[2] = T;
  } else if (w == 1) {
    uint32_t T = 0xFFFFFFFFu, cp = 0;
    if (a.drop)
      cp = sq_gather(a, a.wg_ptop + (size_t)b * a.nwg * kSqM, a.ords_p + (size_t)b * a.ords_ld, 1, margin, false, ptmp,
                     kSqPCand, &T);
    if (lane == 0) misc[1] = cp, misc[3] = T;
  }
  __syncthreads();
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
  if (w == 0) {
    uint64_t gm = 0;
    for (int i = lane; i < (int)cp; i += 64) gm = gm > cand[ce + i] ? gm : cand[ce + i];
    gm = wave_max_u64(gm);
    sq_emit_any(a, b, cand, (int)ce, gm);
  }
}

template <int CPB, int RS, int QPW>
hipError_t launch_sq3(const SqArgs& a, hipStream_t s) {
  const size_t lds = sq_lds_bytes<CPB, RS>(a);
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  // dynamic LDS beyond 64 KiB needs the per-kernel opt-in, at the size launched (grows only)
  static size_t allowed = 64 * 1024;
  if (lds > allowed) {
    const hipError_t e = hipFuncSetAttribute((const void*)sq_scan_kernel<CPB, RS, QPW>,
                                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    allowed = lds;
  }
  hipLaunchKernelGGL((sq_scan_kernel<CPB, RS, QPW>), dim3(a.nwg), dim3(kSqThreads), lds, s, a);
  return hipGetLastError();
}

template <int CPB>
hipError_t launch_sq2(const SqArgs& a, hipStream_t s) {
  // (RS, QPW) by batch: 4 rows x 1 query, 4 x 2, 2 x 2 (x 2 query sets), 1 x 2 (x 4 sets;
  // two query groups of waves above 8 queries)
  if (a.B == 1) return launch_sq3<CPB, 4, 1>(a, s);
  if (a.B == 2) return launch_sq3<CPB, 4, 2>(a, s);
  if (a.B <= 4) return launch_sq3<CPB, 2, 2>(a, s);
  return launch_sq3<CPB, 1, 2>(a, s);
}

}  // namespace

hipError_t launch_sq_scan(const SqArgs& a, hipStream_t s) {
  if (a.B < 1 || a.B > kSqMaxB || a.ldx > kRrMaxD || (a.ldx & 31) || a.ldb < a.ldx || (a.ldb & 63) || a.ldb > 512 ||
      a.K < 1 || a.K > kSqMaxK || a.rpw < 4 || (a.rpw & 3) || a.rpw > kSqMaxRows || a.nwg < 1 || a.nwg > kSqMaxWg ||
      (int64_t)a.nwg * a.rpw < a.n || (int64_t)(a.nwg - 1) * a.rpw >= a.n || a.n < 1 || a.ords_ld < a.n ||
      !a.present || !a.Xb || !a.X || !a.stats || !a.q_out || (a.drop && (!a.ords_p || !a.wg_ptop)))
    return hipErrorInvalidValue;
  const int cpb = (int)((a.ldb + 127) / 128);
  if (cpb <= 1) return launch_sq2<1>(a, s);
  if (cpb <= 2) return launch_sq2<2>(a, s);
  if (cpb <= 3) return launch_sq2<3>(a, s);
  return launch_sq2<4>(a, s);
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
