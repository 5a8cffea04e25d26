// sq.hip — small-batch exact search: B <= 16 query rows of one side against an f32 index.
//
// The reference's own request shape is one query: get_similar_sets scores ONE target row
// (recommendation_system.py:213-217), the CF path one user row (:438), the pgvector retriever
// one embedding with k = 20 (lego_nlp_recommeder.py:305, 1394).  For such batches the bf16
// MFMA scan + candidate lists + exact re-rank of the large-batch path is three dependent
// launches of mostly latency; here ONE pass over the f32 rows computes every score exactly —
// f32 products summed in f64 in rescore_rows' fixed order (select_util.h: lane p of a 16-lane
// group takes the 16-B chunks p, p+16, ... in order, then the DPP tree), rounded to f32 — so
// the keys are bit-identical to the rescored keys of every other path and no re-rank is
// needed.  At B = 1 the pass reads the 38.7 MB of f32 rows once (HBM / MALL bound); at B = 16
// it is bound by the f64 FMA rate (each row's chunks feed QPW queries per lane).
//
//   row pass   workgroup blk owns rows [blk·rpw, +rpw): 4 waves, each 16-lane group one
//              (row, query set) slot; per query the workgroup keeps the order image of every
//              row (LDS), then leaves its top kSqM keys, its present maximum (rank 0) and the
//              order images themselves (for overflowed lists) in global memory
//   merge      per query (one wave): L = a lower bound of the K-th largest workgroup maximum
//              (16-bit prefix search: K distinct items reach it, so every exact top-K member
//              has an order image >= L); candidates = list keys >= L, plus — for a list whose
//              kSqM-th key reaches L, i.e. which may have dropped such items — every row of
//              that workgroup >= L; sort in registers, drop rank 0, emit.  More than kSqCand
//              candidates (masses of equal scores): an exact wave select over all rows.
//
// The merge is its own launch (one wave per query), or — a.ticket set — runs in the workgroup
// whose arrival comes last (one launch): the hand-off then follows MI355X_MICROARCH.md's
// inter-workgroup rule for sc1 traffic: every hand-off store sc1 (write-through), each
// storing wave drains (s_waitcnt vmcnt(0)), a workgroup barrier, ONE agent-scope atomic add
// per workgroup on one counter, and every load of the handed-off bytes in the last
// workgroup an sc1 load.
#include "common.h"
#include "qnorm.h"
#include "select_util.h"

namespace bb {
namespace {

constexpr int kSqThreads = 256;
constexpr int kSqWaves = kSqThreads / 64;

template <bool SC1>
__device__ __forceinline__ void st32(uint32_t* p, uint32_t v) {
  if constexpr (SC1) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else *p = v;
}
template <bool SC1>
__device__ __forceinline__ void st64(uint64_t* p, uint64_t v) {
  if constexpr (SC1) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else *p = v;
}
template <bool SC1>
__device__ __forceinline__ uint32_t ld32(const uint32_t* p) {
  if constexpr (SC1) return __hip_atomic_load(const_cast<uint32_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else return *p;
}
template <bool SC1>
__device__ __forceinline__ uint64_t ld64(const uint64_t* p) {
  if constexpr (SC1) return __hip_atomic_load(const_cast<uint64_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else return *p;
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

// ballot compaction of `take` lanes' keys into cb[base..): returns the new base (uniform)
__device__ __forceinline__ uint32_t wave_append(bool take, uint64_t key, uint64_t* cb, uint32_t base) {
  const uint64_t m = __ballot(take);
  const uint32_t pos = base + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
  if (take && pos < (uint32_t)kSqCand) cb[pos] = key;
  return base + (uint32_t)__popcll(m);
}

// Sort the first C (<= 64·E) keys of cb descending in registers and write query b's result:
// the K best, rank 0 dropped when it is the head (wave_sort_emit's rule), k_final of them; or
// the key list + the present maximum (BB_Q_OUT_KEYS).
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
  if (lane == 0) a.max_out[b] = a.drop ? gmax : 0ull;
}

// Exact fallback of one query (more than kSqCand candidates reached L: masses of equal
// scores): T = the largest order image with >= K rows at or above it, by a bitwise search
// over every row's image; then the rows above T and, in row (= id) order, the ties at T up
// to K keys.
template <bool SC1>
__device__ void sq_fallback(const SqArgs& a, int b, uint64_t* cb, uint64_t gmax) {
  const int lane = threadIdx.x & 63;
  const uint32_t* ords = a.ords + (size_t)b * a.ords_ld;
  const int n = a.n, K = a.K;
  uint32_t T = 0;
  for (int bit = 31; bit >= 0; --bit) {
    const uint32_t c = T | (1u << bit);
    int cnt = 0;
    for (int r0 = 0; r0 < n; r0 += 64) {
      const int row = r0 + lane;
      const uint32_t o = row < n ? ld32<SC1>(ords + row) : 0u;
      cnt += __popcll(__ballot(o >= c));
    }
    if (cnt >= K) T = c;
  }
  uint32_t base = 0;
  const uint32_t lo = T ? T + 1u : 1u;  // strictly above T (every eligible row when T == 0)
  for (int r0 = 0; r0 < n; r0 += 64) {
    const int row = r0 + lane;
    const uint32_t o = row < n ? ld32<SC1>(ords + row) : 0u;
    base = wave_append(o >= lo, make_key(o, a.gid0 + (uint32_t)row), cb, base);
  }
  if (T) {
    for (int r0 = 0; r0 < n && base < (uint32_t)K; r0 += 64) {
      const int row = r0 + lane;
      const uint32_t o = row < n ? ld32<SC1>(ords + row) : 0u;
      const bool tie = o == T;
      const uint64_t m = __ballot(tie);
      const uint32_t rk = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
      if (tie && base + rk < (uint32_t)K) cb[base + rk] = make_key(o, a.gid0 + (uint32_t)row);
      base = min((uint32_t)K, base + (uint32_t)__popcll(m));
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  sq_emit<2>(a, b, cb, (int)base, gmax);  // base <= K <= kSqMaxK = 128
}

// Merge of query b by one wave: the workgroups' lists -> the exact top-K (see the header).
template <bool SC1>
__device__ void sq_merge_wave(const SqArgs& a, int b, uint64_t* cb) {
  const int lane = threadIdx.x & 63;
  const int nwg = a.nwg, K = a.K;
  const uint64_t* top = a.wg_top + (size_t)b * nwg * kSqM;
  constexpr int NL = kSqMaxWg / 64;  // lists per lane
  uint64_t ent[NL][kSqM];
#pragma unroll
  for (int i = 0; i < NL; ++i) {
    const int t = lane + 64 * i;
#pragma unroll
    for (int j = 0; j < kSqM; ++j) ent[i][j] = t < nwg ? ld64<SC1>(top + (size_t)t * kSqM + j) : 0ull;
  }
  uint64_t gmax = 0;
  if (a.drop) {
#pragma unroll
    for (int i = 0; i < NL; ++i) {
      const int t = lane + 64 * i;
      const uint64_t pm = t < nwg ? ld64<SC1>(a.wg_pmax + (size_t)b * nwg + t) : 0ull;
      gmax = gmax > pm ? gmax : pm;
    }
    gmax = wave_max_u64(gmax);
  }
  // L: the largest multiple of 2^16 with >= K workgroup maxima at or above it
  uint32_t prefix = 0;
  for (int bit = 31; bit >= 16; --bit) {
    const uint32_t c = prefix | (1u << bit);
    int cnt = 0;
#pragma unroll
    for (int i = 0; i < NL; ++i) cnt += __popcll(__ballot(ordk_of(ent[i][0]) >= c));
    if (cnt >= K) prefix = c;
  }
  const uint32_t L = prefix ? prefix : 1u;
  uint32_t base = 0;
#pragma unroll
  for (int i = 0; i < NL; ++i)
#pragma unroll
    for (int j = 0; j < kSqM; ++j) base = wave_append(ordk_of(ent[i][j]) >= L, ent[i][j], cb, base);
  // overflowed lists: every row of that workgroup at or above L that the list did not hold
#pragma unroll
  for (int i = 0; i < NL; ++i) {
    uint64_t ovm = __ballot(ordk_of(ent[i][kSqM - 1]) >= L);
    while (ovm) {
      const int src = __ffsll((unsigned long long)ovm) - 1;
      ovm &= ovm - 1;
      const uint64_t last = __shfl(ent[i][kSqM - 1], src);
      const int q0 = (src + 64 * i) * a.rpw, q1 = min(a.n, q0 + a.rpw);
      const uint32_t* ords = a.ords + (size_t)b * a.ords_ld;
      for (int r0 = q0; r0 < q1; r0 += 64) {
        const int row = r0 + lane;
        const uint32_t o = row < q1 ? ld32<SC1>(ords + row) : 0u;
        const uint64_t key = make_key(o, a.gid0 + (uint32_t)row);
        base = wave_append(o >= L && key < last, key, cb, base);
      }
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  if (base > (uint32_t)kSqCand) {
    sq_fallback<SC1>(a, b, cb, gmax);
    return;
  }
  const int C = (int)base;
  if (C <= 64) sq_emit<1>(a, b, cb, C, gmax);
  else if (C <= 128) sq_emit<2>(a, b, cb, C, gmax);
  else sq_emit<4>(a, b, cb, C, gmax);
}

// LDS-DMA of one 1-KiB piece (the wave's 64 lanes x 16 B, lane-linear at dst), M0 saved and
// restored in the same statement (the compiler does not preserve it around inline asm)
__device__ __forceinline__ void glds16(const void* src, uint32_t dst) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(src), "s"(dst) : "memory");
}
// this wave's LDS-DMA of the chunk c has landed when at most n of its pieces are outstanding
// (one statement with the barrier: no memory access moves across it)
template <int N>
__device__ __forceinline__ void wait_barrier() {
  asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"i"(N) : "memory");
}

// Row pass.  The workgroup's rows are one contiguous block of the row-major f32 matrix; it
// streams through an LDS ring of NBUF chunks of 16 rows by LDS-DMA (each wave issues CPL
// 1-KiB pieces per chunk — a 16-row chunk is 64·ldx <= 4·CPL KiB — NBUF-1 chunks ahead), so
// the whole block's bytes are in flight early; the only vector-memory operations of the loop
// are those DMAs, counted by vmcnt.  Lane (g, p): 16-lane group g = 4 slots per wave, p its
// chunk lane.  Slot g takes row slot g % RS of the wave's RS rows and query set g / RS (QPW
// queries); a wave covers QW = (4/RS)·QPW queries, and with more queries than that the waves
// split into nqg query groups (kSqWaves / nqg row phases each).  Eligibility is applied after
// the pass (the loop stores the raw order image of every (query, row)).
template <int CPL, int RS>
constexpr int sq_nbuf() { return CPL <= 4 ? 6 : CPL == 6 ? (RS >= 2 ? 6 : 4) : 3; }

template <int CPL, int RS, int QPW, bool FUSED>
__global__ __launch_bounds__(kSqThreads) void sq_scan_kernel(SqArgs a) {
  constexpr int QW = (4 / RS) * QPW;
  constexpr int NBUF = sq_nbuf<CPL, RS>();
  constexpr int CHB = 4096 * CPL;  // bytes of one ring chunk (16 rows of up to 64·CPL floats)
  extern __shared__ __attribute__((aligned(16))) char sq_smem[];
  __shared__ uint32_t last_flag;
  const int B = a.B;
  const int ldx = (int)a.ldx, nch = ldx >> 2;
  char* ring = sq_smem;
  float* qs = (float*)(sq_smem + NBUF * CHB);         // [B][ldx] f32 query rows
  uint32_t* sel = (uint32_t*)(qs + B * ldx);          // [B][rpw] raw order images
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int p = lane & 15, g = lane >> 4;
  const int rs = g % RS, qsub = g / RS;
  const int nqg = (B + QW - 1) / QW;
  const int qg = w % nqg, ph = w / nqg, nph = kSqWaves / nqg;
  const int blk = blockIdx.x;
  const int r0 = blk * a.rpw, r1 = min(a.n, r0 + a.rpw), nr = r1 - r0;
  const int nck = (nr + 15) >> 4;
  const char* Xb = (const char*)a.X + (size_t)r0 * ldx * 4;   // the block
  const int blk_bytes = nr * ldx * 4;
  const uint32_t ring_lds = (uint32_t)(size_t)((__attribute__((address_space(3))) char*)ring);
  auto stage = [&](int c) __attribute__((always_inline)) {
    const uint32_t dst0 = ring_lds + (uint32_t)((c % NBUF) * CHB);
#pragma unroll
    for (int i = 0; i < CPL; ++i) {
      const int piece = w + 4 * i;
      const int off = c * 64 * ldx + piece * 1024 + lane * 16;   // byte offset in the block
      glds16(Xb + (off < blk_bytes ? off : 0), __builtin_amdgcn_readfirstlane(dst0 + piece * 1024));
    }
  };
#pragma unroll
  for (int c = 0; c < NBUF - 1; ++c)
    if (c < nck) stage(c);

  // query rows, as prep_kernel writes its f32 operand: normalised raw rows (qnorm.h), the
  // stored rows of item ids, or CF rows as they are; zero past the row
  for (int b = w; b < B; b += kSqWaves) {
    float* qrow = qs + b * ldx;
    if (a.q_kind == 1) {  // (all loads of the row in flight together, as load_chunk)
      const int64_t id = a.q_ids[b] - a.q_id_offset;
      const bool ok = id >= 0 && id < a.n;
      const float* src = a.X + (size_t)(ok ? id : 0) * ldx;
      float v[kQnC];
#pragma unroll
      for (int c = 0; c < kQnC; ++c) v[c] = src[min(lane + 64 * c, ldx - 1)];
#pragma unroll
      for (int c = 0; c < kQnC; ++c)
        if (lane + 64 * c < ldx) qrow[lane + 64 * c] = ok ? v[c] : 0.f;
    } else {
      double xq[kQnC];
      load_chunk<kQnC>(a.q_src, a.q_dtype, (size_t)b * a.q_ld, 0, a.q_d, lane, xq);
      const double nrm = a.q_kind == 0 ? qn_norm(xq) : 1.0;
#pragma unroll
      for (int c = 0; c < kQnC; ++c) {
        const int i = lane + 64 * c;
        if (i < ldx) qrow[i] = qn_elem(xq[c], nrm);
      }
    }
  }
  __syncthreads();  // (its vmcnt(0) also lands the prologue's chunks)
  double qd[QPW][CPL][4];
  int qb[QPW];
#pragma unroll
  for (int i = 0; i < QPW; ++i) {
    qb[i] = qg * QW + qsub * QPW + i;
#pragma unroll
    for (int j = 0; j < CPL; ++j) {
      const int c = p + 16 * j;
      const f4v v = (qb[i] < B && c < nch) ? lds_f4(qs + qb[i] * ldx, c) : f4v{0.f, 0.f, 0.f, 0.f};
      qd[i][j][0] = (double)v.x;
      qd[i][j][1] = (double)v.y;
      qd[i][j][2] = (double)v.z;
      qd[i][j][3] = (double)v.w;
    }
  }

  for (int c = 0; c < nck; ++c) {
    // this wave's pieces of chunk c landed (later chunks may stay in flight), then every wave's
    const int ahead = min(nck - 1 - c, NBUF - 2);
    if (ahead <= 0) wait_barrier<0>();
    else if (ahead == 1) wait_barrier<CPL>();
    else if (ahead == 2) wait_barrier<2 * CPL>();
    else if (ahead == 3) wait_barrier<3 * CPL>();
    else wait_barrier<4 * CPL>();
    // refill the buffer read in the previous phase (every wave has passed this barrier, its
    // reads consumed)
    if (c + NBUF - 1 < nck) stage(c + NBUF - 1);
    const float* buf = (const float*)(ring + (c % NBUF) * CHB);
    const int rows_c = min(16, nr - 16 * c);
    for (int s0 = ph * RS; s0 < 16; s0 += nph * RS) {  // wave-uniform
      const int ri = s0 + rs;  // row within the chunk
      const float* xr = buf + (ri < rows_c ? ri : 0) * ldx;
      double acc[QPW];
#pragma unroll
      for (int i = 0; i < QPW; ++i) acc[i] = 0.0;
#pragma unroll
      for (int j = 0; j < CPL; ++j) {
        const f4v xv = lds_f4(xr, min(p + 16 * j, nch - 1));
        const double x0 = (double)xv.x, x1 = (double)xv.y, x2 = (double)xv.z, x3 = (double)xv.w;
#pragma unroll
        for (int i = 0; i < QPW; ++i) {
          acc[i] = fma(x0, qd[i][j][0], acc[i]);
          acc[i] = fma(x1, qd[i][j][1], acc[i]);
          acc[i] = fma(x2, qd[i][j][2], acc[i]);
          acc[i] = fma(x3, qd[i][j][3], acc[i]);
        }
      }
#pragma unroll
      for (int i = 0; i < QPW; ++i) acc[i] = sum16_f64(acc[i]);
      if (p == 0 && ri < rows_c) {
#pragma unroll
        for (int i = 0; i < QPW; ++i)
          if (qb[i] < B) sel[qb[i] * a.rpw + 16 * c + ri] = ord_of((float)acc[i] + 0.0f);
      }
    }
  }
  __syncthreads();

  // per query: eligibility, the order images of the rows, the top kSqM keys, the present maximum
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
      if (i < nr) st32<FUSED>(a.ords + (size_t)b * a.ords_ld + row, o[e]);
    }
    uint64_t mine = 0;
#pragma unroll
    for (int t = 0; t < kSqM; ++t) {
      uint64_t best = 0;
#pragma unroll
      for (int e = 0; e < kSqMaxRows / 64; ++e) {
        const uint64_t k = o[e] ? make_key(o[e], a.gid0 + (uint32_t)(r0 + lane + 64 * e)) : 0ull;
        best = best > k ? best : k;
      }
      best = wave_max_u64(best);
#pragma unroll
      for (int e = 0; e < kSqMaxRows / 64; ++e)
        if (o[e] && make_key(o[e], a.gid0 + (uint32_t)(r0 + lane + 64 * e)) == best) o[e] = 0u;
      if (lane == t) mine = best;
    }
    if (lane < kSqM) st64<FUSED>(a.wg_top + ((size_t)b * a.nwg + blk) * kSqM + lane, mine);
    if (a.drop) {
      uint64_t pm = 0;
#pragma unroll
      for (int e = 0; e < kSqMaxRows / 64; ++e) {
        const uint64_t k = op[e] ? make_key(op[e], a.gid0 + (uint32_t)(r0 + lane + 64 * e)) : 0ull;
        pm = pm > k ? pm : k;
      }
      pm = wave_max_u64(pm);
      if (lane == 0) st64<FUSED>(a.wg_pmax + (size_t)b * a.nwg + blk, pm);
    }
  }
  if constexpr (FUSED) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its sc1 stores
    __syncthreads();
    if (tid == 0) {
      const unsigned long long old = __hip_atomic_fetch_add(a.ticket, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      last_flag = (old + 1ull) % (unsigned long long)a.nwg == 0ull ? 1u : 0u;
    }
    __syncthreads();
    if (!last_flag) return;
    uint64_t* cb = (uint64_t*)sq_smem + w * kSqCand;  // the ring is no longer read
    for (int b = w; b < B; b += kSqWaves) sq_merge_wave<true>(a, b, cb);
  }
}

template <int CPL, int RS>
size_t sq_lds_bytes(const SqArgs& a) {
  return (size_t)sq_nbuf<CPL, RS>() * 4096 * CPL + (size_t)a.B * a.ldx * 4 + (size_t)a.B * a.rpw * 4;
}

// Separate merge launch: one wave per query.
__global__ __launch_bounds__(64) void sq_merge_kernel(SqArgs a) {
  __shared__ uint64_t cb[kSqCand];
  if ((int)blockIdx.x < a.B) sq_merge_wave<false>(a, blockIdx.x, cb);
}

template <int CPL, int RS, int QPW, bool FUSED>
hipError_t launch_sq4(const SqArgs& a, hipStream_t s) {
  const size_t lds = sq_lds_bytes<CPL, RS>(a);
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  static bool attr = false;  // (per instantiation; idempotent)
  if (!attr) {
    const hipError_t e = hipFuncSetAttribute((const void*)sq_scan_kernel<CPL, RS, QPW, FUSED>,
                                             hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e != hipSuccess) return e;
    attr = true;
  }
  hipLaunchKernelGGL((sq_scan_kernel<CPL, RS, QPW, FUSED>), dim3(a.nwg), dim3(kSqThreads), lds, s, a);
  return hipGetLastError();
}

template <int CPL, int RS, int QPW>
hipError_t launch_sq3(const SqArgs& a, hipStream_t s) {
  return a.ticket ? launch_sq4<CPL, RS, QPW, true>(a, s) : launch_sq4<CPL, RS, QPW, false>(a, s);
}

template <int CPL>
hipError_t launch_sq2(const SqArgs& a, hipStream_t s) {
  // (RS, QPW) by batch: 4 rows x 1 query, 4 x 2, 2 x 2 (x 2 query sets), 1 x 2 (x 4 sets;
  // two query groups of waves above 8 queries)
  if (a.B == 1) return launch_sq3<CPL, 4, 1>(a, s);
  if (a.B == 2) return launch_sq3<CPL, 4, 2>(a, s);
  if (a.B <= 4) return launch_sq3<CPL, 2, 2>(a, s);
  return launch_sq3<CPL, 1, 2>(a, s);
}

}  // namespace

hipError_t launch_sq_scan(const SqArgs& a, hipStream_t s) {
  const int nch = (int)(a.ldx >> 2);
  if (a.B < 1 || a.B > kSqMaxB || a.ldx > kRrMaxD || (a.ldx & 3) || a.K < 1 || a.K > kSqMaxK || a.rpw < 4 ||
      (a.rpw & 3) || a.rpw > kSqMaxRows || a.nwg < 1 || a.nwg > kSqMaxWg || (int64_t)a.nwg * a.rpw < a.n ||
      (int64_t)(a.nwg - 1) * a.rpw >= a.n || a.n < 1 || a.ords_ld < a.n || !a.present ||
      (a.out_scores ? (!a.out_ids || a.k_final < 1 || a.k_final > a.K) : (!a.keys_out || !a.max_out)))
    return hipErrorInvalidValue;
  const int cpl = (nch + 15) / 16;
  if (cpl <= 1) return launch_sq2<1>(a, s);
  if (cpl <= 2) return launch_sq2<2>(a, s);
  if (cpl <= 4) return launch_sq2<4>(a, s);
  if (cpl <= 6) return launch_sq2<6>(a, s);
  return launch_sq2<8>(a, s);
}

hipError_t launch_sq_merge(const SqArgs& a, hipStream_t s) {
  if (a.B < 1 || a.B > kSqMaxB || a.ticket) return hipErrorInvalidValue;
  hipLaunchKernelGGL(sq_merge_kernel, dim3(a.B), dim3(64), 0, s, a);
  return hipGetLastError();
}

}  // namespace bb
