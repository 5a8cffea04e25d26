// scan4_kernel.h — bf16 query-resident scan with 64 queries per wave (256 per workgroup).
//
// Why: scan2_kernel<bf16> keeps 32 queries per wave (128 per CU), so every 2-byte item
// element staged into LDS feeds 2·128 flops.  At the bf16 MFMA rate (4,096 flop/clk/CU) that
// needs 32 B/clk/CU of L2 -> LDS traffic (≈19.7 TB/s chip-wide), more than LDS-DMA sustains
// (≈17–19 TB/s measured from a shared L2, MI355X_MICROARCH.md "Indexed rows"), and the
// 1M / 10M-row configs ran at 0.20–0.28 of the bf16 peak.  Holding two
// 32-query blocks per wave doubles the reuse of every staged tile: 16 B/clk/CU, half the item
// stream, and twice the MFMA work per barrier.
//
// Registers (one wave per SIMD, 512 per lane): the two query blocks take 8·U registers
// (U = 16-wide k steps; d = 768: 384, d = 384: 192).  The first 256 live in AGPRs, the rest
// in VGPRs; both are legal MFMA B operands on gfx950.  Two schedules:
// * d <= 512 (interleaved, IL): per k-step one fragment read feeds A_u and B_u, two
//   accumulator sets alternate with the tiles, and both blocks' epilogues of tile t-1 are
//   woven into tile t after its DMA pieces.  Half the LDS fragment reads per MFMA: the
//   MFMA + LDS loop runs at 1.52 PF/s against 1.34 for the chained schedule.
// * d = 768 (chained): no registers for a second accumulator set, so ONE accumulator per
//   block and the tile is two accumulation chains, block A then block B, each block's
//   epilogue woven into the OTHER block's chain:
//     chain A of tile t  <- epilogue of block B of tile t-1, eligibility words of tile t+1,
//                           LDS-DMA staging of tile t+1
//     chain B of tile t  <- epilogue of block A of tile t
//   Item fragments are read once per chain (one ds_read_b128 per MFMA).
// Measurements: tools/scan4_probe.hip, profiles/r01*_scan4_probe.jsonl.
//
// Same contract as scan2_kernel.h — LDS tile layout (XOR swizzle), XCD-aware blockIdx ->
// (query group, item chunk) mapping, tile maxima for the slab select — except that scores
// go out as scan3's blocked image (sblk_quad: every store a full 1-KiB wave write), or the
// streaming epilogue (kScanStream) appending candidates to per-lane regions
// ((q·n_chunks + chunk)·2 + h, one region set per query as before).
#pragma once
#include "list_epi.h"
#include "scan2_kernel.h"

namespace bb {

constexpr int kScan4Queries = kScanWaves * 64;  // queries per workgroup
#ifndef BB_SCAN4_PF
#define BB_SCAN4_PF 4
#endif
constexpr int kScan4Pf = BB_SCAN4_PF;  // interleaved schedule: LDS fragment prefetch distance (k-steps)
#ifndef BB_SCAN4_CHAIN_PF
#define BB_SCAN4_CHAIN_PF 2
#endif
constexpr int kScan4ChainPf = BB_SCAN4_CHAIN_PF;  // chained (d = 768) schedule: the same, in MFMA steps

// Item chunks of a scan4 launch: ~256 workgroups (one per CU).
inline int scan4_n_chunks(int Mpad, int tiles) {
  const int n_groups = Mpad / kScan4Queries;
  const int n_chunks = (256 + n_groups - 1) / n_groups;
  return n_chunks < tiles ? n_chunks : tiles;
}

// Item chunks of a list scan (kScanList) of rows KU 16-B chunks wide.  Narrow rows (KU <= 16:
// the r <= 128 CF factors of a hybrid search) are bound by the list epilogue's VALU, not the
// MFMA, at one wave per SIMD (configs[2]: the r = 50 scan 22 us beside 33 us for the d = 384
// content side with six times its MFMA work); their kernel fits two workgroups per CU, so
// they get twice the chunks (512 workgroups) to fill them.
inline int scan4_list_chunks(int Mpad, int tiles, int ku) {
  if (ku > 16) return scan4_n_chunks(Mpad, tiles);
  const int n_groups = Mpad / kScan4Queries;
  const int n_chunks = (512 + n_groups - 1) / n_groups;
  return n_chunks < tiles ? n_chunks : tiles;
}

// Streaming state of one query (scan2's StreamLane without the region pointer, which is
// recomputed on the rare append: at d = 768 every VGPR counts).
struct Stream4 {
  uint32_t thr = 0xFFFFFFFFu;
  float thrf = __builtin_inff();  // the bound as a float: x >= thrf <=> ord(x) >= thr (±0 aside)
  uint32_t n = 0;
  uint32_t rp = 0;
  uint64_t rkey = 0;
};

// Appends of one half tile.  hits: bit g = accumulator register g is eligible and reaches the
// bound (built branch-free in the woven slices).  The wave parks its 16 registers in LDS
// (4 conflict-free 1-KiB writes) and each lane reads back the register of its next hit —
// a per-lane dynamic index into registers would compile to long compare/select chains,
// and per-register branches stall the MFMA stream (measured: either took the 1M-row stream
// pass from 6.1 to ~10-11 ms).  One store per hit; the loop runs as often as the busiest
// lane has hits (usually once).  A full region keeps counting (cand_select reports the
// overflow) and its last slot absorbs the extra stores.
template <int ABL>
__device__ __forceinline__ void s4_flush(const GemmArgs& a, const f32x16s& p, int tile0, int h, uint32_t hits,
                                         Stream4& s, size_t region, float* park) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int j = 0; j < 4; ++j) *(float4*)(park + j * 256 + lane * 4) = make_float4(p[4 * j], p[4 * j + 1], p[4 * j + 2], p[4 * j + 3]);
  uint64_t* reg = a.cand + region * (size_t)a.cand_cap;
  const uint32_t last = (uint32_t)a.cand_cap - 1u;
  while (__any(hits != 0u)) {
    if (hits) {
      const uint32_t g = (uint32_t)__builtin_ctz(hits);
      hits &= hits - 1u;
      const float v = park[(g >> 2) * 256 + lane * 4 + (g & 3u)];
      const uint32_t it = (g & 3u) + 8u * (g >> 2) + 4u * (uint32_t)h;
      const uint64_t key = make_key(ord_of(v), a.gid0 + (uint32_t)tile0 + it);
      if constexpr (ABL & 64)
        s.rkey ^= key;  // probe: everything but the store
      else
        reg[s.n < last ? s.n : last] = key;
      ++s.n;
    }
  }
}

// This lane's eligible registers of a half tile as a 16-bit mask (bit g = register g):
// in range and set in ok = present ∧ mask ∧ ¬excl.
__device__ __forceinline__ uint32_t s4_elig16(uint32_t ok, int tile0, int n_valid, int h) {
  const int rem = n_valid - tile0;
  const uint32_t inr = rem >= 32 ? 0xFFFFFFFFu : rem <= 0 ? 0u : ((1u << rem) - 1u);
  const uint32_t w = (ok & inr) >> (4 * h);  // register g <-> item (g & 3) + 8 (g >> 2) + 4h
  return (w & 0xFu) | ((w >> 4) & 0xF0u) | ((w >> 8) & 0xF00u) | ((w >> 12) & 0xF000u);
}

// rank 0: as stream_rank0 (scan2_kernel.h)
__device__ __forceinline__ void s4_rank0(const GemmArgs& a, const f32x16s& p, int tile0, uint32_t pw, int h,
                                         uint32_t tp, Stream4& s) {
  if (!__any(tp > s.rp)) return;
  if (tp > s.rp) {
    const float mv = float_of_ord(tp);
    bool found = false;
#pragma unroll
    for (int g = 0; g < 16; ++g) {
      const int it = (g & 3) + 8 * (g >> 2) + 4 * h;
      if (!found && tile0 + it < a.n_valid && ((pw >> it) & 1u) && p[g] == mv) {
        s.rkey = make_key(ord_of(p[g]), a.gid0 + (uint32_t)(tile0 + it));
        found = true;
      }
    }
    s.rp = tp;
  }
}

// u-step of a chain on which woven slice s is issued
constexpr int scan4_at(int s, int U) { return (s + 2 < U) ? s + 2 : U - 1; }
// chain A: block B's epilogue (slices 0..E-1 from u = 2, after the accumulator tie), the
// next tile's words (slice E), then the LDS-DMA pieces spaced SP u-steps apart (slices
// E+1..): each DMA holds the wave's issue for ~20+ cycles; spread out rather than back to
// back they cost 2-3 % less.  With their source offsets precomputed (no VALU per piece),
// staging costs ~5 % of the d = 768 no-store scan (tools/scan4_probe: no_staging vs
// no_stores); splitting them over both chains measured 4 % slower.
constexpr int scan4_atA(int s, int U, int E, int pieces) {
  const int sp = (U - (E + 3)) / (pieces > 0 ? pieces : 1) > 1 ? (U - (E + 3)) / pieces : 1;
  const int u = s < E ? s + 2 : s == E ? E + 2 : E + 3 + (s - E - 1) * sp;
  return u < U ? u : U - 1;
}

// ABL (tools/scan4_probe only): 1 = no epilogue, 2 = no staging after the first tile, 4 = no
// per-tile wait + barrier, 8 = no S stores, 16 = no tile-maxima stores, 32 = no streaming
// appends (compares only), 64 = streaming appends without their stores, 128 = a three-deep
// ring on the chained schedule, 256 = (with 65536) the streaming compare slices without
// their uniform branch (measured: 4 % slower without hits, 2-5 % faster at a 0.2 % hit rate), 1024 = the chained schedule at d <= 512, 2048 = no query
// loads (zero operand), 65536 = the streaming compares and appends woven over slices 1-5 (the
// round-4 placement) instead of under slice 0's one branch.
template <int KU, int ABL = 0, bool PM = false>
__device__ __forceinline__ void scan4_body(const GemmArgs& a, int n_chunks, int tiles_total, int L) {
  typedef uint16_t T;
  constexpr int U = KU / 2;        // u-steps (one bf16 MFMA each) per tile and block
  constexpr int ROWB = KU * 16;
  constexpr int TILE_B = 32 * ROWB;
  constexpr int G = (KU % 16 == 0) ? 8 : 4;
  constexpr int PIECES = KU / 8;   // 1 KiB LDS-DMA pieces per wave per tile
  constexpr int NA = 64;           // query registers (u32x4) that live in AGPRs
  // interleaved schedule (both blocks per fragment read, two accumulator sets) where the
  // registers allow it: all queries in AGPRs (d <= 512); ABL 1024 (probe) forces the chains
  constexpr bool IL = KU <= 64 && !(ABL & 1024);
  static_assert(ROWB <= kScanRowMax, "row too wide for the scan kernel");
  static_assert(KU % 8 == 0, "KU must split into whole 1 KiB pieces per wave");
  constexpr bool STREAM = (ABL & kScanStream) != 0;
  constexpr bool F16 = (ABL & kScanF16) != 0;  // f16 operands: the re-rank copy of an f32 index
  // item tile ring — three tiles deep on the interleaved schedule (two tiles of LDS-DMA in flight
  // while one is read: the ring the MALL / L2 latency needs at one workgroup per CU), two on the
  // chained d = 768 one — + (streaming) a 4-KiB register parking area per wave.  ABL 128
  // (probe): three on the chained one too (three 48-KiB tiles + the park = all 160 KiB) —
  // measured equal (tools/scan4_probe: the chained loop is bound by LDS bandwidth, not latency)
  constexpr int kParkB = STREAM ? kScanWaves * 4096 : 0;
  constexpr int RING = (IL || (ABL & 128)) ? 3 : 2;
  static_assert(RING * TILE_B + kParkB <= 163840, "LDS ring + park exceed 160 KiB");
  __shared__ __attribute__((aligned(256))) char smem[RING * TILE_B + kParkB];

  const int n_groups = a.Mpad / kScan4Queries;
  const int total = n_groups * n_chunks;
  const int xcd = L & 7, local = L >> 3, q8 = total >> 3, r8 = total & 7;
  const int t = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + local;
  const int chunk = t / n_groups, group = t - chunk * n_groups;
  const int tile_lo = (int)((int64_t)chunk * tiles_total / n_chunks);
  const int tile_hi = (int)((int64_t)(chunk + 1) * tiles_total / n_chunks);

  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 31, h = lane >> 5;
  const int qA = group * kScan4Queries + wave * 64 + r, qB = qA + 32;
  if (tile_lo >= tile_hi) return;  // uniform per workgroup
  // BB_SCAN_TRACE probe runs (a.trace): s_memrealtime stamps, 8 words per workgroup — start,
  // query prologue done, first tile, fifth tile, loop done, end; word 6 = tiles
  auto stamp = [&](int slot) __attribute__((always_inline)) {
    if (a.trace && tid == 0) a.trace[(size_t)L * 8 + slot] = __builtin_amdgcn_s_memrealtime();
  };
  const uint64_t clk0 = a.trace ? __builtin_amdgcn_s_memtime() : 0;  // shader clock (word 7: cycles)
  stamp(0);

  // LDS fragment addresses (scan2 layout: chunk (2u + h) ^ swz(r) of row r): per-lane chunk
  // offsets in registers on the interleaved schedule, one v_xor per read on the chained
  // d = 768 one (whose two query blocks leave 128 VGPRs for everything else); the LDS-DMA
  // source offsets are precomputed on both (below)
  const int swz = scan_swz<KU>(r);
  const int rrow = r * ROWB;
  const char* Xg = (const char*)a.X;
  const size_t ldxb = (size_t)a.ldx * sizeof(T);
  // LDS-DMA source offset of this lane's 16 B in piece p, relative to the tile's first row
  // (launch_scan4 guarantees ldx < 2^23, so it fits 32 bits and every product is 24-bit):
  // chunk c of the tile image -> row c / KU by multiply-shift (exact for c < 32·KU), chunk
  // (c mod KU) ^ swz(row).  ~7 full-rate VALU; the tile base rides in SGPRs (saddr form), so
  // no 64-bit address math per piece (the signed 64-bit form cost ~28 issue slots a piece,
  // ~20 % of the d = 768 scan)
  static_assert(32 * KU * KU < (1 << 20), "row = c * kDivM >> 20 exact for c < 32 KU");
  constexpr uint32_t kDivM = ((1u << 20) + KU - 1) / KU;
  const uint32_t ldxb32 = (uint32_t)ldxb;
  auto soff = [&](int p) __attribute__((always_inline)) {
    uint32_t ln = lane;
    asm volatile("" : "+v"(ln));  // opaque per use: no hoisted per-piece registers
    const uint32_t c = (uint32_t)(wave * PIECES + p) * 64u + ln;
    const uint32_t row = __umul24(c, kDivM) >> 20;
    uint32_t cin;  // c - row·KU as one full-rate 24-bit mad (the compiler picks a 64-bit one)
    asm("v_mad_i32_i24 %0, %1, %2, %3" : "=v"(cin) : "v"(row), "s"(-KU), "v"(c));
    const uint32_t ch = cin ^ (uint32_t)scan_swz<KU>((int)row);
    return __umul24(row, ldxb32) + (ch << 4);
  };
  const uint32_t lds_base = (uint32_t)(size_t)((__attribute__((address_space(3))) char*)smem);
  // interleaved schedule (d <= 512): the query operand leaves registers for the per-piece
  // source offsets — precomputed once (the list epilogue there is VALU-bound)
  // (the chained d = 768 schedule too, since its stream epilogue stopped holding sixteen mask
  // constants in VGPRs: 7 VALU less per piece in the MFMA gaps, 12 pieces a tile)
  constexpr bool kSoffR = true;
  uint32_t soffr[kSoffR ? PIECES : 1];
  if constexpr (kSoffR) {
#pragma unroll
    for (int p = 0; p < PIECES; ++p) soffr[p] = soff(p);
  }
  // inline asm, as in scan2: the compiler's waitcnt pass must not wait for these
  auto stage_piece = [&](int tile, int buf, int p) __attribute__((always_inline)) {
    uint32_t so;
    if constexpr (kSoffR) so = soffr[p];
    else so = soff(p);
    const uint64_t tb = (uint64_t)(size_t)(Xg + (size_t)tile * 32 * ldxb);
    // (readfirstlane returns int: widen through uint32_t, or the low word sign-extends)
    const uint32_t tlo = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)tb);
    const uint32_t thi = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(tb >> 32));
    const char* src = (const char*)(size_t)(((uint64_t)thi << 32) | (uint64_t)tlo);
    const uint32_t dst = __builtin_amdgcn_readfirstlane(lds_base + buf * TILE_B + (wave * PIECES + p) * 1024);
    asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2" ::"s"(dst), "v"(so), "s"(src)
                 : "memory");
  };

  // first tile(s) in flight before the query loads
#pragma unroll
  for (int p = 0; p < PIECES; ++p) stage_piece(tile_lo, 0, p);
  if constexpr (RING == 3) {
    const int t1 = tile_lo + 1 < tile_hi ? tile_lo + 1 : tile_lo;  // branch-free staging target
#pragma unroll
    for (int p = 0; p < PIECES; ++p) stage_piece(t1, 1, p);
  }

  // The prologue's other loads go out with the first tiles, ahead of the query operand — the
  // code quanta, the streaming bounds and the first tile's eligibility words — so the whole
  // prologue is the operand's round trips, not one more after them (the operand's pinning
  // waits retire these too: loads complete in order).
  constexpr bool S16 = (ABL & kScanS16) != 0 && !STREAM;
  constexpr bool LIST = (ABL & kScanList) != 0 && !STREAM && !S16;
  float hsA = 0.f, hsB = 0.f;
  if constexpr (S16 || LIST) {
    hsA = qA < a.M_valid ? a.s_h[qA] : 0.f;
    hsB = qB < a.M_valid ? a.s_h[qB] : 0.f;
  }
  uint64_t tkA = 0ull, tkB = 0ull;
  if constexpr (STREAM) {
    if (qA < a.M_valid) tkA = a.thr_keys[(size_t)qA * a.thr_ld + a.thr_ld - 1];
    if (qB < a.M_valid) tkB = a.thr_keys[(size_t)qB * a.thr_ld + a.thr_ld - 1];
  }
  const size_t w0 = (size_t)(a.slab_start >> 5);
  const uint32_t* erowA = a.excl + (size_t)(qA < a.M_valid ? qA : a.M_valid - 1) * a.excl_ld;
  const uint32_t* erowB = a.excl + (size_t)(qB < a.M_valid ? qB : a.M_valid - 1) * a.excl_ld;
  // eligibility words of the current tile (pw, mw, ewA, ewB) and of the previous tile for
  // block B's deferred epilogue (ppw, pmw, pewB)
  uint32_t pw = a.present[w0 + tile_lo], mw = a.mask[w0 + tile_lo], ewA = erowA[w0 + tile_lo],
           ewB = erowB[w0 + tile_lo];

  // queries: block A (qA), block B (qB); register j = b·U + u lives in an AGPR iff j < NA
  u32x4v qv[2 * U];
  {
    const char* rowp[2];
    bool ok[2];
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      const int q = b ? qB : qA;
      ok[b] = q < a.M_valid;
      if (a.q_ids) {  // similar / hybrid: the stored (normalised, padded) item row of the liked set
        const int64_t lid = ok[b] ? a.q_ids[q] - a.q_id_offset : 0;
        ok[b] = ok[b] && lid >= 0 && lid < a.q_n_items;
        rowp[b] = (const char*)a.q_items_base + (size_t)(ok[b] ? lid : 0) * a.ldx * sizeof(T);
      } else {
        rowp[b] = (const char*)a.Q + (size_t)(ok[b] ? q : 0) * a.ldq * sizeof(T);
      }
    }
    // lane-order operand (q_perm, prep wrote every row up to Mpad): 1 KiB per wave load.
    // Loads go out in batches of kQB plain loads before the batch's AGPR pinning: with the
    // pinning asm between consecutive loads the compiler waited for each load on its own
    // (one L2 round trip per query register).  (Inline-asm loads with a separate wait are
    // NOT safe here: the compiler may copy or reuse a destination register before the wait.)
    const uint4* qp = (const uint4*)a.Q + ((size_t)(group * 4 + wave) * (2 * U)) * 64 + lane;
    constexpr int kQB = 16;
#pragma unroll
    for (int j0 = 0; j0 < 2 * U; j0 += kQB) {
      uint4 t[kQB];
#pragma unroll
      for (int jj = 0; jj < kQB; ++jj) {
        const int j = j0 + jj, b = j / U, u = j % U;
        if (j >= 2 * U) continue;
        t[jj] = (ABL & 2048) ? make_uint4(0u, 0u, 0u, 0u)
                : a.q_perm   ? qp[(size_t)j * 64]
                             : *(const uint4*)(rowp[b] + (2 * u + h) * 16);
      }
#pragma unroll
      for (int jj = 0; jj < kQB; ++jj) {
        const int j = j0 + jj, b = j / U;
        if (j >= 2 * U) continue;
        qv[j] = ok[b] || a.q_perm ? __builtin_bit_cast(u32x4v, t[jj]) : u32x4v{0, 0, 0, 0};
        if (j < NA)
          asm volatile("" : "+a"(qv[j]));
        else
          asm volatile("" : "+v"(qv[j]));
      }
    }
  }

  float* park = (float*)(smem + RING * TILE_B) + wave * 1024;
  // int16 score image (kScanS16): code scales 1/(h·32767) of the two query blocks
  float skA = 0.f, skB = 0.f;
  if constexpr (S16) {
    const float hA = hsA, hB = hsB;
    skA = hA > 0.f ? 1.0f / (hA * 32767.f) : 0.f;
    skB = hB > 0.f ? 1.0f / (hB * 32767.f) : 0.f;
  }
  // bounded candidate lists (kScanList, list_epi.h; interleaved schedule only): per block the
  // code scale 1/(65535·h), the lane's top-5 of the current period and the rank-0 top-2.  A
  // finished period's lists are packed and stored at the start of the NEXT tile body, ahead
  // of its DMA pieces, so the end-of-tile vmcnt wait never waits for a store's round trip.
  static_assert(!LIST || IL, "list epilogue: interleaved schedule (rows up to 512 wide) only");
  float k2A = 0.f, k2B = 0.f;
  if constexpr (LIST) {
    const float hA = hsA, hB = hsB;
    k2A = hA > 0.f ? 1.0f / (hA * 65535.f) : 0.f;
    k2B = hB > 0.f ? 1.0f / (hB * 65535.f) : 0.f;
  }
  ListTop5 lstA, lstB;
  ListTop2 r0A, r0B;
  uint4 pendA = make_uint4(0u, 0u, 0u, 0u), pendB = make_uint4(0u, 0u, 0u, 0u);
  bool pend = false;
  int l_cnt = 0, l_period = 0, pend_period = 0;
  const int l_nb = a.Mpad >> 5;
  const bool liveA = __any(qA < a.M_valid), liveB = __any(qB < a.M_valid);  // padded blocks store nothing
  auto list_put = [&](int period, const uint4& vA, const uint4& vB) __attribute__((always_inline)) {
    if (liveA) *(uint4*)(a.lists + 4 * list_slot(chunk, period, a.l_np, l_nb, qA >> 5, lane)) = vA;
    if (liveB) *(uint4*)(a.lists + 4 * list_slot(chunk, period, a.l_np, l_nb, qB >> 5, lane)) = vB;
  };
  // streaming pilot (kScanPilot): per block the lane's top-PM eligible half-tile maxima
  constexpr bool PILOT = (ABL & kScanPilot) != 0 && !STREAM && !S16 && !LIST;
  constexpr int kPM = IL ? 8 : 4;  // (the chained d = 768 schedule has no registers for more)
  uint32_t pmA[kPM], pmB[kPM];
#pragma unroll
  for (int i = 0; i < kPM; ++i) pmA[i] = pmB[i] = 0u;
  auto pm_ins = [&](uint32_t (&t)[kPM], uint32_t v) __attribute__((always_inline)) {
    uint32_t n[kPM];
    n[0] = maxu(t[0], v);
#pragma unroll
    for (int i = 1; i < kPM; ++i) n[i] = med3u(t[i - 1], t[i], v);
#pragma unroll
    for (int i = 0; i < kPM; ++i) t[i] = n[i];
  };
  auto pm_store = [&]() __attribute__((always_inline)) {
    const int nbq = a.Mpad >> 5;
    uint32_t* oA = a.pilot_top + ((size_t)(chunk * nbq + (qA >> 5)) * 64 + lane) * kPM;
    uint32_t* oB = a.pilot_top + ((size_t)(chunk * nbq + (qB >> 5)) * 64 + lane) * kPM;
#pragma unroll
    for (int i = 0; i < kPM; i += 4) {
      *(uint4*)(oA + i) = make_uint4(pmA[i], pmA[i + 1], pmA[i + 2], pmA[i + 3]);
      *(uint4*)(oB + i) = make_uint4(pmB[i], pmB[i + 1], pmB[i + 2], pmB[i + 3]);
    }
  };
  Stream4 slA, slB;
  auto region = [&](int q) __attribute__((always_inline)) { return ((size_t)q * n_chunks + chunk) * 2 + h; };
  if constexpr (STREAM) {  // bound = the last key of the query's pilot list (stream_begin)
    // (an image at or below ord(-inf) takes every finite score: thrf = -inf)
    if (qA < a.M_valid) {
      const uint32_t o = ordk_of(tkA);
      slA.thr = o ? o : 1u;
      slA.thrf = slA.thr <= 0x007FFFFFu ? -__builtin_inff() : float_of_ord(slA.thr);
    }
    if (qB < a.M_valid) {
      const uint32_t o = ordk_of(tkB);
      slB.thr = o ? o : 1u;
      slB.thrf = slB.thr <= 0x007FFFFFu ? -__builtin_inff() : float_of_ord(slB.thr);
    }
  }
  uint32_t ppw = 0, pmw = 0, pewB = 0, nw_p = 0, nw_m = 0, nw_eA = 0, nw_eB = 0;

  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  stamp(1);
  // consume every plain load now (no LDS-DMA outstanding): the compiler's own waits for
  // them would otherwise land behind later staging and wait for it
  asm volatile("" : "+v"(pw), "+v"(mw), "+v"(ewA), "+v"(ewB));
  if constexpr (STREAM) asm volatile("" : "+v"(slA.thr), "+v"(slB.thr), "+v"(slA.thrf), "+v"(slB.thrf));
  if constexpr (S16) asm volatile("" : "+v"(skA), "+v"(skB));
  if constexpr (LIST) asm volatile("" : "+v"(k2A), "+v"(k2B));
  asm volatile("s_nop 4");

  f32x16s accA = {}, accB = {};

  // Epilogue of one block's tile, as kEpi small slices woven into the other block's chain
  // (each a few instructions, so none outgrows an MFMA issue gap):
  //   0      tile maxima (eligible te, present tp) of this lane's half tile
  //   slab:  1 cross-half combine, 2..5 the accumulator as four full 1-KiB stores of the
  //          blocked score image (sblk_quad), 6 the tile-maxima word
  //   stream: 0 also the wave-uniform "some lane's maximum reaches its bound" flag and the
  //          lane's 16-bit eligibility; 1..4 compare 4 registers each against the bound
  //          (branch-free); 5 the appends (s4_flush); 6 rank 0.
  //   ep: low 16 bits eligibility, high 16 bits registers at or above the bound.
  auto epi_slice = [&](auto SS, const f32x16s& p, int ptile, uint32_t epw, uint32_t emw, uint32_t eew, int q,
                       Stream4& sl, uint32_t& te, uint32_t& tp, uint32_t& ep, bool& any) __attribute__((always_inline)) {
    constexpr int s = decltype(SS)::value;
    const int ptile0 = ptile * 32;
    if constexpr (ABL & 1) return;
    if constexpr (s == 0) {
      const uint32_t ok = epw & emw & ~eew;
      tile_maxima(p, ptile0, a.n_valid, epw, ok, h, te, tp);
      if constexpr (STREAM) {
        any = __any(te >= sl.thr);
        if constexpr (ABL & 65536) {
          if (any) ep = s4_elig16(ok, ptile0, a.n_valid, h);  // (read by the woven compare / append slices)
        } else if (any || a.cand_pmax) {
          // (and rank 0, slice 6 of the weave: a tile without hits in a search without a rank-0
          // drop — semantic, CF — passes ONE branch)
          if (a.cand_pmax) s4_rank0(a, p, ptile0, epw, h, tp, sl);
          if (any) {
            // the eligibility, the compares and the appends under ONE uniform branch: a tile
            // without hits (most of them) pays one branch per block instead of five (~22 cycles
            // each, 12 % of the d = 384 streaming scan, tools/scan4_probe cfg 3); the hit
            // bits from inline constants, four at a time (selects of 1 << (16 + g) made the
            // compiler hold sixteen constants in VGPRs for the whole loop)
            ep = s4_elig16(ok, ptile0, a.n_valid, h);
#pragma unroll
            for (int g0 = 0; g0 < 16; g0 += 4) {
              uint32_t m = 0;
#pragma unroll
              for (int gg = 0; gg < 4; ++gg) m |= p[g0 + gg] >= sl.thrf ? 1u << gg : 0u;
              asm volatile("" : "+v"(m));  // (keeps the shift out of the select constants)
              ep |= m << (16 + g0);
            }
            if constexpr (!(ABL & 32)) s4_flush<ABL>(a, p, ptile0, h, (ep >> 16) & ep, sl, region(q), park);
          }
        }
      }
      if constexpr (PILOT) {
        if (q == qA) pm_ins(pmA, te);
        else pm_ins(pmB, te);
      }
    } else if constexpr (PILOT) {
      // (no score image, no maxima rows: the lane's top-PM list is the pilot's output)
    } else if constexpr (STREAM) {
      // ABL 65536 (probe): the round-4 weave — compares in slices 1-4, appends in slice 5,
      // each under its own branch; by default they run in slice 0 (above)
      if constexpr (s <= 4) {
        if constexpr (!(ABL & 65536)) return;
        // (ABL 256, probe: the compares without the uniform branch)
        if ((ABL & 256) || any) {
          // four bits from inline constants (1, 2, 4, 8), shifted once: selects of 1 << (16 + g)
          // made the compiler hold sixteen constants in VGPRs for the whole loop
          constexpr int g0 = 4 * (s - 1);
          uint32_t m = 0;
#pragma unroll
          for (int gg = 0; gg < 4; ++gg) m |= p[g0 + gg] >= sl.thrf ? 1u << gg : 0u;
          asm volatile("" : "+v"(m));  // (keeps the shift out of the select constants)
          ep |= m << (16 + g0);
        }
      } else if constexpr (s == 5) {
        if constexpr ((ABL & 65536) && !(ABL & 32))
          if (any) s4_flush<ABL>(a, p, ptile0, h, (ep >> 16) & ep, sl, region(q), park);
      } else if constexpr (s == 6) {
        if constexpr (ABL & 65536)
          if (a.cand_pmax) s4_rank0(a, p, ptile0, epw, h, tp, sl);
      }
    } else {
      if constexpr (s == 1) {
        const uint32_t te2 = xor32(te), tp2 = xor32(tp);
        te = te2 > te ? te2 : te;
        tp = tp2 > tp ? tp2 : tp;
      } else if constexpr (s <= 5) {
        if constexpr (!(ABL & 8)) {
          constexpr int j = s - 2;
          const size_t e = sblk_lane(q, h, a.ldt) + (size_t)(ptile * 4 + j) * 256;
          if constexpr (S16) {
            const float sk = q == qA ? skA : skB;
            *(uint2*)((int16_t*)a.S + e) =
                make_uint2(s16_pack(p[4 * j], p[4 * j + 1], sk), s16_pack(p[4 * j + 2], p[4 * j + 3], sk));
          } else {
            *(float4*)(a.S + e) = make_float4(p[4 * j], p[4 * j + 1], p[4 * j + 2], p[4 * j + 3]);
          }
        }
      } else if constexpr (s == 6) {
        if constexpr (!(ABL & 16)) if (PM || !h || a.pmax) (h ? a.pmax : a.tmax)[(size_t)q * a.ldt + ptile] = h ? tp : te;
      }
    }
  };
  constexpr int kEpi = 7;
  // List epilogue of one block's tile (kLE slices): 0 eligibility, 1..16 the eight register
  // pairs (codes + masked keys + two top-5 inserts, one insert per slice), 17 rank 0.
  constexpr int kLE = 18;
  auto list_slice = [&](auto SS, const f32x16s& p, int ptile, uint32_t epw, uint32_t emw, uint32_t eew, float k2,
                        ListTop5& L, ListTop2& R, uint32_t& e16, bool& full, uint32_t& kodd) __attribute__((always_inline)) {
    constexpr int s = decltype(SS)::value;
    const int ptile0 = ptile * 32;
    if constexpr (ABL & 1) return;  // (probe: no epilogue)
    if constexpr (s == 0) {
      e16 = list_elig16(epw & emw & ~eew, ptile0, a.n_valid, h);
      full = __all(e16 == 0xFFFFu);
    } else if constexpr (s <= 16) {
      constexpr int pp = (s - 1) >> 1;
      if constexpr (((s - 1) & 1) == 0) {
        uint32_t w = list_codes(p[2 * pp], p[2 * pp + 1], k2);
        if (!full) {
          const uint32_t lo = 0u - ((e16 >> (2 * pp)) & 1u), hi = 0u - ((e16 >> (2 * pp + 1)) & 1u);
          w &= (lo & 0xFFFFu) | (hi & 0xFFFF0000u);
        }
        const uint32_t ix = list_pb2(l_cnt) + list_pair_pos(pp);
        L.ins(__builtin_amdgcn_perm(w, ix, 0x05040100u));
        kodd = __builtin_amdgcn_perm(w, ix, 0x07060302u);
      } else {
        L.ins(kodd);
      }
    } else if constexpr (s == 17) {
      if (a.r0lists) {
        const float m = list_present_max(p, list_elig16(epw, ptile0, a.n_valid, h));
        R.ins(list_r0_key(m, k2, (uint32_t)(ptile - tile_lo)));
      }
    }
  };
  uint32_t le16A = 0, le16B = 0, lkoA = 0, lkoB = 0;
  bool lfullA = true, lfullB = true;
  // slice placement inside a chain: epilogue slices from u = 2 (after the tie of the other
  // accumulator), then (chain A) the next tile's words and staging pieces
  constexpr int kSlicesA = PIECES + 1 + kEpi;
  // End of a tile: wait for the LDS-DMA of the next tile, not for block A's score-image
  // stores issued after it (vmcnt counts loads, stores and LDS-DMA together, in order).
  constexpr bool kStores = !STREAM && !LIST && !PILOT && !(ABL & (1 | 8));

  // One tile: chain A over buffer BUF (+ block B's epilogue of tile-1 when EPIB), chain B
  // (+ block A's epilogue of this tile).
  // The LDS ring slot of the tile is a runtime value (one tile body, not one per slot): the
  // slot's row base goes in one register per tile, the chunk offset is recomputed per use.
  // Staging runs RING - 1 tiles ahead, into the slot tile - 1 read (free since its barrier).
  auto tile_body = [&](auto EPIB, int tile, int slot) __attribute__((always_inline)) {
    constexpr bool epib = decltype(EPIB)::value;
    const int stile = tile + RING - 1 < tile_hi ? tile + RING - 1 : tile;  // branch-free staging target
    const int sslot = RING == 3 ? (slot == 0 ? 2 : slot - 1) : slot ^ 1;
    const int wtile = tile + 1 < tile_hi ? tile + 1 : tile;  // words of the next tile
    const char* fb = smem + slot * TILE_B + rrow;
    // Fragment u: chunk (2g + h) ^ swz of this lane's row, g = u % G, k-group u / G.  With rows
    // and slots whole multiples of 256 B (the LDS array starts 256-aligned), fb's low 8 bits are
    // zero and (2g + h) ^ swz = 2g ^ (h ^ swz), so fb + 16·((2g + h) ^ swz) = fbc ^ 32g with
    // fbc = fb | 16·(h ^ swz): ONE v_xor per read (an asm statement, so it is recomputed per
    // use instead of hoisted into G registers the d = 768 schedule does not have), the k-group
    // an immediate.  The old form took three VALU per read in the MFMA gaps.
    constexpr bool kXorFrag = ROWB % 256 == 0 && TILE_B % 256 == 0;
    const uint32_t fbc = (uint32_t)(size_t)((const __attribute__((address_space(3))) char*)fb) | (uint32_t)((h ^ swz) << 4);
    auto frag = [&](int u) __attribute__((always_inline)) {
      if constexpr (kXorFrag) {
        uint32_t ad = fbc;
        if (u % G) asm volatile("v_xor_b32 %0, %1, %2" : "=v"(ad) : "i"((u % G) * 32), "v"(fbc));
        return *(const __attribute__((address_space(3))) u32x4v*)((const __attribute__((address_space(3))) char*)(size_t)ad +
                                                                 (u / G) * G * 32);
      } else {
        int sw = swz;
        asm volatile("" : "+v"(sw));  // opaque per use: no hoisted per-u address registers
        return *(const u32x4v*)(fb + (((2 * (u % G) + h) ^ sw) << 4) + (u / G) * G * 32);
      }
    };
    uint32_t teB = 0, tpB = 0, teA = 0, tpA = 0, epA = 0, epB = 0;
    bool anyA = false, anyB = false;
    // (PFC + 2)-slot fragment ring over both chains (step s: block s / U, k-step s % U),
    // prefetch distance PFC; a fragment stays live one step past its MFMA (inline-asm MFMAs
    // are opaque to hazard tracking: no ds_read may land in registers an in-flight MFMA reads)
    constexpr int PFC = kScan4ChainPf, NRC = PFC + 2;
    u32x4v fq[NRC];
    static_for<PFC>([&](auto II) { fq[decltype(II)::value] = frag(decltype(II)::value % U); });
    static_for<2 * U>([&](auto SS) {
      constexpr int st = decltype(SS)::value;
      constexpr int b = st / U, u = st % U;
      if constexpr (st + PFC < 2 * U) fq[(st + PFC) % NRC] = frag((st + PFC) % U);
      const u32x4v fv = fq[st % NRC];
      f32x16s& c = b ? accB : accA;
      if constexpr (st < NA) {
        if constexpr (u == 0) {
          if constexpr (F16)
            asm volatile("v_mfma_f32_32x32x16_f16 %0, %1, %2, 0" : "=&v"(c) : "v"(fv), "a"(qv[st]));
          else
            asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, 0" : "=&v"(c) : "v"(fv), "a"(qv[st]));
        } else {
          if constexpr (F16)
            asm volatile("v_mfma_f32_32x32x16_f16 %0, %1, %2, %0" : "+v"(c) : "v"(fv), "a"(qv[st]));
          else
            asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(c) : "v"(fv), "a"(qv[st]));
        }
      } else {
        // VGPR-resident query operand: the s_nop covers a VALU write (a copy the register
        // allocator may place) -> MFMA read hazard the compiler cannot see through asm — two
        // wait states (cdna_hip_programming.md §5.7: a just-written "v" operand -> MFMA
        // operand, s_nop 1; it was s_nop 4, three cycles more in 32 of every 96 MFMA gaps)
        if constexpr (u == 0) {
          if constexpr (F16)
            asm volatile("s_nop 1\n\tv_mfma_f32_32x32x16_f16 %0, %1, %2, 0" : "=&v"(c) : "v"(fv), "v"(qv[st]));
          else
            asm volatile("s_nop 1\n\tv_mfma_f32_32x32x16_bf16 %0, %1, %2, 0" : "=&v"(c) : "v"(fv), "v"(qv[st]));
        } else {
          if constexpr (F16)
            asm volatile("s_nop 1\n\tv_mfma_f32_32x32x16_f16 %0, %1, %2, %0" : "+v"(c) : "v"(fv), "v"(qv[st]));
          else
            asm volatile("s_nop 1\n\tv_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(c) : "v"(fv), "v"(qv[st]));
        }
      }
      if constexpr (st > 0) asm volatile("" ::"v"(fq[(st + NRC - 1) % NRC]));
      // the other block's accumulator: its chain ended >= 2 MFMAs ago; the tie makes every
      // VALU read of it come after this point, with an extra wait for the MFMA to retire
      if constexpr (u == 1) {
        if constexpr (b == 0) {
          if constexpr (epib) asm volatile("s_nop 15" : "+v"(accB));
        } else {
          asm volatile("s_nop 15" : "+v"(accA));
        }
      }
      if constexpr (b == 0) {
        static_for<kSlicesA>([&](auto SL) {
          constexpr int s = decltype(SL)::value;
          if constexpr (scan4_atA(s, U, kEpi, PIECES) == u) {
            if constexpr (s < kEpi) {
              if constexpr (epib) epi_slice(SL, accB, tile - 1, ppw, pmw, pewB, qB, slB, teB, tpB, epB, anyB);
            } else if constexpr (s == kEpi) {
              nw_p = a.present[w0 + wtile];
              nw_m = a.mask[w0 + wtile];
              nw_eA = erowA[w0 + wtile];
              nw_eB = erowB[w0 + wtile];
            } else {
              if constexpr (!(ABL & 2)) stage_piece(stile, sslot, s - kEpi - 1);
            }
          }
        });
      } else {
        static_for<kEpi>([&](auto SL) {
          constexpr int s = decltype(SL)::value;
          if constexpr (scan4_at(s, U) == u) epi_slice(SL, accA, tile, pw, mw, ewA, qA, slA, teA, tpA, epA, anyA);
        });
      }
    });
    ppw = pw;
    pmw = mw;
    pewB = ewB;
    if constexpr (!(ABL & 4)) {
      // the youngest vector-memory ops: block A's score-image stores (chain B), issued after
      // the last DMA piece, and (three-deep ring) the pieces of tile + 2 — everything older
      // (the next tile's pieces, the words) has landed once at most that many remain (vmcnt
      // retires in order; streaming appends after the pieces only make the wait longer)
      constexpr int young = (kStores ? 4 : 0) + (RING == 3 && !(ABL & 2) ? PIECES : 0);
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(young) : "memory");
      __syncthreads();
    }
    pw = nw_p;
    mw = nw_m;
    ewA = nw_eA;
    ewB = nw_eB;
    asm volatile("" : "+v"(pw), "+v"(mw), "+v"(ewA), "+v"(ewB));
  };

  using B0 = std::integral_constant<int, 0>;
  using B1 = std::integral_constant<int, 1>;
  using EY = std::integral_constant<bool, true>;
  using EN = std::integral_constant<bool, false>;

  if constexpr (IL) {
    // ---- interleaved schedule (d <= 512): per k-step one fragment read feeds both blocks'
    // MFMAs (A_u, B_u), halving LDS fragment reads per MFMA — with one read per MFMA the
    // MFMA + LDS loop ran at ~0.69 of the clocked peak, against ~0.87 for scan3's two MFMAs
    // per read.  Two accumulator sets alternate with the tiles (set = buffer = tile parity),
    // and both blocks' epilogues of tile t-1 are woven into tile t, after its DMA pieces.
    f32x16s accA1 = {}, accB1 = {};
    uint32_t pewA = 0;
    int fxo[G];  // LDS byte offset of chunk (2g + h) ^ swz of this lane's row (scan2 layout)
#pragma unroll
    for (int g = 0; g < G; ++g) fxo[g] = ((2 * g + h) ^ swz) << 4;
    // Sparse list epilogue (masks: configs[2]'s ~2 % dense constraint mask).  The mask and the
    // item space are per item, so whether accumulator register g can hold an eligible item is
    // the same for every lane of a half: u = the union over both halves (uniform).  When u has
    // at most kSparseRegs registers, the list epilogue of the previous tile inserts only those
    // (a scalar loop, the register picked by a uniform index) instead of all sixteen register
    // pairs — the masked-out ones would insert code 0, a no-op.  The lists are the same keys.
    // in three slices per block, each woven into its own MFMA gap: 0 the lane's eligibility
    // word, 1 the inserts of the registers u names, 2 rank 0 (the present maximum)
    auto list_sparse = [&](auto SS, const f32x16s& p, int ptile, uint32_t eew, float k2, ListTop5& L, ListTop2& R,
                           uint32_t u, uint32_t& e16) __attribute__((always_inline)) {
      constexpr int s = decltype(SS)::value;
      if constexpr (ABL & 1) return;  // (probe: no epilogue)
      const int ptile0 = ptile * 32;
      if constexpr (s == 0) {
        e16 = list_elig16(ppw & pmw & ~eew, ptile0, a.n_valid, h);
      } else if constexpr (s == 1) {
        const uint32_t pb = (uint32_t)l_cnt << 4;
        for (uint32_t uu = u; uu; uu &= uu - 1u) {
          const int g = __builtin_ctz(uu);
          const float v = p[g];
          const uint32_t c =
              __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_pknorm_u16(fmaf(v, k2, 0.5f), 0.f)) & 0xFFFFu;
          L.ins(((e16 >> g) & 1u) ? (c << 16) | pb | (uint32_t)g : 0u);
        }
      } else if (a.r0lists) {
        const float m = list_present_max(p, list_elig16(ppw, ptile0, a.n_valid, h));
        R.ins(list_r0_key(m, k2, (uint32_t)(ptile - tile_lo)));
      }
    };
    auto il_body = [&](auto BUF, auto EPI, auto SPC, int tile, uint32_t su, int slot) __attribute__((always_inline)) {
      constexpr int buf = decltype(BUF)::value;  // accumulator set (tile parity); LDS ring slot: `slot`
      constexpr bool epi = decltype(EPI)::value;
      constexpr bool SP = decltype(SPC)::value;  // sparse list epilogue (registers su only)
      f32x16s& cA = buf ? accA1 : accA;
      f32x16s& cB = buf ? accB1 : accB;
      f32x16s& pA = buf ? accA : accA1;  // the previous tile's set
      f32x16s& pB = buf ? accB : accB1;
      // staging runs two tiles ahead (ring slot slot - 1 mod 3, read by tile - 1, free since the
      // last barrier); the words of the next tile go out first, so the end-of-tile wait can leave
      // the youngest tile's DMA in flight
      const int stile = tile + 2 < tile_hi ? tile + 2 : tile;
      const int sslot = slot == 0 ? 2 : slot - 1;
      const int wtile = tile + 1 < tile_hi ? tile + 1 : tile;
      // fragment addresses from the per-lane chunk offsets fxo (registers are not short on this
      // schedule): one add per distinct chunk and tile, the k-group offset an immediate
      const char* fbase = smem + slot * TILE_B + rrow;
      auto frag = [&](int u) __attribute__((always_inline)) {
        return *(const u32x4v*)(fbase + fxo[u % G] + (u / G) * G * 32);
      };
      uint32_t teA = 0, tpA = 0, teB = 0, tpB = 0, epA = 0, epB = 0;
      bool anyA = false, anyB = false;
      // fragment ring in k-steps: prefetch distance PF (BB build knob kScan4Pf), ring PF + 2
      constexpr int PF = KU <= 48 ? kScan4Pf : 2, NR = PF + 2;  // (d = 512: no registers for more)
      u32x4v fq[NR];
      static_for<(PF < U ? PF : U)>([&](auto II) { fq[decltype(II)::value] = frag(decltype(II)::value); });
      static_for<2 * U>([&](auto SS) {
        constexpr int st = decltype(SS)::value;
        constexpr int u = st >> 1, b = st & 1;
        // fragment u-1 stays live until A_u has issued (inline-asm MFMAs are opaque to hazard
        // tracking)
        if constexpr (b == 0 && u + PF < U) fq[(u + PF) % NR] = frag(u + PF);
        const u32x4v fv = fq[u % NR];
        f32x16s& c = b ? cB : cA;
        if constexpr (u == 0) {
          if constexpr (F16)
            asm volatile("v_mfma_f32_32x32x16_f16 %0, %1, %2, 0" : "=&v"(c) : "v"(fv), "a"(qv[b * U + u]));
          else
            asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, 0" : "=&v"(c) : "v"(fv), "a"(qv[b * U + u]));
        } else {
          if constexpr (F16)
            asm volatile("v_mfma_f32_32x32x16_f16 %0, %1, %2, %0" : "+v"(c) : "v"(fv), "a"(qv[b * U + u]));
          else
            asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(c) : "v"(fv), "a"(qv[b * U + u]));
        }
        if constexpr (b == 0 && u > 0) asm volatile("" ::"v"(fq[(u + NR - 1) % NR]));
        if constexpr (st == 1 && epi) asm volatile("s_nop 15" : "+v"(pA), "+v"(pB));
        if constexpr (LIST) {
          // slices: the pending period store (step 0, ahead of the DMA), DMA pieces (even
          // steps from 2), the next tile's words, then the previous tile's list epilogue of
          // block A and block B (odd steps between the pieces, then one per step) and the
          // period counter
          constexpr int kE = SP ? 7 : 2 * kLE + 1;
          static_for<PIECES + 2 + kE>([&](auto SL) {
            constexpr int s = decltype(SL)::value;
            constexpr int e = s - PIECES - 2;  // epilogue slice index (s >= PIECES + 2)
            constexpr int at0 = s == 0 ? 0 : s <= PIECES ? 2 * s : s == PIECES + 1 ? 1
                                : e < PIECES ? 3 + 2 * e : 2 * PIECES + 3 + (e - PIECES);
            constexpr int at = at0 < 2 * U ? at0 : 2 * U - 1;
            if constexpr (at == st) {
              if constexpr (s == 0) {
                if (pend) {
                  list_put(pend_period, pendA, pendB);
                  pend = false;
                }
              } else if constexpr (s <= PIECES) {
                stage_piece(stile, sslot, s - 1);
              } else if constexpr (s == PIECES + 1) {
                nw_p = a.present[w0 + wtile];
                nw_m = a.mask[w0 + wtile];
                nw_eA = erowA[w0 + wtile];
                nw_eB = erowB[w0 + wtile];
              } else if constexpr (epi) {
                if constexpr (SP && e < 6) {
                  if constexpr (e < 3)
                    list_sparse(std::integral_constant<int, e>{}, pA, tile - 1, pewA, k2A, lstA, r0A, su, le16A);
                  else
                    list_sparse(std::integral_constant<int, e - 3>{}, pB, tile - 1, pewB, k2B, lstB, r0B, su, le16B);
                } else if constexpr (!SP && e < kLE) {
                  list_slice(std::integral_constant<int, e>{}, pA, tile - 1, ppw, pmw, pewA, k2A, lstA, r0A, le16A, lfullA,
                             lkoA);
                } else if constexpr (!SP && e < 2 * kLE) {
                  list_slice(std::integral_constant<int, e - kLE>{}, pB, tile - 1, ppw, pmw, pewB, k2B, lstB, r0B, le16B,
                             lfullB, lkoB);
                } else {
                  if (++l_cnt == a.l_period) {
                    pendA = lstA.pack();
                    pendB = lstB.pack();
                    pend = true;
                    pend_period = l_period++;
                    lstA.reset();
                    lstB.reset();
                    l_cnt = 0;
                  }
                }
              }
            }
          });
          return;
        }
        // slices: DMA pieces (every other step from st = 2), the next tile's words, then
        // the previous tile's epilogue of block A and of block B
        constexpr int kS = PIECES + 1 + 2 * kEpi;
        static_for<kS>([&](auto SL) {
          constexpr int s = decltype(SL)::value;
          constexpr int at0 = s < PIECES ? 2 + 2 * s : s == PIECES ? 1 : 2 + 2 * PIECES + (s - PIECES);
          constexpr int at = at0 < 2 * U ? at0 : 2 * U - 1;
          if constexpr (at == st) {
            if constexpr (s < PIECES) {
              if constexpr (!(ABL & 2)) stage_piece(stile, sslot, s);
            } else if constexpr (s == PIECES) {
              nw_p = a.present[w0 + wtile];
              nw_m = a.mask[w0 + wtile];
              nw_eA = erowA[w0 + wtile];
              nw_eB = erowB[w0 + wtile];
            } else if constexpr (epi) {
              constexpr int e = s - PIECES - 1;
              if constexpr (e < kEpi)
                epi_slice(std::integral_constant<int, e>{}, pA, tile - 1, ppw, pmw, pewA, qA, slA, teA, tpA, epA, anyA);
              else
                epi_slice(std::integral_constant<int, e - kEpi>{}, pB, tile - 1, ppw, pmw, pewB, qB, slB, teB, tpB, epB,
                          anyB);
            }
          }
        });
      });
      ppw = pw;
      pmw = mw;
      pewA = ewA;
      pewB = ewB;
      if constexpr (!(ABL & 4)) {
        // the youngest vector-memory ops: the DMA pieces of tile + 2 and, after them, the
        // previous tile's score-image stores — everything older (the next tile's pieces and
        // words) has landed once at most that many remain (vmcnt retires in order)
        constexpr int young = (kStores && epi ? 8 : 0) + ((ABL & 2) ? 0 : PIECES);
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(young) : "memory");
        __syncthreads();
      }
      pw = nw_p;
      mw = nw_m;
      ewA = nw_eA;
      ewB = nw_eB;
      asm volatile("" : "+v"(pw), "+v"(mw), "+v"(ewA), "+v"(ewB));
    };
    using SN = std::integral_constant<bool, false>;
    using SY = std::integral_constant<bool, true>;
    // one tile with the previous tile's epilogue: sparse when at most kSparseRegs registers can
    // hold an eligible item of it (one uniform branch per tile, decided on the item words)
    constexpr int kSparseRegs = 8;
    int slot = 0;  // LDS ring slot of the tile being computed
    auto il_step = [&](auto BUF, int tile) __attribute__((always_inline)) {
      if constexpr (LIST) {
        const uint32_t w = __builtin_amdgcn_readfirstlane(ppw & pmw);
        const int pt0 = (tile - 1) * 32;
        const uint32_t u = list_elig16(w, pt0, a.n_valid, 0) | list_elig16(w, pt0, a.n_valid, 1);
        if (__builtin_popcount(u) <= kSparseRegs)
          il_body(BUF, EY{}, SY{}, tile, u, slot);
        else
          il_body(BUF, EY{}, SN{}, tile, 0u, slot);
      } else {
        il_body(BUF, EY{}, SN{}, tile, 0u, slot);
      }
    };
    auto next_slot = [&]() __attribute__((always_inline)) { slot = slot == 2 ? 0 : slot + 1; };
    il_body(B0{}, EN{}, SN{}, tile_lo, 0u, slot);
    stamp(2);
    next_slot();
    int tile = tile_lo + 1;
    for (;;) {
      if (tile >= tile_hi) break;
      il_step(B1{}, tile);
      ++tile;
      next_slot();
      if (tile >= tile_hi) break;
      il_step(B0{}, tile);
      ++tile;
      next_slot();
      if (tile == tile_lo + 5) stamp(3);
    }
    stamp(4);
    // both blocks' epilogues of the last tile (not overlapped)
    auto last = [&](f32x16s& lA, f32x16s& lB) __attribute__((always_inline)) {
      asm volatile("s_nop 15\n\ts_nop 15\n\ts_nop 15\n\ts_nop 15" : "+v"(lA), "+v"(lB));
      if constexpr (LIST) {
        if (pend) list_put(pend_period, pendA, pendB);
        static_for<kLE>([&](auto SL) {
          list_slice(SL, lA, tile - 1, ppw, pmw, pewA, k2A, lstA, r0A, le16A, lfullA, lkoA);
        });
        static_for<kLE>([&](auto SL) {
          list_slice(SL, lB, tile - 1, ppw, pmw, pewB, k2B, lstB, r0B, le16B, lfullB, lkoB);
        });
        if (a.r0lists) {
          if (liveA) *(uint2*)(a.r0lists + 2 * list_slot(chunk, 0, 1, l_nb, qA >> 5, lane)) = make_uint2(r0A.k0, r0A.k1);
          if (liveB) *(uint2*)(a.r0lists + 2 * list_slot(chunk, 0, 1, l_nb, qB >> 5, lane)) = make_uint2(r0B.k0, r0B.k1);
        }
        list_put(l_period, lstA.pack(), lstB.pack());  // the last (possibly partial) period
        if (a.trace && tid == 0) a.trace[(size_t)L * 8 + 6] = (uint64_t)(tile_hi - tile_lo);
        if (a.trace && tid == 0) a.trace[(size_t)L * 8 + 7] = __builtin_amdgcn_s_memtime() - clk0;
        stamp(5);
        return;
      }
      uint32_t te = 0, tp = 0, ep = 0;
      bool any = false;
      static_for<kEpi>([&](auto SL) { epi_slice(SL, lA, tile - 1, ppw, pmw, pewA, qA, slA, te, tp, ep, any); });
      te = tp = ep = 0;
      any = false;
      static_for<kEpi>([&](auto SL) { epi_slice(SL, lB, tile - 1, ppw, pmw, pewB, qB, slB, te, tp, ep, any); });
    };
    if (((tile - 1 - tile_lo) & 1) == 0)
      last(accA, accB);
    else
      last(accA1, accB1);
    if constexpr (PILOT) pm_store();
    if constexpr (STREAM) {
      a.cand_cnt[region(qA)] = slA.n;
      a.cand_cnt[region(qB)] = slB.n;
      if (a.cand_pmax) {
        a.cand_pmax[region(qA)] = slA.rkey;
        a.cand_pmax[region(qB)] = slB.rkey;
      }
    }
  } else {
  int slot = 0;  // LDS ring slot of the tile being computed
  tile_body(EN{}, tile_lo, slot);
  int tile = tile_lo + 1;
  for (; tile < tile_hi; ++tile) {
    slot = slot == RING - 1 ? 0 : slot + 1;
    tile_body(EY{}, tile, slot);
  }
  // block B's epilogue of the last tile (not overlapped)
  asm volatile("s_nop 15\n\ts_nop 15\n\ts_nop 15\n\ts_nop 15" : "+v"(accB));
  {
    uint32_t te = 0, tp = 0, ep = 0;
    bool any = false;
    static_for<kEpi>([&](auto SL) { epi_slice(SL, accB, tile - 1, ppw, pmw, pewB, qB, slB, te, tp, ep, any); });
  }
  if constexpr (PILOT) pm_store();
  if constexpr (STREAM) {
    a.cand_cnt[region(qA)] = slA.n;
    a.cand_cnt[region(qB)] = slB.n;
    if (a.cand_pmax) {
      a.cand_pmax[region(qA)] = slA.rkey;
      a.cand_pmax[region(qB)] = slB.rkey;
    }
  }
  }  // !IL
}

template <int KU, int ABL = 0>
__global__ __launch_bounds__(kScanWaves * 64, 1) void scan4_kernel(GemmArgs a, int n_chunks, int tiles_total) {
  scan4_body<KU, ABL>(a, n_chunks, tiles_total, blockIdx.x);
}

// Both sides of a hybrid search in one launch (content KU0, CF KU1): workgroups [0, nb0)
// scan side 0, the rest side 1 — one launch ramp and tail, and the CF side's short tiles
// fill the CUs beside the content side's long ones.
template <int KU0, int KU1, int ABL>
__global__ __launch_bounds__(kScanWaves * 64, 1) void scan4_dual_kernel(GemmArgs a0, GemmArgs a1, int nc0, int t0,
                                                                        int nc1, int t1, int nb0) {
  if ((int)blockIdx.x < nb0)
    scan4_body<KU0, ABL, true>(a0, nc0, t0, blockIdx.x);
  else
    scan4_body<KU1, ABL, true>(a1, nc1, t1, blockIdx.x - nb0);
}

}  // namespace bb
