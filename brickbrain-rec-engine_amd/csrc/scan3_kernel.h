// scan3_kernel.h — fp32-accurate scan on the bf16 MFMA: split-precision "bf16x6".
//
// An fp32 value splits exactly into three bf16 planes, x = xh + xm + xl (8+8+8 mantissa
// bits). The cosine score q·x is the sum of the nine plane products. This kernel keeps
// the six terms of order >= 2^-16 relative:
//   xh·qh + xm·qh + xh·qm + xl·qh + xh·ql + xm·qm
// and drops xm·ql, xl·qm and xl·ql, which are ~2^-24 and below. Each bf16 product is
// exact, and the MFMA accumulates in f32.
//
// Accuracy, measured against an f64 reference on unit vectors (d = 384, see
// tools/bf16x6_error.py): max error 1.0e-7 (numpy fp32: 1.5e-7). It is fp32-class, so the
// parity bar is unchanged.
//
// Cost per 16-wide k step is six v_mfma_f32_32x32x16_bf16 (6 × 32 cycles) against eight
// v_mfma_f32_32x32x2_f32 (8 × 64 cycles): 2.7× less MFMA time. Unlike the fp32 MFMA, the
// bf16 MFMA leaves the SIMD's vector issue free for most of its cycles, so the woven
// epilogue overlaps.
//
// Layout:
// * Items are stored as the t3 tile image (common.h): per 32-row tile, plane-major 16-B
//   chunks with the 32 rows of a chunk adjacent — the LDS order. Tiles are staged by
//   LDS-DMA into a double buffer with contiguous 1-KiB pieces; fragment reads are
//   contiguous 1-KiB wave reads (conflict-free, no swizzle).
// * Queries come split by the prep kernel, as a "q3f" image in load order (common.h), so
//   each of the 3·U query loads per lane is one coalesced 1-KiB wave access. They are
//   issued behind the first tile's LDS-DMA. qh and qm are resident in AGPRs, ql in VGPRs.
// * Epilogue: per-tile maxima as scan2_kernel.h; scores go out as the blocked image
//   (sblk_quad, common.h) — each wave stores its accumulator as-is, 4 full 1-KiB writes.
#pragma once
#include "scan2_kernel.h"

namespace bb {

constexpr int kScan3MaxKP = 48;  // 2 tiles of 32 rows × 3 planes × 768 B = 144 KiB LDS

// Query planes of this lane for k-step u from the prep kernel's q3f image (common.h):
// chunk (2u + h) of each plane of query q, three coalesced 1-KiB wave loads.  Rows past
// M_valid are zero rows written by prep.
template <int U>
__device__ __forceinline__ void scan3_load_query_step(const char* blk, int u, u32x4v& qh, u32x4v& qm, u32x4v& ql) {
  qh = *(const u32x4v*)(blk + u * 1024);
  qm = *(const u32x4v*)(blk + (U + u) * 1024);
  ql = *(const u32x4v*)(blk + (2 * U + u) * 1024);
}

// KP: 16-B chunks per plane row (Dpad·2/16).  ABL: as scan2, plus 64 = no query loads and
// 128 = no first-tile staging, 256 = timeline into a.trace (probe only).
template <int KP, int ABL = 0>
__global__ __launch_bounds__(kScanWaves * 64, 1) void scan3_kernel(GemmArgs a, int n_chunks, int tiles_total) {
  constexpr int U = KP / 2;                 // 16-wide k steps per tile
  constexpr int ROWB = 3 * KP * 16;         // bytes of one item row (three planes)
  constexpr int TILE_B = 32 * ROWB;
  constexpr int PIECES = TILE_B / (1024 * kScanWaves);
  static_assert(KP % 8 == 0 && KP <= kScan3MaxKP, "unsupported plane width");
  static_assert(TILE_B % (1024 * kScanWaves) == 0, "tile must split into whole 1 KiB pieces per wave");
  __shared__ __attribute__((aligned(16))) char smem[2 * TILE_B];

  const int n_groups = a.Mpad / (kScanWaves * 32);
  const int total = n_groups * n_chunks;
  const int L = blockIdx.x;
  const int xcd = L & 7, local = L >> 3, q8 = total >> 3, r8 = total & 7;
  const int t = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + local;
  const int chunk = t / n_groups, group = t - chunk * n_groups;
  const int tile_lo = (int)((int64_t)chunk * tiles_total / n_chunks);
  const int tile_hi = (int)((int64_t)(chunk + 1) * tiles_total / n_chunks);

  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 31, h = lane >> 5;
  const int q = group * kScanWaves * 32 + wave * 32 + r;
  if (tile_lo >= tile_hi) return;  // uniform per workgroup
  // probe-only timeline: s_memrealtime (100 MHz) per phase, s_memtime (core clock) span
  auto stamp = [&](int slot) __attribute__((always_inline)) {
    if constexpr (ABL & 256) {
      if (tid == 0) a.trace[blockIdx.x * 32 + slot] = __builtin_amdgcn_s_memrealtime();
    }
  };
  uint64_t clk0 = 0;
  if constexpr (ABL & 256) clk0 = __builtin_amdgcn_s_memtime();
  stamp(0);

  // Items come as the t3 tile image (common.h): a tile is one contiguous block in LDS order,
  // so a wave's 1-KiB LDS-DMA piece is a contiguous 1 KiB of HBM (uniform SGPR address plus
  // a constant lane offset, no per-tile vector arithmetic), and the fragment of plane P at
  // u-step u (chunks 2u, 2u+1 of all 32 rows) is the contiguous 1 KiB at (P·KP + 2u)·512.
  const char* Xg = (const char*)a.X;
  const uint32_t lds_base = (uint32_t)(size_t)((__attribute__((address_space(3))) char*)smem);
  const int lane16 = lane * 16;
  uint32_t lb[2][2];  // fragment read bases: buffer b, offsets below / from 32 KiB
#pragma unroll
  for (int b = 0; b < 2; ++b) {
    lb[b][0] = lds_base + b * TILE_B + lane16;
    lb[b][1] = lb[b][0] + 32768;
    asm volatile("" : "+v"(lb[b][0]), "+v"(lb[b][1]));
  }
  auto stage_piece = [&](int tile, int buf, int p) __attribute__((always_inline)) {
    const int pc = wave * PIECES + p;
    const char* src = Xg + (size_t)tile * TILE_B + pc * 1024;
    const uint32_t dst = lds_base + buf * TILE_B + pc * 1024;
    asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2" ::"s"(dst), "v"(lane16), "s"(src)
                 : "memory");
  };

  const size_t w0 = (size_t)(a.slab_start >> 5);
  const uint32_t* erow = a.excl + (size_t)(q < a.M_valid ? q : a.M_valid - 1) * a.excl_ld;
  // blocked score image (sblk_quad): this wave's 4-KiB block per tile, lane-linear
  float* Sblk = a.S + sblk_lane(q, h, a.ldt);
  constexpr bool STREAM = (ABL & kScanStream) != 0;
  StreamLane sl;
  const size_t region = ((size_t)q * n_chunks + chunk) * 2 + h;
  if constexpr (STREAM) stream_begin(a, q, region, sl);

  // first tile's LDS-DMA ahead of the query loads: both streams are in flight together
  if constexpr (!(ABL & 128)) {
#pragma unroll
    for (int p = 0; p < PIECES; ++p) stage_piece(tile_lo, 0, p);
  }
  // Query stream: k-steps [0, QD) load here, behind the first tile's pieces; steps
  // [QD, U) load inside the first tile, QD steps ahead of their MFMAs, so the ~288 KiB of
  // queries per workgroup stream in under the first tile's MFMAs.  The compiler waits for
  // each query register at its first use (pinned to AGPRs there).
  constexpr int QD = U / 2;
  const char* qblk = (const char*)a.Q + (size_t)(q >> 5) * 3 * U * 1024 + lane16;
  u32x4v qh[U], qm[U], ql[U];
  auto load_q = [&](int u) __attribute__((always_inline)) {
    if constexpr (ABL & 64) {
      qh[u] = qm[u] = ql[u] = u32x4v{0, 0, 0, 0};
    } else {
      scan3_load_query_step<U>(qblk, u, qh[u], qm[u], ql[u]);
      asm volatile("" ::: "memory");  // keep the step order: the waits count on it
    }
  };
#pragma unroll
  for (int u = 0; u < QD; ++u) load_q(u);
  stamp(1);  // prologue loads issued
  // loads retire in order: once at most the 3·QD query loads are outstanding, the older
  // pieces of the first tile have landed
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * QD) : "memory");
  __syncthreads();
  stamp(2);
  asm volatile("s_nop 4");

  f32x16s accE = {}, accO = {};
  uint32_t pw = 0, mw = 0, ew = 0;
  uint32_t nw_p = 0, nw_m = 0, nw_e = 0;

  constexpr int kEpiSlices = 8 + PIECES;
  auto tile_body = [&](auto BUF, auto EPI, int tile, f32x16s& c, const f32x16s& p) __attribute__((always_inline)) {
    constexpr int buf = decltype(BUF)::value;
    constexpr bool epi = decltype(EPI)::value && !(ABL & 1);
    constexpr bool first = !decltype(EPI)::value;  // the first tile (streams the queries)
    const int ptile = tile - 1;
    const int stile = tile + 1 < tile_hi ? tile + 1 : tile;
    uint32_t te = 0, tp = 0;
    const int ptile0 = ptile * 32;
    // fragment of plane P at u-step u: ds_read two steps ahead
    // (two base registers per buffer keep every ds_read offset inside its 16-bit field)
    auto frag = [&](int P, int u) __attribute__((always_inline)) {
      const int off = (P * KP + 2 * u) * 512;
      const uint32_t base = off < 32768 ? lb[buf][0] : lb[buf][1];
      return *(const __attribute__((address_space(3))) u32x4v*)(size_t)(base + (off < 32768 ? off : off - 32768));
    };
    // 4-slot ring, prefetch distance 2.  Inline-asm MFMAs are opaque to the compiler's
    // hazard tracking, so a fragment's registers are kept live (empty asm use) until the
    // next step's MFMAs are issued: no ds_read may land in registers an in-flight MFMA
    // still reads.
    u32x4v fh[4], fm[4], fl[4];
    fh[0] = frag(0, 0);
    fm[0] = frag(1, 0);
    fl[0] = frag(2, 0);
    if constexpr (U > 1) {
      fh[1] = frag(0, 1);
      fm[1] = frag(1, 1);
      fl[1] = frag(2, 1);
    }
    static_for<U>([&](auto UU) {
      constexpr int u = decltype(UU)::value;
      if constexpr (u + 2 < U) {
        fh[(u + 2) % 4] = frag(0, u + 2);
        fm[(u + 2) % 4] = frag(1, u + 2);
        fl[(u + 2) % 4] = frag(2, u + 2);
      }
      const u32x4v xh = fh[u % 4], xm = fm[u % 4], xl = fl[u % 4];
      if constexpr (first) {
        if constexpr (u + QD < U) load_q(u + QD);
        asm volatile("" : "+a"(qh[u]), "+a"(qm[u]));
      }
      // one accumulation chain, largest term first
      if constexpr (u == 0)
        asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, 0" : "=&v"(c) : "v"(xh), "a"(qh[u]));
      else
        asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(c) : "v"(xh), "a"(qh[u]));
      asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(c) : "v"(xm), "a"(qh[u]));
      asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(c) : "v"(xh), "a"(qm[u]));
      asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(c) : "v"(xl), "a"(qh[u]));
      // ql may be parked in AGPRs by the register allocator and copied back right before
      // this MFMA: the s_nop covers the VALU-write -> MFMA-read hazard the compiler cannot
      // see through inline asm
      asm volatile("s_nop 4\n\tv_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(c) : "v"(xh), "v"(ql[u]));
      asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(c) : "v"(xm), "a"(qm[u]));
      if constexpr (u > 0) asm volatile("" ::"v"(fh[(u + 3) % 4]), "v"(fm[(u + 3) % 4]), "v"(fl[(u + 3) % 4]));
      // schedule: the next tile's LDS-DMA pieces first (two per u-step, so its HBM/MALL
      // latency has most of the tile to land), then the previous tile's epilogue
      static_for<kEpiSlices>([&](auto SS) {
        constexpr int s = decltype(SS)::value;
        // staging: two pieces per u-step, from step 0; in the first tile only after its
        // last query loads, so no query wait ever covers a freshly issued piece
        constexpr int s_stage = (first ? QD : 0) + (s - 8) / 2;
        constexpr int s_epi = U / 2 + s;
        constexpr int su0 = s >= 8 ? s_stage : s_epi;
        constexpr int su = su0 < U ? su0 : U - 1;
        if constexpr (su == u) {
          if constexpr (s == 0) {
            if constexpr (epi && !(ABL & 32)) tile_maxima(p, ptile0, a.n_valid, pw, pw & mw & ~ew, h, te, tp);
          } else if constexpr (s == 1) {
            if constexpr (epi && STREAM) {
              stream_append(p, ptile0, a.n_valid, pw & mw & ~ew, h, te, sl, (uint32_t)a.cand_cap, a.gid0);
            } else if constexpr (epi && !(ABL & 32)) {
              const uint32_t te2 = xor32(te), tp2 = xor32(tp);
              te = te2 > te ? te2 : te;
              tp = tp2 > tp ? tp2 : tp;
            }
          } else if constexpr (s == 2 && STREAM) {
            if constexpr (epi) {
              if (a.cand_pmax) stream_rank0(p, ptile0, a.n_valid, pw, h, tp, sl, a.gid0);
            }
          } else if constexpr (s < 6) {
            if constexpr (epi && !(ABL & 8) && !STREAM) {
              constexpr int j = s - 2;
              *(float4*)(Sblk + (size_t)ptile * 1024 + j * 256) = make_float4(p[4 * j], p[4 * j + 1], p[4 * j + 2], p[4 * j + 3]);
            }
          } else if constexpr (s == 6) {
            if constexpr (epi && !(ABL & 16) && !STREAM) if (!h || a.pmax) (h ? a.pmax : a.tmax)[(size_t)q * a.ldt + ptile] = h ? tp : te;
          } else if constexpr (s == 7) {
            nw_p = a.present[w0 + tile];
            nw_m = a.mask[w0 + tile];
            nw_e = erow[w0 + tile];
          } else {
            if constexpr (!(ABL & 2)) stage_piece(stile, buf ^ 1, s - 8);
          }
        }
      });
    });
    // The MFMAs are inline asm, so the compiler cannot see their result latency: this
    // ties the accumulator to a wait long enough for the last MFMA to retire, before any
    // register copy or read of it the compiler may place after this point.
    asm volatile("s_nop 15\n\ts_nop 15\n\ts_nop 15\n\ts_nop 15" : "+v"(c));
    pw = nw_p;
    mw = nw_m;
    ew = nw_e;
    if constexpr (!(ABL & 4)) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
  };

  auto last_epilogue = [&](int tile, const f32x16s& p) __attribute__((always_inline)) {
    if constexpr (ABL & 1) return;
    asm volatile("s_nop 15\n\ts_nop 15\n\ts_nop 15\n\ts_nop 15");  // asm-MFMA result -> VALU read
    uint32_t te = 0, tp = 0;
    tile_maxima(p, tile * 32, a.n_valid, pw, pw & mw & ~ew, h, te, tp);
    if constexpr (STREAM) {
      stream_append(p, tile * 32, a.n_valid, pw & mw & ~ew, h, te, sl, (uint32_t)a.cand_cap, a.gid0);
      if (a.cand_pmax) stream_rank0(p, tile * 32, a.n_valid, pw, h, tp, sl, a.gid0);
      return;
    }
    const uint32_t te2 = xor32(te), tp2 = xor32(tp);
    te = te2 > te ? te2 : te;
    tp = tp2 > tp ? tp2 : tp;
#pragma unroll
    for (int j = 0; j < 4; ++j)
      *(float4*)(Sblk + (size_t)tile * 1024 + j * 256) = make_float4(p[4 * j], p[4 * j + 1], p[4 * j + 2], p[4 * j + 3]);
    if (!h || a.pmax) (h ? a.pmax : a.tmax)[(size_t)q * a.ldt + tile] = h ? tp : te;
  };

  using B0 = std::integral_constant<int, 0>;
  using B1 = std::integral_constant<int, 1>;
  using EY = std::integral_constant<bool, true>;
  using EN = std::integral_constant<bool, false>;
  tile_body(B0{}, EN{}, tile_lo, accE, accO);
  int tile = tile_lo + 1;
  for (;;) {
    stamp(2 + tile - tile_lo);
    if (tile >= tile_hi) {
      last_epilogue(tile - 1, accE);
      break;
    }
    tile_body(B1{}, EY{}, tile, accO, accE);
    ++tile;
    stamp(2 + tile - tile_lo);
    if (tile >= tile_hi) {
      last_epilogue(tile - 1, accO);
      break;
    }
    tile_body(B0{}, EY{}, tile, accE, accO);
    ++tile;
  }
  if constexpr (STREAM) stream_end(a, region, sl);
  if constexpr (ABL & 256) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    stamp(29);
    if (tid == 0) {
      a.trace[blockIdx.x * 32 + 30] = __builtin_amdgcn_s_memtime() - clk0;
      a.trace[blockIdx.x * 32 + 31] = (uint64_t)(tile_hi - tile_lo);
    }
  }
}

}  // namespace bb
