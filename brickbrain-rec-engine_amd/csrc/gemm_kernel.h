// gemm_kernel.h — the MFMA score-slab kernel template (included by gemm.hip and the tile
// micro-benchmark in tools/).  See gemm.hip for the design notes.
#pragma once
#include "common.h"

namespace bb {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short bf16x8 __attribute__((ext_vector_type(8)));

// T = float or uint16_t (bf16 bits); WM×WN waves per workgroup; each wave owns SM×SN
// 32×32 output tiles.  A operand = ITEMS (rows of the MFMA output), B operand = QUERIES
// (columns), so in the accumulator a lane holds 16 item scores of ONE query:
//   query = lane & 31 (+ tile col), item = (g&3) + 8(g>>2) + 4(lane>>5) (+ tile row).
// ROWB = bytes of every operand row staged per k-tile (128 or 256).
template <typename T, int WM, int WN, int SM, int SN, int ROWB = 128>
__global__ __launch_bounds__(WM* WN * 64) void gemm_nt_kernel(GemmArgs a) {
  constexpr int NT = WM * WN * 64;
  constexpr int BI = WM * SM * 32, BQ = WN * SN * 32;  // items × queries per workgroup
  constexpr int BK = ROWB / (int)sizeof(T);  // elements per k-tile
  constexpr int STRIDE = ROWB + 16;          // padded LDS row -> conflict-free ds_read_b128
  constexpr int CH = ROWB / 16;              // 16-B chunks per row
  constexpr int LX = BI * CH / NT;           // 16-B loads per thread per k-tile (items)
  constexpr int LQ = BQ * CH / NT;           //                                  (queries)
  static_assert(LQ * NT == BQ * CH && LX * NT == BI * CH, "tile/thread mismatch");
  constexpr int BUF = (BI + BQ) * STRIDE;
  __shared__ __attribute__((aligned(16))) char smem[2 * BUF];

  // XCD-aware, bijective block -> tile remap: the workgroups that share an item panel
  // (same bi, different query blocks) are consecutive in t and fall in one XCD group, so
  // the panel is fetched from HBM/MALL once per XCD and re-read from that XCD's L2
  // (speed only; any placement is correct).
  const int nbq = a.Mpad / BQ, nbi = a.Ncols / BI;
  const int total = nbq * nbi;
  const int L = blockIdx.x;
  const int xcd = L & 7, local = L >> 3, q8 = total >> 3, r8 = total & 7;
  const int t = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + local;
  const int bi = t / nbq, bq = t - bi * nbq;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int r = lane & 31, h = lane >> 5;

  const char* Xg = (const char*)a.X + (size_t)bi * BI * a.ldx * sizeof(T);
  const char* Qg = (const char*)a.Q + (size_t)bq * BQ * a.ldq * sizeof(T);
  const size_t ldxb = (size_t)a.ldx * sizeof(T), ldqb = (size_t)a.ldq * sizeof(T);

  // staging as plain unrolled loops (no lambdas) so rx / rq stay in VGPRs
  uint4 rx[LX], rq[LQ];
#define BB_GEMM_GLOAD(kt_)                                                          \
  {                                                                                 \
    _Pragma("unroll") for (int i = 0; i < LX; ++i) {                                \
      const int c = tid + i * NT, row = c / CH, ch = c % CH;                        \
      rx[i] = *(const uint4*)(Xg + row * ldxb + (size_t)(kt_) * ROWB + ch * 16);    \
    }                                                                               \
    _Pragma("unroll") for (int i = 0; i < LQ; ++i) {                                \
      const int c = tid + i * NT, row = c / CH, ch = c % CH;                        \
      rq[i] = *(const uint4*)(Qg + row * ldqb + (size_t)(kt_) * ROWB + ch * 16);    \
    }                                                                               \
  }
#define BB_GEMM_LSTORE(buf_)                                                        \
  {                                                                                 \
    char* lb_ = smem + (buf_) * BUF;                                                \
    _Pragma("unroll") for (int i = 0; i < LX; ++i) {                                \
      const int c = tid + i * NT, row = c / CH, ch = c % CH;                        \
      *(uint4*)(lb_ + row * STRIDE + ch * 16) = rx[i];                              \
    }                                                                               \
    _Pragma("unroll") for (int i = 0; i < LQ; ++i) {                                \
      const int c = tid + i * NT, row = c / CH, ch = c % CH;                        \
      *(uint4*)(lb_ + (BI + row) * STRIDE + ch * 16) = rq[i];                       \
    }                                                                               \
  }

  f32x16 acc[SM][SN];
#pragma unroll
  for (int m = 0; m < SM; ++m)
#pragma unroll
    for (int n = 0; n < SN; ++n)
#pragma unroll
      for (int g = 0; g < 16; ++g) acc[m][n][g] = 0.f;

  const int nk = a.Kpad / BK;
  BB_GEMM_GLOAD(0);
  BB_GEMM_LSTORE(0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) BB_GEMM_GLOAD(kt + 1);
    const char* base = smem + cur * BUF;
#pragma unroll
    for (int u = 0; u < CH / 2; ++u) {
      uint4 fa[SM], fb[SN];
#pragma unroll
      for (int m = 0; m < SM; ++m)
        fa[m] = *(const uint4*)(base + (wm * SM * 32 + m * 32 + r) * STRIDE + (2 * u + h) * 16);
#pragma unroll
      for (int n = 0; n < SN; ++n)
        fb[n] = *(const uint4*)(base + (BI + wn * SN * 32 + n * 32 + r) * STRIDE + (2 * u + h) * 16);
#pragma unroll
      for (int m = 0; m < SM; ++m)
#pragma unroll
        for (int n = 0; n < SN; ++n) {
          if constexpr (sizeof(T) == 4) {
            const float* pa = (const float*)&fa[m];
            const float* pb = (const float*)&fb[n];
#pragma unroll
            for (int c = 0; c < 4; ++c)
              acc[m][n] = __builtin_amdgcn_mfma_f32_32x32x2f32(pa[c], pb[c], acc[m][n], 0, 0, 0);
          } else {
            acc[m][n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, fa[m]),
                                                                __builtin_bit_cast(bf16x8, fb[n]),
                                                                acc[m][n], 0, 0, 0);
          }
        }
    }
    if (kt + 1 < nk) BB_GEMM_LSTORE(cur ^ 1);
    __syncthreads();
  }

  // ---- epilogue: scores + per-(query, 32-item tile) maxima for the selection bound ----
  // Lane owns query q; registers g = 4j..4j+3 are 4 consecutive items 8j+4h+0..3, stored
  // as one 16-B row segment.  tmax = max order-image over ELIGIBLE items of the tile
  // (present ∧ mask ∧ ¬excl, 0 if none); pmax = max over PRESENT items (rank-0 search).
#pragma unroll
  for (int n = 0; n < SN; ++n) {
    const int q = bq * BQ + wn * SN * 32 + n * 32 + r;
    float* Srow = a.S + (size_t)q * a.lds;
#pragma unroll
    for (int m = 0; m < SM; ++m) {
      const int tile0 = bi * BI + wm * SM * 32 + m * 32;  // first item (slab column) of the tile
#pragma unroll
      for (int j = 0; j < 4; ++j)
        *(float4*)(Srow + tile0 + 8 * j + 4 * h) =
            make_float4(acc[m][n][4 * j], acc[m][n][4 * j + 1], acc[m][n][4 * j + 2], acc[m][n][4 * j + 3]);
      if (a.tmax) {
        const int64_t w = (a.slab_start + tile0) >> 5;  // tile0 is a multiple of 32
        const uint32_t pw = a.present ? a.present[w] : ~0u;
        const uint32_t mw = a.mask ? a.mask[w] : ~0u;
        const uint32_t ew = (a.excl && q < a.M_valid) ? a.excl[(size_t)q * a.excl_ld + w] : 0u;
        uint32_t te = 0, tp = 0;
#pragma unroll
        for (int g = 0; g < 16; ++g) {
          const int it = (g & 3) + 8 * (g >> 2) + 4 * h;  // item within the tile
          const bool pr = tile0 + it < a.n_valid && ((pw >> it) & 1u);
          const uint32_t o = ord_of(acc[m][n][g]);
          const uint32_t op = pr ? o : 0u;
          const uint32_t oe = (pr && ((mw >> it) & 1u) && !((ew >> it) & 1u)) ? o : 0u;
          tp = op > tp ? op : tp;
          te = oe > te ? oe : te;
        }
        const uint32_t te2 = __shfl_xor(te, 32), tp2 = __shfl_xor(tp, 32);
        te = te2 > te ? te2 : te;
        tp = tp2 > tp ? tp2 : tp;
        if (h == 0) {
          a.tmax[(size_t)q * a.ldt + (tile0 >> 5)] = te;
          if (a.pmax) a.pmax[(size_t)q * a.ldt + (tile0 >> 5)] = tp;
        }
      }
    }
  }
}

#undef BB_GEMM_GLOAD
#undef BB_GEMM_LSTORE

}  // namespace bb
