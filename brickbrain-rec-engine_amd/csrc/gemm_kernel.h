// gemm_kernel.h — the MFMA score-slab kernel template (included by gemm.hip and the
// tile micro-benchmark in tools/).  See gemm.hip for the design notes.
#pragma once
#include "common.h"

namespace bb {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short bf16x8 __attribute__((ext_vector_type(8)));

// T = float or uint16_t (bf16 bits); WM×WN waves per workgroup, SM×SN 32×32 tiles per wave.
template <typename T, int WM, int WN, int SM, int SN>
__global__ __launch_bounds__(WM* WN * 64) void gemm_nt_kernel(GemmArgs a) {
  constexpr int NT = WM * WN * 64;
  constexpr int BM = WM * SM * 32, BN = WN * SN * 32;
  constexpr int ROWB = 128;                  // bytes of one row per k-tile
  constexpr int BK = ROWB / (int)sizeof(T);  // elements per k-tile
  constexpr int STRIDE = ROWB + 16;          // padded LDS row
  constexpr int CH = ROWB / 16;              // 16-B chunks per row
  constexpr int LQ = BM * CH / NT;           // 16-B loads per thread per k-tile (Q)
  constexpr int LX = BN * CH / NT;           //                                   (X)
  static_assert(LQ * NT == BM * CH && LX * NT == BN * CH, "tile/thread mismatch");
  constexpr int BUF = (BM + BN) * STRIDE;
  __shared__ __attribute__((aligned(16))) char smem[2 * BUF];

  // XCD-aware, bijective block -> tile remap: tiles that share an item panel (same bn)
  // are consecutive in t and land in one XCD group, so the panel is read from HBM/MALL
  // once per XCD and re-read from that XCD's L2 (speed only; any placement is correct).
  const int nbm = a.Mpad / BM, nbn = a.Ncols / BN;
  const int total = nbm * nbn;
  const int L = blockIdx.x;
  const int xcd = L & 7, local = L >> 3, q8 = total >> 3, r8 = total & 7;
  const int t = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + local;
  const int bn = t / nbm, bm = t - bn * nbm;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int r = lane & 31, h = lane >> 5;

  const char* Qg = (const char*)a.Q + (size_t)bm * BM * a.ldq * sizeof(T);
  const char* Xg = (const char*)a.X + (size_t)bn * BN * a.ldx * sizeof(T);
  const size_t ldqb = (size_t)a.ldq * sizeof(T), ldxb = (size_t)a.ldx * sizeof(T);

  uint4 rq[LQ], rx[LX];
  auto gload = [&](int kt) {
#pragma unroll
    for (int i = 0; i < LQ; ++i) {
      const int c = tid + i * NT, row = c / CH, ch = c % CH;
      rq[i] = *(const uint4*)(Qg + row * ldqb + (size_t)kt * ROWB + ch * 16);
    }
#pragma unroll
    for (int i = 0; i < LX; ++i) {
      const int c = tid + i * NT, row = c / CH, ch = c % CH;
      rx[i] = *(const uint4*)(Xg + row * ldxb + (size_t)kt * ROWB + ch * 16);
    }
  };
  auto lstore = [&](int buf) {
    char* base = smem + buf * BUF;
#pragma unroll
    for (int i = 0; i < LQ; ++i) {
      const int c = tid + i * NT, row = c / CH, ch = c % CH;
      *(uint4*)(base + row * STRIDE + ch * 16) = rq[i];
    }
#pragma unroll
    for (int i = 0; i < LX; ++i) {
      const int c = tid + i * NT, row = c / CH, ch = c % CH;
      *(uint4*)(base + (BM + row) * STRIDE + ch * 16) = rx[i];
    }
  };

  f32x16 acc[SM][SN];
#pragma unroll
  for (int m = 0; m < SM; ++m)
#pragma unroll
    for (int n = 0; n < SN; ++n)
#pragma unroll
      for (int g = 0; g < 16; ++g) acc[m][n][g] = 0.f;

  const int nk = a.Kpad / BK;
  gload(0);
  lstore(0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) gload(kt + 1);
    const char* base = smem + cur * BUF;
#pragma unroll
    for (int u = 0; u < CH / 2; ++u) {
      uint4 fa[SM], fb[SN];
#pragma unroll
      for (int m = 0; m < SM; ++m)
        fa[m] = *(const uint4*)(base + (wm * SM * 32 + m * 32 + r) * STRIDE + (2 * u + h) * 16);
#pragma unroll
      for (int n = 0; n < SN; ++n)
        fb[n] = *(const uint4*)(base + (BM + wn * SN * 32 + n * 32 + r) * STRIDE + (2 * u + h) * 16);
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
            bf16x8 va = __builtin_bit_cast(bf16x8, fa[m]);
            bf16x8 vb = __builtin_bit_cast(bf16x8, fb[n]);
            acc[m][n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(va, vb, acc[m][n], 0, 0, 0);
          }
        }
    }
    if (kt + 1 < nk) lstore(cur ^ 1);
    __syncthreads();
  }

  // epilogue: register g of tile (m, n) -> S[query row][item col]
#pragma unroll
  for (int m = 0; m < SM; ++m)
#pragma unroll
    for (int n = 0; n < SN; ++n) {
      const size_t col = (size_t)bn * BN + wn * SN * 32 + n * 32 + r;
#pragma unroll
      for (int g = 0; g < 16; ++g) {
        const size_t row = (size_t)bm * BM + wm * SM * 32 + m * 32 + (g & 3) + 8 * (g >> 2) + 4 * h;
        a.S[row * a.lds + col] = acc[m][n][g];
      }
    }
}

}  // namespace bb
