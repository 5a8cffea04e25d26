// scan_kernel.h — query-resident MFMA scan: the production score-slab kernel for short
// reductions (Kpad·sizeof(T) <= 1536 B: d <= 384 fp32, d <= 768 bf16).
//
// Why this shape: a cosine scan is a GEMM with a short reduction (d = 384) and few query
// rows against many item rows.  Keeping each wave's 32 query rows in VGPRs for the whole
// reduction (the MFMA B operand: 192 VGPRs fp32 / 96 bf16 at d = 384) means the only
// operand that moves is the item tile, staged once per 32 items through a double-buffered
// LDS ring and read by all 4 waves; a barrier is crossed once per 32×(4×32)×d tile
// (12.3K MFMA cycles fp32), so the global-load latency of the next tile hides entirely
// behind the current one.  Workgroups = (query group of 128) × (item chunk); chunks are
// balanced to ±1 tile and laid out XCD-aware so the groups sharing a chunk share an L2.
//
// Epilogue (identical contract to gemm_kernel.h): S row segments + per-(query, 32-item
// tile) maxima over eligible / present items for the select kernel.
#pragma once
#include "common.h"

namespace bb {

typedef float f32x16s __attribute__((ext_vector_type(16)));
typedef short bf16x8s __attribute__((ext_vector_type(8)));

constexpr int kScanWaves = 4;   // waves per workgroup, 32 queries each
constexpr int kScanRowMax = 1536;  // bytes of one padded-d row the scan kernel accepts

// chunk swizzle of row r: 16 distinct slots when a row spans a multiple of 16 chunks
template <int KU>
__device__ __forceinline__ int scan_swz(int r) {
  return (KU % 16 == 0) ? (r & 15) : (r & 7);
}

// x of lane (l ^ 32): one v_permlane32_swap (gfx950), no LDS round trip — a ds_bpermute
// here would make the next s_waitcnt lgkmcnt drain the MFMA fragment prefetch queue.
__device__ __forceinline__ uint32_t xor32(uint32_t x) {
  const auto r = __builtin_amdgcn_permlane32_swap(x, x, false, false);
  return (threadIdx.x & 32) ? r[0] : r[1];
}

// Epilogue of one 32-item tile for this lane's query: 16-B row segments of S and the
// tile maxima over eligible (present ∧ mask ∧ ¬excl) and present items.  Branch-free:
// both lane halves hold the combined maxima and store the same word.
__device__ __forceinline__ void scan_epilogue(const GemmArgs& a, float* Srow, int q, int h, int tile,
                                              const float (&v)[16], uint32_t pw, uint32_t mw, uint32_t ew) {
  const int tile0 = tile * 32;
#pragma unroll
  for (int j = 0; j < 4; ++j)
    *(float4*)(Srow + tile0 + 8 * j + 4 * h) = make_float4(v[4 * j], v[4 * j + 1], v[4 * j + 2], v[4 * j + 3]);
  const uint32_t ok = pw & mw & ~ew;
  uint32_t te = 0, tp = 0;
#pragma unroll
  for (int g = 0; g < 16; ++g) {
    const int it = (g & 3) + 8 * (g >> 2) + 4 * h;
    const uint32_t o = ord_of(v[g]);
    const bool in = tile0 + it < a.n_valid;
    const uint32_t op = (in && ((pw >> it) & 1u)) ? o : 0u;
    const uint32_t oe = (in && ((ok >> it) & 1u)) ? o : 0u;
    tp = op > tp ? op : tp;
    te = oe > te ? oe : te;
  }
  const uint32_t te2 = xor32(te), tp2 = xor32(tp);
  te = te2 > te ? te2 : te;
  tp = tp2 > tp ? tp2 : tp;
  // one store instruction: the lower half writes tmax, the upper half pmax
  if (!h || a.pmax) (h ? a.pmax : a.tmax)[(size_t)q * a.ldt + tile] = h ? tp : te;
}

// KU = Kpad·sizeof(T)/16: 16-byte chunks per row (f32: 4 k-steps each; bf16: 1 MFMA each).
// ABL: ablation bits for tools/scan_probe only (0 in the library): 1 = no epilogue
// stores, 2 = no staging after the first tile, 4 = no per-tile wait + barrier.
template <typename T, int KU, int ABL = 0>
__global__ __launch_bounds__(kScanWaves * 64, 1) void scan_kernel(GemmArgs a, int n_chunks, int tiles_total) {
  constexpr int ROWB = KU * 16;
  constexpr int TILE_B = 32 * ROWB;
  static_assert(ROWB <= kScanRowMax, "row too wide for the scan kernel");
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
  const int q = group * kScanWaves * 32 + wave * 32 + r;  // this lane's query row

  // ---- resident B operand: 16-B chunk (2u + h) of query row q, u = 0 .. KU/2-1 ----
  uint4 qf[KU / 2];
  {
    const char* qrow = (const char*)a.Q + (size_t)q * a.ldq * sizeof(T);
#pragma unroll
    for (int u = 0; u < KU / 2; ++u) qf[u] = *(const uint4*)(qrow + (2 * u + h) * 16);
  }

  // ---- item tile staging: LDS-DMA (global_load_lds_dwordx4), no VGPR round trip ----
  // The LDS image of a tile is 32 unpadded rows of ROWB bytes with the 16-B chunk index
  // XOR-swizzled by the row (chunk' = chunk ^ SW(row)), so the ds_read_b128 fragment reads
  // of 16 distinct rows at one chunk hit 16 distinct bank slots.  LDS-DMA writes lane-
  // linearly (wave base + 16·lane), so the swizzle is applied to each lane's SOURCE address
  // (cdna_hip_programming.md §5.4 rule 21).  Each wave moves KU/8 pieces of 1 KiB.
  static_assert((KU * 32 * 16) % (1024 * kScanWaves) == 0, "tile must split into whole 1 KiB pieces per wave");
  constexpr int PIECES = KU * 32 * 16 / 1024 / kScanWaves;
  const char* Xg = (const char*)a.X;
  const size_t ldxb = (size_t)a.ldx * sizeof(T);
  auto stage = [&](int tile, int buf) {
#pragma unroll
    for (int p = 0; p < PIECES; ++p) {
      const int off = (wave * PIECES + p) * 1024;          // wave-uniform LDS piece base
      const int mine = off + lane * 16;                    // this lane's LDS bytes
      const int row = mine / ROWB;
      const int chunk = ((mine % ROWB) >> 4) ^ scan_swz<KU>(row);
      const char* src = Xg + ((size_t)tile * 32 + row) * ldxb + chunk * 16;
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                       (__attribute__((address_space(3))) void*)(smem + buf * TILE_B + off),
                                       16, 0, 0);
    }
  };

  // eligibility bitsets: the host always passes valid pointers (all-ones / all-zeros
  // buffers stand in for "no mask" / "no exclusions", excl_ld = 0), so the epilogue is
  // branch-free and can live in the same basic block as the next tile's MFMA chain.
  const size_t w0 = (size_t)(a.slab_start >> 5);
  const uint32_t* erow = a.excl + (size_t)(q < a.M_valid ? q : a.M_valid - 1) * a.excl_ld;
  float* Srow = a.S + (size_t)q * a.lds;
  if (tile_lo >= tile_hi) return;  // uniform per workgroup

  stage(tile_lo, 0);
  uint32_t pw = a.present[w0 + tile_lo], mw = a.mask[w0 + tile_lo], ew = erow[w0 + tile_lo];
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // LDS-DMA landed (then the barrier)
  __syncthreads();

  // One tile's MFMA chain: 32 items (LDS buffer `buf`) × this wave's 32 resident queries.
  // Two independent accumulation chains (even / odd 16-B chunks) keep the pipe fed.
  const int swz = scan_swz<KU>(r);
  auto mfma_tile = [&](int buf, float (&out)[16]) __attribute__((always_inline)) {
    f32x16s acc0, acc1;
#pragma unroll
    for (int g = 0; g < 16; ++g) {
      acc0[g] = 0.f;
      acc1[g] = 0.f;
    }
    const char* arow = smem + buf * TILE_B + r * ROWB;
#pragma unroll
    for (int u = 0; u < KU / 2; ++u) {
      const uint4 fa = *(const uint4*)(arow + (((2 * u + h) ^ swz) << 4));
      if constexpr (sizeof(T) == 4) {
        const uint4 fb = qf[u];
        const float pa[4] = {__uint_as_float(fa.x), __uint_as_float(fa.y), __uint_as_float(fa.z),
                             __uint_as_float(fa.w)};
        const float pb[4] = {__uint_as_float(fb.x), __uint_as_float(fb.y), __uint_as_float(fb.z),
                             __uint_as_float(fb.w)};
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          if (u & 1)
            acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(pa[c], pb[c], acc1, 0, 0, 0);
          else
            acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(pa[c], pb[c], acc0, 0, 0, 0);
        }
      } else {
        if (u & 1)
          acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8s, fa),
                                                         __builtin_bit_cast(bf16x8s, qf[u]), acc1, 0, 0, 0);
        else
          acc0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8s, fa),
                                                         __builtin_bit_cast(bf16x8s, qf[u]), acc0, 0, 0, 0);
      }
    }
#pragma unroll
    for (int g = 0; g < 16; ++g) out[g] = acc0[g] + acc1[g];
  };

  // Software pipeline: iteration t runs tile t's MFMA chain and, in the same basic block,
  // tile t-1's epilogue (stores + tile maxima on registers kept from the previous
  // iteration), so that VALU work fills the MFMA issue shadows of the single wave per SIMD.
  // The first tile is peeled (no previous epilogue), keeping the loop body branch-free.
  float pv[16];
  int ptile = tile_lo;
  {
    if (!(ABL & 2) && tile_lo + 1 < tile_hi) stage(tile_lo + 1, 1);
    mfma_tile(0, pv);
    if constexpr (!(ABL & 4)) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
  }
  for (int tile = tile_lo + 1; tile < tile_hi; ++tile) {
    const int cur = (tile - tile_lo) & 1;
    // Issue order matters for the end-of-tile wait: the previous tile's epilogue stores go
    // out first, then the bitset loads, then the next tile's LDS-DMA, then a whole tile of
    // MFMAs — so by the vmcnt(0) before the barrier every one of them has long completed.
    if constexpr (!(ABL & 1)) scan_epilogue(a, Srow, q, h, ptile, pv, pw, mw, ew);
    const uint32_t npw = a.present[w0 + tile], nmw = a.mask[w0 + tile], new_ = erow[w0 + tile];
    asm volatile("" ::: "memory");
    if (!(ABL & 2) && tile + 1 < tile_hi) stage(tile + 1, cur ^ 1);  // lands while this tile computes
    float nv[16];
    mfma_tile(cur, nv);
#pragma unroll
    for (int g = 0; g < 16; ++g) pv[g] = nv[g];
    ptile = tile;
    pw = npw;
    mw = nmw;
    ew = new_;
    if constexpr (!(ABL & 4)) {
      // the next tile's LDS-DMA must have landed before any wave reads it, and every wave
      // must be done reading this buffer before the next iteration re-stages it
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
  }
  if (!(ABL & 1)) scan_epilogue(a, Srow, q, h, ptile, pv, pw, mw, ew);
#pragma unroll
  for (int g = 0; g < 16; ++g) asm volatile("" ::"v"(pv[g]));
}

}  // namespace bb
