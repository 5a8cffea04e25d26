// gemm.hip — S = Q̂ · X̂ᵀ score slabs on MFMA (gfx950).
//
// The dense contraction behind every scoring mode: sklearn cosine_similarity's
// safe_sparse_dot(X̂, Ŷᵀ) (recommendation_system.py:214), the CF np.dot(u, Fᵀ) (:438) and
// pgvector's sequential-scan dot products (lego_nlp_recommeder.py:1394).  Both operands are
// row-major with the reduction dimension contiguous ("NT"), rows padded with zeros.
//
// Structure: one workgroup = WM×WN waves, each wave owns SM×SN 32×32 output tiles.
// Operands are staged global -> registers -> LDS (double buffer, one barrier per k-tile;
// the next tile's global loads are issued before the MFMAs of the current one).  A k-tile is
// 128 bytes of every row (32 f32 / 64 bf16); LDS rows are padded to 144 B so the 16-B
// fragment reads (ds_read_b128) of 16 rows hit 16 distinct bank slots.
//
// Fragment mapping.  The MFMA reduction index may be permuted freely as long as A and B
// use the same permutation, so lane half h reads the contiguous 16-B chunk 2u+h of its row:
//   f32  v_mfma_f32_32x32x2_f32 : one chunk = 4 k-steps (element c of lane half h is
//                                 d = 8u + 4h + c), exact f32 fmaf chain
//   bf16 v_mfma_f32_32x32x16_bf16: one chunk = one MFMA (k = 8h + j), f32 accumulate
// Accumulator C/D layout (gfx950): col = lane & 31, row = (g&3) + 8(g>>2) + 4(lane>>5).
// A = queries (rows of S), B = items (columns of S): each epilogue store of a register is
// 32 consecutive item scores of one query row (128-B segments).
#include "gemm_kernel.h"

namespace bb {

// production tile configurations
struct CfgF32 {
  static constexpr int WM = 2, WN = 2, SM = 1, SN = 1;  // 64 x 64 block tile
};
struct CfgBF16 {
  static constexpr int WM = 2, WN = 2, SM = 2, SN = 2;  // 128 x 128 block tile
};

int gemm_tile_m(int dtype) {
  return dtype == BF16 ? CfgBF16::WM * CfgBF16::SM * 32
                       : CfgF32::WM * CfgF32::SM * 32;
}
int gemm_tile_n(int dtype) {
  return dtype == BF16 ? CfgBF16::WN * CfgBF16::SN * 32
                       : CfgF32::WN * CfgF32::SN * 32;
}
int gemm_tile_k(int dtype) { return dtype == BF16 ? 64 : 32; }

hipError_t launch_gemm(int dtype, const GemmArgs& a, hipStream_t s) {
  const int bm = gemm_tile_m(dtype), bn = gemm_tile_n(dtype), bk = gemm_tile_k(dtype);
  if (a.Mpad % bm || a.Ncols % bn || a.Kpad % bk || a.Mpad <= 0 || a.Ncols <= 0) return hipErrorInvalidValue;
  const int blocks = (a.Mpad / bm) * (a.Ncols / bn);
  if (dtype == BF16) {
    constexpr int nt = CfgBF16::WM * CfgBF16::WN * 64;
    hipLaunchKernelGGL((gemm_nt_kernel<uint16_t, CfgBF16::WM, CfgBF16::WN, CfgBF16::SM, CfgBF16::SN>), dim3(blocks), dim3(nt), 0, s, a);
  } else {
    constexpr int nt = CfgF32::WM * CfgF32::WN * 64;
    hipLaunchKernelGGL((gemm_nt_kernel<float, CfgF32::WM, CfgF32::WN, CfgF32::SM, CfgF32::SN>), dim3(blocks), dim3(nt), 0, s, a);
  }
  return hipGetLastError();
}

}  // namespace bb
