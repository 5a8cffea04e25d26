// gemm.hip — S = Q̂ · X̂ᵀ score slabs on MFMA (gfx950), with the selection bound fused in.
//
// The dense contraction behind every scoring mode: sklearn cosine_similarity's
// safe_sparse_dot(X̂, Ŷᵀ) (recommendation_system.py:214), the CF np.dot(u, Fᵀ) (:438) and
// pgvector's sequential-scan dot products (lego_nlp_recommeder.py:1394).  Both operands are
// row-major with the reduction dimension contiguous ("NT"), rows padded with zeros.
//
// Structure (gemm_kernel.h): one workgroup = WM×WN waves, each wave owns SM×SN 32×32
// output tiles.  Operands are staged global -> registers -> LDS (double buffer, one barrier
// per k-tile; the next tile's global loads are issued before the MFMAs of the current one).
// A k-tile is 128 bytes of every row (32 f32 / 64 bf16); LDS rows are padded to 144 B so
// the 16-B fragment reads (ds_read_b128) of 16 rows hit 16 distinct bank slots.
//
// Fragment mapping.  The MFMA reduction index may be permuted freely as long as A and B
// use the same permutation, so lane half h reads the contiguous 16-B chunk 2u+h of its row:
//   f32  v_mfma_f32_32x32x2_f32 : one chunk = 4 k-steps (element c of lane half h is
//                                 d = 8u + 4h + c), exact f32 fmaf chain
//   bf16 v_mfma_f32_32x32x16_bf16: one chunk = one MFMA (k = 8h + j), f32 accumulate
// A = items, B = queries: accumulator register g of lane l is item (g&3)+8(g>>2)+4(l>>5)
// of query l&31, so the epilogue stores 16-B row segments of S and reduces each query's
// per-32-item-tile maximum over eligible items with one cross-half swap.  Those maxima let
// the select kernel bound the K-th score from ~N/32 values and read only the ~K tiles that
// can hold a top-K member (select.hip).
#include <cstdlib>

#include "gemm_kernel.h"
#include "scan3_kernel.h"
#include "list_epi.h"

namespace bb {

// production tile configurations: WM×WN waves, SM×SN 32×32 tiles per wave
struct CfgF32 {
  static constexpr int WM = 2, WN = 2, SM = 1, SN = 1;  // 64 items × 64 queries
};
struct CfgBF16 {
  static constexpr int WM = 2, WN = 2, SM = 2, SN = 2;  // 128 items × 128 queries
};

int gemm_tile_m(int dtype) {  // queries per block (Mpad multiple)
  return dtype == BF16 ? CfgBF16::WN * CfgBF16::SN * 32 : CfgF32::WN * CfgF32::SN * 32;
}
int gemm_tile_n(int dtype) {  // items per block (Ncols multiple)
  return dtype == BF16 ? CfgBF16::WM * CfgBF16::SM * 32 : CfgF32::WM * CfgF32::SM * 32;
}
int gemm_tile_k(int dtype) { return dtype == BF16 ? 64 : 32; }

template <typename T, int KU>
static void launch_scan_t(const GemmArgs& a, hipStream_t s) {
  if constexpr (sizeof(T) == 2) {
    if (scan4_used(BF16, a.Mpad)) {
      launch_scan4(a, KU, s);
      return;
    }
  }
  const int n_groups = a.Mpad / (kScanWaves * 32);
  const int tiles = a.Ncols / 32;
  // one workgroup per CU (LDS + VGPR budget): ~256 workgroups, chunks balanced to ±1 tile
  // (list scans: kScanListWg, common.h — the host's list geometry uses the same count)
  const int n_chunks = scan_n_chunks(a.Mpad, tiles, a.lists ? kScanListWg : 256);
  if constexpr (sizeof(T) == 2 && KU <= kRrMaxD / 8) {
    // the exact re-rank path: the f16 copy of an f32 index (launch_gemm checked a.f16)
    if (a.lists) {  // bounded candidate lists
      bb_launch((scan2_kernel<T, KU, kScanList | kScanF16>), dim3(n_groups * n_chunks), dim3(kScanWaves * 64),
                         0, s, a, n_chunks, tiles);
      return;
    }
    if (a.s_h && !a.cand) {  // int16 score image
      bb_launch((scan2_kernel<T, KU, kScanS16 | kScanF16>), dim3(n_groups * n_chunks), dim3(kScanWaves * 64),
                         0, s, a, n_chunks, tiles);
      return;
    }
    if (a.f16) {  // f32 score slab
      bb_launch((scan2_kernel<T, KU, kScanF16>), dim3(n_groups * n_chunks), dim3(kScanWaves * 64), 0, s, a,
                         n_chunks, tiles);
      return;
    }
  }
  if (a.cand)
    bb_launch((scan2_kernel<T, KU, kScanStream>), dim3(n_groups * n_chunks), dim3(kScanWaves * 64), 0, s, a,
                       n_chunks, tiles);
  else
    bb_launch((scan2_kernel<T, KU>), dim3(n_groups * n_chunks), dim3(kScanWaves * 64), 0, s, a, n_chunks,
                       tiles);
}

template <typename T>
static bool launch_scan(const GemmArgs& a, hipStream_t s) {
  const int ku = (int)(a.Kpad * sizeof(T) / 16);
  switch (ku) {
    case 8: launch_scan_t<T, 8>(a, s); return true;
    case 16: launch_scan_t<T, 16>(a, s); return true;
    case 24: launch_scan_t<T, 24>(a, s); return true;
    case 32: launch_scan_t<T, 32>(a, s); return true;
    case 48: launch_scan_t<T, 48>(a, s); return true;
    case 64: launch_scan_t<T, 64>(a, s); return true;
    case 96: launch_scan_t<T, 96>(a, s); return true;
    default: return false;
  }
}

bool scan_supported(int dtype, int Kpad) {
  const int ku = Kpad * (dtype == BF16 ? 2 : 4) / 16;
  return ku == 8 || ku == 16 || ku == 24 || ku == 32 || ku == 48 || ku == 64 || ku == 96;
}

bool scan3_supported(int Mpad, int Kpad) {
  const int kp = Kpad * 2 / 16;
  return Mpad % (kScanWaves * 32) == 0 && Kpad % 8 == 0 && kp % 8 == 0 && kp >= 8 && kp <= kScan3MaxKP &&
         !ab_env("BB_NO_SPLIT");
}

template <int KP>
static void launch_scan3_t(const GemmArgs& a, hipStream_t s) {
  const int n_groups = a.Mpad / (kScanWaves * 32);
  const int tiles = a.Ncols / 32;
  const int n_chunks = scan_n_chunks(a.Mpad, tiles);
  if (a.cand)
    bb_launch((scan3_kernel<KP, kScanStream>), dim3(n_groups * n_chunks), dim3(kScanWaves * 64), 0, s, a,
                       n_chunks, tiles);
  else
    bb_launch((scan3_kernel<KP>), dim3(n_groups * n_chunks), dim3(kScanWaves * 64), 0, s, a, n_chunks, tiles);
}

hipError_t launch_scan3(const GemmArgs& a, hipStream_t s) {
  // queries only as the prep kernel's q3f image: no fused gather / raw-row prologue here
  if (!scan3_supported(a.Mpad, a.Kpad) || a.Ncols % 32 || (a.slab_start & 31) || a.q_ids || a.q_src)
    return hipErrorInvalidValue;
  switch (a.Kpad * 2 / 16) {
    case 8: launch_scan3_t<8>(a, s); break;
    case 16: launch_scan3_t<16>(a, s); break;
    case 24: launch_scan3_t<24>(a, s); break;
    case 32: launch_scan3_t<32>(a, s); break;
    case 40: launch_scan3_t<40>(a, s); break;
    case 48: launch_scan3_t<48>(a, s); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

bool gemm_uses_scan(int dtype, int Mpad, int Kpad) {
  return Mpad % (kScanWaves * 32) == 0 && scan_supported(dtype, Kpad) && !ab_env("BB_FORCE_TILED_GEMM");
}

hipError_t launch_gemm(int dtype, const GemmArgs& a, hipStream_t s) {
  const int bm = gemm_tile_m(dtype), bn = gemm_tile_n(dtype), bk = gemm_tile_k(dtype);
  if (a.Mpad % bm || a.Ncols % bn || a.Kpad % bk || a.Mpad <= 0 || a.Ncols <= 0 || (a.slab_start & 31))
    return hipErrorInvalidValue;
  // f16 operands (the re-rank copy): 16-bit scans of rows up to kRrMaxD, no streaming; the
  // int16 image and the lists exist on that copy only
  if ((a.f16 && (dtype != BF16 || !gemm_uses_scan(dtype, a.Mpad, a.Kpad) || a.Kpad > kRrMaxD || a.cand ||
                 a.pilot_top)) ||
      (!a.f16 && (a.s_h || a.lists || a.q_istats)))
    return hipErrorInvalidValue;
  // the fused re-rank prologue lives in scan2 (16-bit, query chunks of <= 128 rows) only
  if (a.q_istats && !a.q_raw && (dtype != BF16 || scan4_used(BF16, a.Mpad) || !a.q_f32_out || !a.q_eps_out || a.cand))
    return hipErrorInvalidValue;
  // the raw-query prologue: scan2 (bf16) with the list epilogue, raw f32 rows (d % 4 == 0)
  if (a.q_raw && (dtype != BF16 || scan4_used(BF16, a.Mpad) || !a.lists || !a.q_src || a.q_ids || !a.q_istats ||
                  !a.q_h_out || !a.q_eps_out || a.cand || a.q_d <= 0 || (a.q_d & 3) || a.q_d > a.Kpad || a.q_src_ld < a.q_d))
    return hipErrorInvalidValue;
  // the int16 score image: bf16 scans of rows up to kRrMaxD, slab epilogue only
  if (a.s_h && (dtype != BF16 || a.cand || !gemm_uses_scan(dtype, a.Mpad, a.Kpad) || a.Kpad > kRrMaxD))
    return hipErrorInvalidValue;
  // candidate lists: the bf16 scans of a re-rank search (rows up to kRrMaxD wide), periods of
  // at most kListMaxPeriod tiles covering every chunk
  if (a.lists && (!a.s_h || (a.q_istats && !a.q_raw) || a.cand || a.l_period <= 0 || a.l_period > kListMaxPeriod || a.l_np <= 0 ||
                  (int64_t)a.l_period * a.l_np * scan_chunks(BF16, a.Mpad, a.Ncols / 32, false, a.Kpad * 2 / 16) < a.Ncols / 32))
    return hipErrorInvalidValue;
  // the streaming pilot's top-m maxima: scan4 (bf16), slab mode, no other epilogue output
  if (a.pilot_top && (dtype != BF16 || !scan4_used(BF16, a.Mpad) || !gemm_uses_scan(dtype, a.Mpad, a.Kpad) || a.cand ||
                      a.lists || a.s_h || a.pilot_m != scan4_pilot_m(a.Kpad)))
    return hipErrorInvalidValue;
  // the lane-order query operand: scan4's (q_perm 1) or scan2's (2), prepped rows (no fused
  // query prologue), bf16
  if (a.q_perm && (dtype != BF16 || a.q_perm != (scan4_used(BF16, a.Mpad) ? 1 : 2) || !gemm_uses_scan(dtype, a.Mpad, a.Kpad) ||
                   a.q_ids || a.q_src || a.Kpad % 16))
    return hipErrorInvalidValue;
  if (gemm_uses_scan(dtype, a.Mpad, a.Kpad)) {
    if (dtype == BF16 ? launch_scan<uint16_t>(a, s) : launch_scan<float>(a, s)) return hipGetLastError();
  }
  // the fused query prologue and the streaming epilogue are scan-only
  if (a.q_ids || a.q_src || a.cand) return hipErrorInvalidValue;
  const int blocks = (a.Mpad / bm) * (a.Ncols / bn);
  if (dtype == BF16) {
    constexpr int nt = CfgBF16::WM * CfgBF16::WN * 64;
    bb_launch((gemm_nt_kernel<uint16_t, CfgBF16::WM, CfgBF16::WN, CfgBF16::SM, CfgBF16::SN>),
                       dim3(blocks), dim3(nt), 0, s, a);
  } else {
    constexpr int nt = CfgF32::WM * CfgF32::WN * 64;
    bb_launch((gemm_nt_kernel<float, CfgF32::WM, CfgF32::WN, CfgF32::SM, CfgF32::SN>), dim3(blocks),
                       dim3(nt), 0, s, a);
  }
  return hipGetLastError();
}

}  // namespace bb
