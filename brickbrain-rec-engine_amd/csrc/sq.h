// sq.h — small-batch exact search (sq.hip): the arguments shared by api.hip and the kernels.
//
// B <= kSqMaxB query rows of one side against an f32 index (that has its f16 copy): ONE
// approximate pass over the f16 rows on the matrix cores (f16 rows x f16 hi + lo query
// split, f32 accumulation) — every approximate score a within a proven δ of the exact score s (the f32 products summed in f64 in rescore_rows' fixed order, rounded to
// f32) — leaves per workgroup and query its top kSqM approximate keys (and present keys for the
// rank-0 drop) and every row's approximate order image; the merge (one workgroup per query and
// side) takes the candidates within 2δ of a lower bound of the K-th score, rescores exactly
// those from the f32 rows, and emits the exact top-K with the same bits as every other path.
#pragma once
#include "common.h"

namespace bb {

constexpr int kSqMaxB = 16;
constexpr int kSqMaxK = 128;    // internal list length (K_int) the merge sorts in registers
constexpr int kSqM = 4;         // keys per workgroup list
constexpr int kSqMaxRows = 128; // rows per workgroup
constexpr int kSqMaxWg = 512;   // workgroups (8 lists per merge lane): n <= 65,536
constexpr int kSqCand = 256;    // eligible candidates per query the merge sorts (beyond: the slow exact path)
constexpr int kSqPCand = 64;    // rank-0 candidates per query (beyond: the slow exact path)

struct SqArgs {
  const uint16_t* Xb;       // f16 rows [n][ldb] (the index's round-to-nearest copy, zero padded)
  int64_t ldb;
  const float* X;           // f32 rows [n][ldx], normalised, zero padded: the exact rescore
  int64_t ldx;
  const float* stats;       // rr_stats of the side: max |x̃−x|, max |x|, max |x̃| over the rows
  int32_t n;
  uint32_t gid0;            // global id of row 0
  const uint32_t* present;  // local-row bitsets: the side's item space,
  const uint32_t* mask;     //   the constraint mask (all ones: none),
  const uint32_t* excl;     //   per-query exclusions [B][excl_ld] (none: all zeros, excl_ld 0)
  int64_t excl_ld;
  int32_t drop;             // rank-0 drop: keep the present candidates too
  int32_t B;
  // queries: q_kind 0 = raw rows q_src (q_dtype, stride q_ld, width q_d): the pass scores
  // them as given (times a power-of-two scale), the merge rescores them normalised as
  // prep_kernel does (qnorm.h); 1 = the stored f32 rows of ids q_ids (minus q_id_offset) of X;
  // 2 = q_src rows as they are (CF user factors)
  int32_t q_kind;
  const void* q_src;
  int32_t q_dtype;
  int64_t q_ld;
  int32_t q_d;
  const int64_t* q_ids;
  int64_t q_id_offset;
  int32_t rpw, nwg;         // rows per workgroup (multiple of 4), workgroups
  uint64_t* wg_top;         // [B][nwg][kSqM] eligible approximate keys (0 = empty)
  uint64_t* wg_ptop;        // [B][nwg][kSqM] present approximate keys (drop)
  uint32_t* ords;           // [B][ords_ld] eligible approximate order image per row, 0 = ineligible
  uint32_t* ords_p;         // [B][ords_ld] present approximate order image (drop)
  int64_t ords_ld;
  int32_t K;                // internal list length
  int32_t k_final;          // final outputs (out_scores != null) ...
  float* out_scores;
  int64_t* out_ids;
  int32_t* out_counts;
  uint64_t* keys_out;       // ... or the exact key list [B][K] + max_out [B] (BB_Q_OUT_KEYS, hybrid
  uint64_t* max_out;        //     sides; max_out null: not written)
  int32_t mopt;             // merge variants (BB_SQ_MOPT A/B runs; default 3): 1 = lists by nwg, early exit; 2 = rank emission
  uint64_t* trace;          // probe runs (BB_SQ_TRACE): pass phase stamps [nwg][8], or null
  uint64_t* mtrace;         //   and merge phase stamps [B][8] of this side, or null
};

// the approximate pass, then the merge (a1 != null: both hybrid sides in one launch)
hipError_t launch_sq_scan(const SqArgs& a, hipStream_t s);
hipError_t launch_sq_merge(const SqArgs& a0, const SqArgs* a1, hipStream_t s);

}  // namespace bb
