// common.h — shared device/host definitions of libbrickrec (gfx950 / CDNA4 only).
#pragma once
#include <cstdlib>
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stdint.h>

#include <cstring>
#include <type_traits>
#include <vector>

namespace bb {

// A/B and probe switches (BB_NO_RR, BB_S16, BB_DUAL, BB_SELECT_TRACE, ...): read only when
// BB_AB is set in the environment, so a production process is immune to stray variables;
// tools/gpu_run.sh sets it for its A/B runs.  Defaults are the measured best.
inline const char* ab_env(const char* name) {
  static const bool on = std::getenv("BB_AB") != nullptr;
  return on ? std::getenv(name) : nullptr;
}
// Probe builds only (make PROBES=1): the phase-stamp trace printers (BB_SQ_TRACE,
// BB_SCAN_TRACE, BB_SELECT_TRACE, BB_STREAM_DEBUG).  The shipped library is built with
// kProbes = false, so each printer's guard is a constant and the code is not emitted.
#ifndef BB_PROBES
#define BB_PROBES 0
#endif
constexpr bool kProbes = BB_PROBES != 0;

// ---- item ordering keys ------------------------------------------------------------------
// A candidate is one u64: high word = order-preserving image of the fp32 score, low word =
// 0xFFFFFFFF - global id.  "larger key" == (score desc, id asc), the fixed tie rule of
// SURVEY.md §8a(v).  Key 0 (ord 0 = the image of -NaN 0xFFFFFFFF) marks an empty slot;
// every non-NaN float maps to ord >= 0x007FFFFF, so real candidates are never 0.
__host__ __device__ inline uint32_t ord_of(float f) {
  uint32_t u = __builtin_bit_cast(uint32_t, f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__host__ __device__ inline float float_of_ord(uint32_t o) {
  uint32_t u = (o & 0x80000000u) ? (o & 0x7FFFFFFFu) : ~o;
  return __builtin_bit_cast(float, u);
}
__host__ __device__ inline uint64_t make_key(uint32_t ord, uint32_t gid) {
  return ((uint64_t)ord << 32) | (uint32_t)(0xFFFFFFFFu - gid);
}
__host__ __device__ inline uint32_t gid_of(uint64_t key) { return 0xFFFFFFFFu - (uint32_t)key; }
__host__ __device__ inline uint32_t ordk_of(uint64_t key) { return (uint32_t)(key >> 32); }

// round-to-nearest-even f32 -> bf16 (NaN kept NaN)
__device__ __forceinline__ uint16_t to_bf16(float f) {
  uint32_t u = __builtin_bit_cast(uint32_t, f);
  if ((u & 0x7F800000u) == 0x7F800000u && (u & 0x7FFFFFu)) return (uint16_t)((u >> 16) | 0x40);
  u += 0x7FFFu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

// round-to-nearest-even f32 -> f16, saturating to ±65504 (the re-rank copy of an f32 index
// and its query operands: every bound is computed from the rounded values, so a saturated
// element only widens it; NaN kept NaN)
__device__ __forceinline__ uint16_t to_f16(float f) {
  const float c = f == f ? fminf(fmaxf(f, -65504.f), 65504.f) : f;
  return __builtin_bit_cast(uint16_t, (_Float16)c);
}
__device__ __forceinline__ float f16_val(uint16_t h) { return (float)__builtin_bit_cast(_Float16, h); }

// γ per unit of row width: the f32 accumulation error of the approximate scans' 32x32x16
// MFMA chains, as a fraction of Σ|x̃_j q̃_j| <= Ñ_x·‖q̃‖.  Each MFMA adds 16 exact products to
// its accumulator; whatever the matrix core's order, rounding or truncation, each of those 17
// values is off by at most 2^-23 of the largest partial sum, over width/16 chained MFMAs:
// 17·(width/16)·2^-23 = (17/8)·width·2^-24.
constexpr double kRrGamma = 17.0 / 8.0 * 0x1p-24;

// Kernel launches.  In a profiled family (api.hip timed()), the launch carries the family's
// start / stop events itself (hipExtLaunchKernelGGL: the dispatch's own begin / end
// timestamps, as rocprofv3 reports them — a hipEventRecord pair around the launch adds the
// dispatch and completion latencies, ~2 us per kernel); the family's first kernel starts the
// interval and every kernel moves its end.
struct LaunchProf {
  hipEvent_t start = nullptr, stop = nullptr;
};
inline thread_local LaunchProf tl_launch_prof;

// Prepared searches (bb_plan_create, api.hip): while a plan is being built, every launch of
// the search is recorded — kernel, grid, block, LDS bytes and its arguments converted to the
// kernel's parameter types and packed at their alignments — instead of going out;
// bb_plan_launch replays the record with hipLaunchKernel, so a repeated request costs its
// launches and nothing of the host logic that chose and sized them.
struct CapturedOp {
  int kind = 0;  // 0 kernel launch, 1 memset, 2 device-to-device copy
  const void* func = nullptr;
  dim3 grid, block;
  std::uint32_t shmem = 0;
  std::vector<char> blob;          // the arguments, each at its offset
  std::vector<std::uint32_t> offs;
  void* dst = nullptr;
  const void* src = nullptr;
  std::size_t bytes = 0;
  int value = 0;
};
inline thread_local std::vector<CapturedOp>* tl_capture = nullptr;

template <typename... KArgs>
inline void capture_launch(const void* f, const dim3& grid, const dim3& block, std::uint32_t shmem, KArgs... a) {
  CapturedOp op;
  op.func = f;
  op.grid = grid;
  op.block = block;
  op.shmem = shmem;
  std::size_t off = 0;
  auto put = [&](const auto& v) {
    using T = std::decay_t<decltype(v)>;
    static_assert(alignof(T) <= 16, "kernel argument alignment");
    off = (off + alignof(T) - 1) & ~(alignof(T) - 1);
    op.offs.push_back((std::uint32_t)off);
    op.blob.resize(off + sizeof(T));
    std::memcpy(op.blob.data() + off, &v, sizeof(T));
    off += sizeof(T);
  };
  (put(a), ...);
  tl_capture->push_back(std::move(op));
}

template <typename... KArgs, typename... Args>
inline void bb_launch(void (*kernel)(KArgs...), const dim3& grid, const dim3& block, std::uint32_t shmem, hipStream_t s,
                      Args... args) {
  if (tl_capture) {
    capture_launch<KArgs...>((const void*)kernel, grid, block, shmem, static_cast<KArgs>(args)...);
    return;
  }
  LaunchProf& p = tl_launch_prof;
  if (p.stop) {
    hipExtLaunchKernelGGL(kernel, grid, block, shmem, s, p.start, p.stop, 0, args...);
    p.start = nullptr;
  } else {
    hipLaunchKernelGGL(kernel, grid, block, shmem, s, args...);
  }
}

// ---- tiling constants ---------------------------------------------------------------------
constexpr int kTileRows = 128;     // item / query rows are padded to this multiple
constexpr int kSelectThreads = 256;
constexpr int kSelectStageMax = 32768;  // score row staged in LDS when n_cols <= this
constexpr int kMaxKInt = 512;      // per-side internal list length limit (k_side + 1)

enum Dtype : int {
  F32 = 0,
  BF16 = 1,
  F64 = 2,
  SPLIT3 = 3,  // prep output: bf16 planes as the scan3 q3f image
  F16 = 4      // prep output: the f16 operand of the re-rank scans (never an index dtype)
};

struct GemmArgs {
  const void* Q;      // [Mpad][ldq]   queries (normalised), dtype of the index
  const void* X;      // [Npad][ldx]   item rows of the slab (row 0 = slab start)
  int32_t f16;        // 16-bit operands are f16: the re-rank copy of an f32 index (kScanF16 scans)
  float* S;           // [Mpad][lds]   scores out
  int64_t ldq, ldx, lds;
  int32_t Mpad;       // multiple of the query block tile
  int32_t Ncols;      // multiple of the item block tile
  int32_t Kpad;       // reduction length, multiple of the k-tile
  // fused selection-bound epilogue (tmax == null disables it)
  int32_t M_valid;          // real queries (rows >= M_valid have no exclusion row)
  int32_t n_valid;          // real items in the slab
  int64_t slab_start;       // local item index of slab column 0 (multiple of 32)
  const uint32_t* mask;     // local-item bitsets (null = all)
  const uint32_t* present;
  const uint32_t* excl;     // per-query bitsets [M_valid][excl_ld]
  int64_t excl_ld;
  uint32_t* tmax;           // [Mpad][ldt] eligible max order-image per 32-item tile
  uint32_t* pmax;           // [Mpad][ldt] present max order-image (rank-0 search) or null
  int64_t ldt;
  // fused query prologue (scan2): when set, Q is not read
  const int64_t* q_ids;     // gather item rows of these global ids (minus q_id_offset)
  int64_t q_id_offset, q_n_items;
  const void* q_items_base; // full item matrix (row stride ldx)
  const void* q_src;        // raw f32 query rows [M_valid][q_src_ld]
  int64_t q_src_ld;
  int32_t q_d;              // real query width (chunks past it read as 0)
  int32_t q_normalize;      // L2-normalise q_src rows
  // fused re-rank operands (q_istats set; bf16 scan2 over the bf16 copy of an f32 index):
  // the queries — raw f32 rows q_src, or with q_ids the f32 item rows at q_items_base, both
  // with stride q_src_ld — are rounded to bf16 in-kernel; the workgroups of item chunk 0 also
  // write the f32 rows and the bound ε of each query (as prep_kernel's out_f32 / eps_out)
  const float* q_istats;    // item error statistics (rr_prepare_kernel), or null
  float* q_f32_out;         // [Mpad][q_f32_ld]
  int64_t q_f32_ld;
  float* q_eps_out;         // [Mpad]
  // raw-query re-rank prologue (q_raw; scan2, bf16, list epilogue, semantic search): the bf16
  // operand is the RAW f32 row q_src rounded (no normalisation — a positive scale per query
  // never reorders its items), with the code quantum h derived from the row's norm
  // (scan2_raw_prologue; q_istats = the item statistics); the workgroups of item chunk 0
  // write h (q_h_out) and the raw-unit bound ε' (q_eps_out).  The list select normalises
  // the row itself (qnorm.h, as prep_kernel): no prep launch.
  int32_t q_raw;
  uint64_t* trace;          // probe builds only (scan3 ABL & 256): per-workgroup timestamps
  // streaming top-K (scan ABL & kScanStream): no S slab; every eligible score whose order
  // image reaches the query's bound is appended to a private per-lane candidate region
  // (query q, item chunk c, lane half h) -> region (q·n_chunks + c)·2 + h of cand_cap keys
  const uint64_t* thr_keys; // [Mpad][thr_ld] pilot top-K keys: bound = ord of key thr_ld-1
  int64_t thr_ld;
  uint64_t* cand;           // [Mpad·n_chunks·2][cand_cap] keys
  uint32_t* cand_cnt;       // [Mpad·n_chunks·2] appended per region (> cand_cap = overflow)
  uint64_t* cand_pmax;      // [Mpad·n_chunks·2] rank-0 key per region (present max) or null
  int32_t cand_cap;
  uint32_t gid0;            // global id of column 0
  // int16 score image (scan ABL & kScanS16, exact re-rank path): score s of query q is stored
  // as the code c = round(s / s_h[q]) (saturating, never reached: see rr_quantum), so the
  // slab costs 2 B per score; the select decodes c·s_h[q], whose bound ε (prep) covers it
  const float* s_h;         // [Mpad] quantum per query row
  float* q_h_out;           // fused re-rank prologue: writes the quantum beside q_eps_out
  // bounded candidate lists (scan ABL & kScanList, list_epi.h): no score image; per lane the
  // top-4 keys (u16 code of s / s_h[q], item position in the chunk) of every period of
  // l_period tiles, and (r0lists set) the top-2 present half-tile maxima for rank 0
  uint32_t* lists;          // uint4 at list_slot(chunk, period, l_np, Mpad/32, q >> 5, lane)
  uint32_t* r0lists;        // uint2 at list_slot(chunk, 0, 1, Mpad/32, q >> 5, lane), or null
  int32_t l_period, l_np;
  int32_t q_perm;           // Q holds the prepped operand in lane order: 1 = scan4's (scan4_q_offset), 2 = scan2's
  // streaming pilot (scan ABL kScanPilot): no score image; per lane the top pilot_m of its
  // eligible half-tile maxima over the item chunk, u32 order images at
  // ((chunk·(Mpad/32) + q/32)·64 + lane)·pilot_m (pilot_bound_kernel turns them into bounds)
  uint32_t* pilot_top;
  int32_t pilot_m;
};
// The scan4 query operand in lane order (PrepArgs / GemmArgs.q_perm): 16-B chunk c = 2u + h of
// query row q (Kpad/8 chunks per row, U = Kpad/16 u-steps) sits where lane (r, h) of wave w of
// group g loads query register j = b·U + u — one contiguous 1-KiB wave load per register,
// where row-major rows made every prologue load touch 32 lines for 16 B each.
__host__ __device__ inline size_t scan4_q_offset(int q, int c, int U) {  // in 16-B units
  const int g = q >> 8, w = (q >> 6) & 3, b = (q >> 5) & 1, r = q & 31, u = c >> 1, h = c & 1;
  return ((size_t)(g * 4 + w) * (2 * U) + b * U + u) * 64 + h * 32 + r;
}
// The scan2 query operand in lane order (q_perm == 2): chunk c = 2u + h of query row q sits
// where lane (r = q & 31, h) of the wave holding rows 32·(q >> 5) .. +32 loads it at u-step
// u, so each prologue load of a wave reads 1 KiB contiguous (row-major: 64 pieces of 16 B
// from 32 rows).
__host__ __device__ inline size_t scan2_q_offset(int q, int c, int U) {  // in 16-B units
  return ((size_t)(q >> 5) * U + (c >> 1)) * 64 + (c & 1) * 32 + (q & 31);
}
constexpr int kScanStream = 512;  // scan ABL bit: streaming top-K epilogue
constexpr int kScanS16 = 4096;    // scan ABL bit: int16 score image (GemmArgs.s_h)
constexpr int kScanList = 8192;   // scan ABL bit: bounded candidate lists (GemmArgs.lists)
constexpr int kScanPilot = 16384; // scan ABL bit: streaming pilot, top-m half-tile maxima (GemmArgs.pilot_top)
constexpr int kScanF16 = 32768;   // scan ABL bit: f16 operands (the re-rank copy of an f32 index), not bf16

// Quantum h of the int16 score image of one query and the widened bound of its decoded
// scores.  |approximate score| <= |q̃|·Ñ_x·(1+γ) <= 16384·h, so no code saturates; the
// encode (v_cvt_pknorm_i16_f32 of s·(1/(h·32767)), whatever its rounding) and the f32
// decode c·h move a score by at most h·(1 + 2^-8): ε' = (ε + 1.01·h)(1 + 2^-20) bounds
// |decoded − exact| wherever ε bounded |approximate − exact|.  h = ε/8 keeps the re-rank
// window within ~13 % of its f32-slab width.
__device__ inline void rr_quantum(double eps, double qnorm, double nx, float& eps_out, float& h_out) {
  double h = eps / 8.0;
  const double floor_h = 0x1p-14 * qnorm * nx * (1.0 + 0x1p-10);
  if (h < floor_h) h = floor_h;
  h_out = __double2float_ru(h);
  eps_out = __double2float_ru((eps + 1.01 * (double)h_out) * (1.0 + 0x1p-20));
}

// Two scores -> two int16 codes of the score image (quantum 1/(k·32767)).
__device__ __forceinline__ uint32_t s16_pack(float x, float y, float k) {
  return __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_pknorm_i16(x * k, y * k));
}
__device__ __forceinline__ float s16_lo(uint32_t w, float h) { return (float)(int16_t)(w & 0xFFFFu) * h; }
__device__ __forceinline__ float s16_hi(uint32_t w, float h) { return (float)(int16_t)(w >> 16) * h; }

// Item chunks of a query-resident scan launch (shared by the launcher and the host code
// sizing the streaming candidate regions): one workgroup per CU, ~256 workgroups.
// wg: workgroups aimed at.  The list scans of the exact re-rank path (one slab of an f32
// index, batches in flight: scan2 holds one workgroup per CU with the whole register file)
// aim at 224 — four CUs per XCD left to the other lanes' prep / list select, which otherwise
// wait for the scan to drain: configs[1] 14.1-14.3 -> 15.1-15.5 M q/s on 500 steps, the
// driver's 20 steps 12.1-12.6 -> 13.2-14.6, the scan itself 12.3 -> 13.3 us (r06h, r06h2:
// 232 and 240 gave nothing, 208-216 the same as 224).  BB_SCAN_WG (A/B runs) overrides it.
constexpr int kScanListWg = 224;
inline int scan_n_chunks(int Mpad, int tiles, int wg = 256) {
  static const int wg_env = ab_env("BB_SCAN_WG") ? std::atoi(ab_env("BB_SCAN_WG")) : 0;
  if (wg_env > 0 && wg != 256) wg = wg_env;
  const int n_groups = Mpad / 128;
  int n_chunks = (wg + n_groups - 1) / n_groups;
  return n_chunks < tiles ? n_chunks : tiles;
}

// scan3 query image ("q3f"): the bf16 planes of 32-query wave blocks in the order the scan
// loads them.  For query row q (wave block q >> 5, row r = q & 31 inside it), plane P and
// 16-B chunk c (k-step u = c >> 1, half h = c & 1), the chunk sits at lane h·32 + r of the
// 1-KiB line (block, P, u).  U = 16-wide k steps per row (Dpad / 16).
__host__ __device__ inline size_t q3f_chunk_offset(int q, int c, int P, int U) {
  const int lane = ((c & 1) << 5) | (q & 31);
  return ((((size_t)(q >> 5) * 3 + P) * U + (c >> 1)) * 64 + lane) * 16;
}

// scan3 item image ("t3"): the three bf16 planes of each 32-row tile in LDS order, one
// contiguous block of 32·3·Dpad·2 bytes per tile.  Plane P, 16-B chunk c (8 elements), row r
// of tile t sits at t·TILE_B + ((P·KP + c)·32 + r)·16 with KP = Dpad / 8.  One wave's 1-KiB
// LDS-DMA piece and one wave's ds_read_b128 fragment (chunks 2u, 2u+1 of 32 rows) are both
// contiguous.  Returns the byte offset of the chunk.
__host__ __device__ inline size_t t3_chunk_offset(int64_t row, int c, int P, int Dpad) {
  const int KP = Dpad >> 3;
  return (size_t)(row >> 5) * 32 * 3 * Dpad * 2 + ((size_t)(P * KP + c) * 32 + (row & 31)) * 16;
}

// Score image of the scan kernels ("blocked S"): each (32-query block, tile) accumulator
// stored as 4 KiB contiguous, so every score store is a full 1-KiB wave write (512 B as
// int16).  Store j (accumulator quads j of both lane halves) fills one 1-KiB block; lane
// (r, h) = (query q & 31, half) writes its quad at position 2r + h, so the two halves of a
// query sit side by side: a query's tile spans 4 lines of 4 queries each (32 B per query per
// line), where lane order h·32 + r spread it over 8.  Items 4g..4g+3 (g = item >> 2 within
// the tile; j = g >> 1, h = g & 1) of query q are the float4 at the returned element offset;
// ldt = tiles per query row.
__host__ __device__ inline size_t sblk_quad(int q, int t, int g, int64_t ldt) {
  return (((size_t)(q >> 5) * ldt + t) * 4 + (g >> 1)) * 256 + (2 * (q & 31) + (g & 1)) * 4;
}
// element offset of lane (r, h)'s quads inside its wave's block: + (tile·4 + j)·256
__host__ __device__ inline size_t sblk_lane(int q, int h, int64_t ldt) {
  return (size_t)(q >> 5) * ldt * 1024 + (2 * (q & 31) + h) * 4;
}

// XCD-aware bijection blockIdx -> row of [0, total): workgroup L runs on XCD L & 7, and each
// XCD takes one contiguous run of rows.  Rows that share cache lines (the 32 queries of a
// blocked score image block, sblk_quad) then share that XCD's L2 instead of fetching every
// line into eight L2s.
__device__ __forceinline__ int xcd_row(int L, int total) {
  const int xcd = L & 7, local = L >> 3, q8 = total >> 3, r8 = total & 7;
  return (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + local;
}

struct SelectArgs {
  const float* S;           // scores [B][lds]
  int64_t lds;
  const uint32_t* tmax;     // [B][ldt] per-tile eligible maxima from the GEMM epilogue
  const uint32_t* pmax;     // [B][ldt] per-tile present maxima (rank 0) or null
  int64_t ldt;
  int32_t n_cols;           // real columns in this slab
  int64_t slab_start;       // local item index of column 0
  uint32_t gid0;            // global id of column 0 (= id_offset + slab_start)
  const uint32_t* mask;     // local-item bitset or null
  const uint32_t* present;  // local-item bitset or null: the side's item space (rank-0 too)
  const uint32_t* excl;     // per-query local-item bitset or null
  int64_t excl_ld;          // words per query in excl
  int32_t K;                // internal list length (<= kMaxKInt)
  const uint64_t* carry_in; // [B][K] keys of previous slabs, or null
  uint64_t* keys_out;       // [B][K]
  uint64_t* max_inout;      // [B] running unmasked arg-max key, or null
  int32_t first_slab;       // max_inout is overwritten (not merged) when set
  // final output of single-list modes on the last slab (out_scores == null: keys_out)
  float* out_scores;        // [B][k_final]
  int64_t* out_ids;         // [B][k_final]
  int32_t* out_counts;      // [B] or null
  int32_t k_final;
  int32_t s_blocked;        // S is the scan3 blocked image (sblk_quad), else row-major [B][lds]
  uint64_t* trace;          // probe builds only: per-workgroup phase timestamps, or null
  // exact re-rank of an approximate (one-product bf16 MFMA) score slab (rr_eps != null):
  // every S value is within rr_eps[row] of the exact score x·q of the f32 rows, so the
  // items whose approximate score reaches (K-th approximate) − 2ε hold the exact top-K;
  // they are rescored from the f32 rows (f64 sum, rounded to f32) and ranked by that.
  const float* rr_eps;      // [B] per-query bound ε, or null (S is exact)
  const float* rr_x;        // f32 item rows [Npad][rr_ld]; local row = gid - rr_gid_base
  const float* rr_q;        // f32 query rows [B][rr_ld]
  int64_t rr_ld;
  int32_t rr_d;             // elements of a row to dot (multiple of 4, <= rr_ld)
  uint32_t rr_gid_base;     // global id of local row 0 (the index's id_offset)
  // hand-off from select_kernel to a separate rerank_kernel launch (BB_RR_SPLIT A/B runs);
  // rr_out == null: select_kernel rescores and emits itself (the default)
  uint64_t* rr_out;         // [B][kRrCap] approximate candidate keys within 2ε of the K-th
  uint32_t* rr_cnt;         // [B] candidates, or kRrSlow (masses at the bound: exact slow path)
  uint32_t* rr_thr;         // [B][2] order images: gather bound (slow path), rank-0 bound
  uint32_t* rr_r0;          // [B][kRrR0Cap] rank-0 candidate global ids
  uint32_t* rr_r0n;         // [B] their count, or kRrSlow
  // one-wave re-rank select (select_rr_wave_kernel): 1 = the row overflowed a cap and is left
  // to the block select, which then skips every row whose flag is 0
  uint32_t* rr_flags;       // [B] or null
  // int16 score image (GemmArgs.s_h): S holds codes, score = code · s_h[row]; null = f32 S
  const float* s_h;
  // bounded candidate lists of a kScanList scan (select_list_kernel): the scan's GemmArgs
  // lists / r0lists and geometry (item chunks, tiles, periods per chunk, tiles per period,
  // 32-query blocks); s_h = the code quantum h, rr_eps = ε'
  const uint32_t* lists;
  const uint32_t* r0lists;
  int32_t l_chunks, l_tiles, l_np, l_period, l_nb;
  int32_t ablate;           // probe runs (BB_LS_ABLATE): 1 = every rescore gathers row 0 (cache-resident)
  // raw-query lists (GemmArgs.q_raw): the select normalises row rr_q_raw[row] (real width
  // rr_q_raw_d, stride rr_q_raw_ld) into its LDS query with prep_kernel's arithmetic
  // (qnorm.h); rr_eps = the scan's raw-unit bound, s_h its quantum; rr_q is not read
  const float* rr_q_raw;
  int64_t rr_q_raw_ld;
  int32_t rr_q_raw_d;       // real row width (elements past it are zero, as prep's)
  // constraint-first search (compact.hip): keys carry positions in the packed rows; the final
  // ids written are idmap[position] (global ids), null = keys carry global ids
  const uint32_t* idmap;
};
constexpr int kRrCap = 512;
constexpr int kRrR0Cap = 64;
constexpr int kRrMaxD = 512;   // widest f32 row the re-rank takes (wider: the split scan)
constexpr int kRrRawRows = 16;  // query chunks up to which semantic lists take the raw-query path (no prep launch)
constexpr uint32_t kRrSlow = 0xFFFFFFFFu;

// Streaming top-K, second stage: per query, the exact top-K (full key order) of the
// candidates the streaming scan appended to the query's regions.
struct CandSelectArgs {
  const uint64_t* cand;      // [B·regions][cap]
  const uint32_t* cand_cnt;  // [B·regions]
  const uint64_t* cand_pmax; // [B·regions] rank-0 keys, or null (no rank-0 drop)
  int32_t regions, cap;      // regions per query, keys per region
  int32_t K;                 // internal list length (<= kMaxKInt)
  uint64_t* keys_out;        // [B][K] when out_scores == null
  uint64_t* max_out;         // [B] rank-0 key (with cand_pmax), or null
  float* out_scores;         // [B][k_final] single-list modes: final output (rank-0 dropped)
  int64_t* out_ids;
  int32_t* out_counts;
  int32_t k_final;
  uint32_t* overflow;        // set to 1 when a region overflowed (results of that row invalid)
  const uint64_t* carry_in;  // [B][K] exact list of an earlier item range (joins the candidates), or null
  const uint64_t* max_in;    // [B] rank-0 key of that range (with cand_pmax), or null
};

struct FinalizeArgs {
  const uint64_t* keys;     // [P][sides][B][K_int]
  const uint64_t* max_keys; // [P][B] or null
  int32_t P, sides, B, K_int;  // B = row stride of each [side] key block
  int32_t n_rows;               // queries to finalize (grid size)
  int32_t drop_rank0;       // side 0 (content / similar) drops the global arg-max
  int32_t k;                // final length
  int32_t k_side;           // hybrid per-side length
  int32_t hybrid;
  double w_content, w_cf;
  float* scores;            // [B][k]
  int64_t* ids;             // [B][k]
  int32_t* counts;          // [B] or null
  uint64_t* trace;          // probe runs (BB_SELECT_TRACE): per-row phase stamps, or null
  const uint32_t* idmap;    // packed-row positions -> global ids (SelectArgs.idmap), or null
};
__device__ __forceinline__ int64_t out_id(const uint32_t* idmap, uint32_t g) {
  return idmap ? (int64_t)idmap[g] : (int64_t)g;
}



struct PrepArgs {
  const void* src;          // query rows [B][d] (q_dtype) or null
  int32_t src_dtype;
  int64_t src_ld;
  const int64_t* item_ids;  // global ids (gather from the item matrix) or null
  int64_t id_offset;
  const void* items;        // item matrix [Npad][Dpad] index dtype (for gathers)
  int64_t n_items;
  int32_t d, Dpad;          // real and padded widths
  int32_t normalize;        // 1 = divide by L2 norm (sklearn normalize semantics)
  void* out;                // [Bpad][Dpad] index dtype
  int32_t out_dtype;
  int32_t B, Bpad;
  // re-rank operands (out_dtype == BF16 with out_f32 set): the f32 row [Bpad][Dpad_f] beside
  // the bf16 operand, and the per-row bound ε of |bf16 dot − f32 dot| against items whose
  // error statistics are istats (rr_prepare_kernel): ε = E_x·|q̃| + N_x·|q̃−q| + γ·Ñ_x·|q̃|
  float* out_f32;
  int32_t Dpad_f;
  float* eps_out;           // [Bpad]
  const float* istats;      // [3]: max |x̃−x|, max |x|, max |x̃| over the item rows
  float* h_out;             // [Bpad] int16 score-image quantum (rr_quantum; eps_out widened), or null
  int32_t q_perm;           // the bf16 operand in lane order, not row-major: 1 = scan4's (scan4_q_offset), 2 = scan2's
};

// Constraint-first search (compact.hip): the rows a mask allows, packed.  Positions [0, cap)
// of the packed buffers; position p holds the p-th allowed item (ascending ids).
constexpr int kCompactMaxWords = 2048;   // mask words: indexes of up to 65,536 rows
constexpr int kCompactMaxSlots = 16384;  // packed slots (the auto rule packs at most n / 4 rows)
struct CompactArgs {
  const uint32_t* mask;      // [nw] allowed items (device)
  int64_t n;                 // items of the index
  int32_t nw;                // ceil(n / 32)
  uint32_t id_offset;        // global id of local row 0
  const float* items;        // f32 content rows [Npad][ld], or null (no content side)
  int64_t ld;
  const uint16_t* items_bf;  // their f16 copy [Npad][ld_b]
  int64_t ld_b;
  const uint32_t* items_present;
  const float* cf;           // f32 CF rows [Npad][ldc], or null (no CF side)
  int64_t ldc;
  const uint16_t* cf_bf;
  int64_t ldc_b;
  const uint32_t* cf_present;
  int32_t cap;               // packed slots (multiple of 32; >= stride x the allowed count)
  int32_t stride;            // allowed item p sits in slot p·stride (the other slots: padding)
  int32_t cap_pos;           // cap / stride
  int32_t cnw;               // cap / 32 (words of the packed present bitsets)
  int32_t xnw;               // words per row of the packed exclusions (the shadow's ceil(count / 32))
  int32_t n_word_wg;         // cap / 32 workgroups: id map + present words
  int32_t n_copy_wg;         // workgroups of the row copies (four 16-B pieces per thread)
  int32_t ch_items, ch_items_b, ch_cf, ch_cf_b;  // 16-B pieces per row of each copy (0: absent)
  uint32_t* idmap;           // [cap] global id per position (0xFFFFFFFF: padding)
  float* c_items;
  uint16_t* c_items_bf;
  uint32_t* c_present;       // [cnw]
  float* c_cf;
  uint16_t* c_cf_bf;
  uint32_t* c_cf_present;
  int32_t B;                 // query rows with exclusions
  int32_t n_query_wg;        // exclusion workgroups (4 rows each): ceil(B / 4), 0 without exclusions
  const int64_t* q_items;    // [B] liked sets (global ids) — the rank-0 lookups
  const uint64_t* r0key;     // [n + 1] rank-0 key of each item's own row (the unmasked arg-max); [n]: a zero row's
  uint32_t* c_excl0;         // [B][xnw] content exclusion: the rank-0 item's position, or null
  const uint32_t* excl;      // [B][excl_ld] per-query exclusions over local rows, or null
  int64_t excl_ld;
  uint32_t* c_excl1;         // [B][xnw] the same re-indexed to positions, or null
  PrepArgs prep_c, prep_f;   // the packed search's query prep of each side (Bpad 0: none), run by
                             // the query workgroups (prep_body.h) in place of its prep launch
};
hipError_t launch_compact(const CompactArgs& a, hipStream_t s);

struct MaskArgs {
  const int32_t* parts;
  const int16_t* year;
  const int32_t* theme;
  int64_t n;
  int32_t parts_min, parts_max, year_min, year_max;
  int32_t theme_mode, n_theme_bits;
  const uint32_t* theme_bits;  // device copy
  uint32_t* out;               // [ceil(n/32)] words
};

// launchers (stream-ordered, no sync, no allocation)
hipError_t launch_gemm(int dtype, const GemmArgs& a, hipStream_t s);
bool gemm_uses_scan(int dtype, int Mpad, int Kpad);  // the query-resident scan kernel runs
bool scan3_supported(int Mpad, int Kpad);            // split-bf16 scan for an f32 index
bool scan4_used(int dtype, int Mpad);                // bf16 scan with 64 queries per wave
// item chunks (candidate regions / 2 per query) of the scan launch for these shapes
// item chunks of a scan launch; list_ku > 0: a list scan (kScanList) of rows list_ku 16-B chunks wide
int scan_chunks(int dtype, int Mpad, int tiles, bool split, int list_ku = 0);
bool launch_scan4(const GemmArgs& a, int ku, hipStream_t s);  // scan4_used(BF16, a.Mpad) shapes
int scan4_pilot_m(int kpad);  // GemmArgs.pilot_m of a kScanPilot scan4 launch
bool scan4_dual_supported(int ku0, int ku1);
bool scan4_dual_args_ok(const GemmArgs& a0, const GemmArgs& a1, const char** why);
hipError_t launch_scan4_dual(const GemmArgs& a0, const GemmArgs& a1, hipStream_t s);  // hybrid, int16 image
hipError_t launch_scan3(const GemmArgs& a, hipStream_t s);  // X = item planes, Q = q3f image
hipError_t launch_split_planes(const float* src, int64_t n, int64_t ld, uint16_t* dst, hipStream_t s);
// f32 rows [Npad][ld_f] -> bf16 copy [Npad][ld_b] (RNE, zero padded) + error statistics
// stats[0..2] = max over rows of |x̃−x|, |x|, |x̃| (rounded up; stats must start at 0)
hipError_t launch_rr_prepare(const float* src, int64_t npad, int64_t ld_f, uint16_t* dst, int64_t ld_b,
                             float* stats, hipStream_t s);
int gemm_tile_m(int dtype);
int gemm_tile_n(int dtype);
int gemm_tile_k(int dtype);
hipError_t launch_select(const SelectArgs& a, int B, hipStream_t s);
hipError_t launch_rerank(const SelectArgs& a, int B, hipStream_t s);  // after launch_select, rr_* set
// one wave per query, one-slab re-rank searches (rr_flags set; rows it leaves: launch_select)
hipError_t launch_select_rr_wave(const SelectArgs& a, int B, hipStream_t s);
hipError_t launch_select_rr_wave_dual(const SelectArgs& a0, const SelectArgs& a1, int B, hipStream_t s);
// exact top-K of a kScanList scan (lists set, rr_* operands, one slab): one workgroup per row;
// a1 != null: both sides of a hybrid search in one launch
hipError_t launch_select_list(const SelectArgs& a0, const SelectArgs* a1, int B, hipStream_t s);
hipError_t launch_cand_select(const CandSelectArgs& a, int B, hipStream_t s);
hipError_t launch_finalize(const FinalizeArgs& a, hipStream_t s);
// streaming bound of each query row from a kScanPilot scan: the K-th largest of its
// 2·n_chunks·m half-tile maxima (K distinct half tiles, so K distinct items reach it), as
// a key (ord << 32) in thr_out[row]; 0 (take every eligible item) when fewer than K exist
hipError_t launch_pilot_bound(const uint32_t* top, int n_chunks, int m, int nb, int K, int B, uint64_t* thr_out,
                              hipStream_t s);
hipError_t launch_prep(const PrepArgs& a, hipStream_t s);
hipError_t launch_prep2(const PrepArgs& a0, const PrepArgs& a1, hipStream_t s);
hipError_t launch_mask(const MaskArgs& a, hipStream_t s);
hipError_t launch_clear_bits(uint32_t* bits, const int64_t* ids, int64_t n_ids, int64_t n_items,
                             hipStream_t s);
hipError_t launch_convert_rows(const void* src, int src_dtype, int64_t n, int d, int normalize,
                               void* dst, int dst_dtype, int64_t Dpad, hipStream_t s);

}  // namespace bb
