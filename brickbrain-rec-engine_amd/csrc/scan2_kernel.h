// scan2_kernel.h — query-resident MFMA scan with the epilogue woven into the MFMA stream.
//
// Same contract and data flow as scan_kernel.h (queries resident in VGPRs, 32-item tiles
// staged by LDS-DMA into an XOR-swizzled three-deep ring, S + per-tile maxima epilogue),
// restructured for the single wave per SIMD that this register budget allows:
//   * tiles alternate between two accumulator sets (even / odd), so tile t-1's epilogue
//     (accumulator reads, order images, S stores, tile maxima) and tile t+1's staging are
//     issued as small slices BETWEEN tile t's MFMAs — the VALU / VMEM work runs in the
//     MFMA issue shadows instead of serially between tiles;
//   * LDS fragment addresses are 8 per-lane bases + immediate offsets (no per-step VALU);
//   * staging is branch-free (the tile after the last one re-stages the last tile);
//   * optional fused query prologue: raw f32 query rows are L2-normalised in-kernel
//     (sklearn normalize semantics, f64 sum of squares), or liked-set item rows are
//     gathered by id — replacing the separate prep kernel on the hot path.
#pragma once
#include <utility>

#include "list_epi.h"
#include "scan_kernel.h"

namespace bb {

typedef uint32_t u32x4v __attribute__((ext_vector_type(4)));

template <int... I, typename F>
__device__ __forceinline__ void static_for_impl(std::integer_sequence<int, I...>, F&& f) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  static_for_impl(std::make_integer_sequence<int, N>{}, f);
}

// Two f32 -> one dword of the 16-bit operand (element a low): bf16 (v_cvt_pk_bf16_f32, RNE)
// or, for the f16 re-rank copy (kScanF16), f16 (RNE, saturating: to_f16)
template <bool F16>
__device__ __forceinline__ uint32_t pack16(float a, float b) {
  if constexpr (F16) {
    return (uint32_t)to_f16(a) | ((uint32_t)to_f16(b) << 16);
  } else {
    typedef __bf16 bf2v __attribute__((ext_vector_type(2)));
    const bf2v v = {(__bf16)a, (__bf16)b};
    return __builtin_bit_cast(uint32_t, v);
  }
}
// element c (0: low half) of a packed dword, as f32
template <bool F16>
__device__ __forceinline__ float unpack16(uint32_t w, int c) {
  if constexpr (F16) return f16_val((uint16_t)(c ? w >> 16 : w & 0xFFFFu));
  else return __uint_as_float(c ? (w & 0xFFFF0000u) : (w << 16));
}

// Exact re-rank prologue (16-bit operand from raw f32 rows, GemmArgs.q_f32_out): lane half h
// of query row q holds elements (2u + h)·8 .. +8 of the row.  Normalised in f64 as prep_kernel
// (sklearn normalize); rounded to bf16 (v_cvt_pk_bf16_f32, RNE).
// With rr_write (the workgroups of item chunk 0) the f32 row and ε go out as well:
// ε = E_x·|q̃| + N_x·|q̃−q| + γ·Ñ_x·|q̃| (prep_kernel's RrAcc), with the f32 sums of squares
// scaled by (1 + 2^-10) to cover their rounding (<= 193 terms of 2^-24 each).
// Source: raw rows q_src [M][q_src_ld], or (q_ids) the stored f32 item rows of the liked
// sets, q_items_base [n][q_src_ld] (already normalised; an unknown id gives a zero row).
template <int U, bool F16>
__device__ __forceinline__ void scan2_rr_prologue(const GemmArgs& a, int q, int h, bool rr_write, uint4 (&qf)[U]) {
  bool ok = true;
  const float* row;
  if (a.q_ids) {
    const int64_t lid = a.q_ids[q] - a.q_id_offset;
    ok = lid >= 0 && lid < a.q_n_items;
    row = (const float*)a.q_items_base + (size_t)(ok ? lid : 0) * a.q_src_ld;
  } else {
    row = (const float*)a.q_src + (size_t)q * a.q_src_ld;
  }
  const int d = a.q_d;
  auto load = [&](int u, int s) -> float4 {  // (host: d % 4 == 0, 16-B aligned rows): clamp, load, select
    const int k0 = (2 * u + h) * 8 + 4 * s;
    const float4 t = *(const float4*)(row + (k0 < d ? k0 : d - 4));
    return ok && k0 < d ? t : make_float4(0.f, 0.f, 0.f, 0.f);
  };
  // rows up to 384 wide stay in registers; wider ones are summed first and loaded again
  constexpr bool kTwoPass = U > 24;
  float4 x[kTwoPass ? 1 : 2 * U];
  double s0 = 0.0, s1 = 0.0;
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const float4 v = load(u, s);
      if (!kTwoPass) x[2 * u + s] = v;
      if (a.q_normalize) {
        s0 = fma((double)v.x, (double)v.x, s0);
        s1 = fma((double)v.y, (double)v.y, s1);
        s0 = fma((double)v.z, (double)v.z, s0);
        s1 = fma((double)v.w, (double)v.w, s1);
      }
    }
  // f64 norm, f64 reciprocal: the f32 element is (float)(x·(1/‖x‖)), prep_kernel's
  // (float)(x/‖x‖) but at the ~2^-28 of elements whose quotient falls on an f32 rounding
  // boundary to within the f64 error
  double inv = 1.0;
  bool scale = false;
  if (a.q_normalize) {
    double ss = s0 + s1;
    ss += __shfl_xor(ss, 32);
    const double nrm = sqrt(ss);
    scale = nrm != 0.0;
    inv = scale ? 1.0 / nrm : 1.0;
  }
  auto scl = [&](float v) -> float { return scale ? (float)((double)v * inv) : v; };
  // per k-step: scale, round to the bf16 operand; chunk 0 also stores the f32 row and sums
  // the squares of the rounding error and of the operand
  float* orow = a.q_f32_out + (size_t)q * a.q_f32_ld;
  float e2 = 0.f, b2 = 0.f;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    float4 p = kTwoPass ? load(u, 0) : x[2 * u], r = kTwoPass ? load(u, 1) : x[2 * u + 1];
    p = make_float4(scl(p.x), scl(p.y), scl(p.z), scl(p.w));
    r = make_float4(scl(r.x), scl(r.y), scl(r.z), scl(r.w));
    qf[u] = make_uint4(pack16<F16>(p.x, p.y), pack16<F16>(p.z, p.w), pack16<F16>(r.x, r.y), pack16<F16>(r.z, r.w));
    if (rr_write) {
      const uint32_t w[4] = {qf[u].x, qf[u].y, qf[u].z, qf[u].w};
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int k0 = (2 * u + h) * 8 + 4 * s;
        const float4 v = s ? r : p;
        if (k0 < a.q_f32_ld) *(float4*)(orow + k0) = v;
        const float vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const float bv = unpack16<F16>(w[2 * s + (c >> 1)], c & 1);
          const float e = vv[c] - bv;  // exact (bv is vv[c] rounded to 8 or 11 significant bits)
          e2 = fmaf(e, e, e2);
          b2 = fmaf(bv, bv, b2);
        }
      }
    }
  }
  if (!rr_write) return;
  e2 += __shfl_xor(e2, 32);
  b2 += __shfl_xor(b2, 32);
  if (h == 0) {
    const double sc = 1.0 + 0x1p-10;
    const double e = sqrt((double)e2 * sc), b = sqrt((double)b2 * sc);
    const double gam = kRrGamma * (double)a.Kpad;
    const double eps = (double)a.q_istats[0] * b + (double)a.q_istats[1] * e + gam * (double)a.q_istats[2] * b;
    if (a.q_h_out)
      rr_quantum(eps * (1.0 + 0x1p-20), b, (double)a.q_istats[2], a.q_eps_out[q], a.q_h_out[q]);
    else
      a.q_eps_out[q] = __double2float_ru(eps * (1.0 + 0x1p-20));
  }
}

// Raw-query re-rank prologue (GemmArgs.q_raw): lane half h of query row q holds elements
// (2u + h)·8 .. +8 of the RAW f32 row, rounded to bf16 (RNE) — no normalisation and no
// prep launch.  The code quantum of the list epilogue comes from the row's f32 sum of
// squares n2 (the lane pair's two halves, added in either order: the same bits):
//   Q = sqrt(n2·(1 + 2^-10)) >= ‖q‖       (f32 rounding of <= 512 squares)
//   h = 2^-12·Q·(1 + 2^-8)·Ñ_x, rounded up  ->  |x̃·q̃| <= Ñ_x·‖q̃‖ <= 4096·h: codes fit 16 bits
// Every workgroup derives the same h.  Those of item chunk 0 store it (q_h_out) and the
// scan's error bound in raw units (q_eps_out), as prep's RrAcc but on the raw row:
//   ε = E_x·‖q̃‖ + N_x·‖q̃ − q‖ + γ·Ñ_x·‖q̃‖          (f32 sums of squares scaled by 1 + 2^-10)
//   ε' = (ε·(1+2^-20) + 1.01·h + Q·(N_x·(2^-23 + 2^-40) + 2^-20))·(1+2^-20)
// where the Q term covers the exact score's own roundings (the normalised f32 row, the f64
// sum rounded to f32) against x·q/‖q‖, scaled to raw units.
template <int U, bool F16>
__device__ __forceinline__ float scan2_raw_prologue(const GemmArgs& a, int q, int h, bool write, uint4 (&qf)[U]) {
  const float* row = (const float*)a.q_src + (size_t)q * a.q_src_ld;
  const int d = a.q_d;
  float n2 = 0.f, e2 = 0.f, b2 = 0.f;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    float4 v[2];
#pragma unroll
    for (int s = 0; s < 2; ++s) {  // (host: d % 4 == 0, 16-B aligned rows): clamp, load, select
      const int k0 = (2 * u + h) * 8 + 4 * s;
      const float4 t = *(const float4*)(row + (k0 < d ? k0 : d - 4));
      v[s] = k0 < d ? t : make_float4(0.f, 0.f, 0.f, 0.f);
      n2 = fmaf(v[s].x, v[s].x, n2);
      n2 = fmaf(v[s].y, v[s].y, n2);
      n2 = fmaf(v[s].z, v[s].z, n2);
      n2 = fmaf(v[s].w, v[s].w, n2);
    }
    qf[u] = make_uint4(pack16<F16>(v[0].x, v[0].y), pack16<F16>(v[0].z, v[0].w), pack16<F16>(v[1].x, v[1].y),
                       pack16<F16>(v[1].z, v[1].w));
    if (write) {  // (wave-uniform: the workgroups of item chunk 0)
      const uint32_t w[4] = {qf[u].x, qf[u].y, qf[u].z, qf[u].w};
      const float vv[8] = {v[0].x, v[0].y, v[0].z, v[0].w, v[1].x, v[1].y, v[1].z, v[1].w};
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        const float bv = unpack16<F16>(w[c >> 1], c & 1);
        const float e = vv[c] - bv;  // exact (bv is vv[c] rounded to 8 or 11 significant bits)
        e2 = fmaf(e, e, e2);
        b2 = fmaf(bv, bv, b2);
      }
    }
  }
  n2 += __shfl_xor(n2, 32);
  const double Q = sqrt((double)n2 * (1.0 + 0x1p-10));
  const float hq = __double2float_ru(0x1p-12 * Q * (1.0 + 0x1p-8) * (double)a.q_istats[2]);
  if (write) {
    e2 += __shfl_xor(e2, 32);
    b2 += __shfl_xor(b2, 32);
    if (h == 0) {
      const double sc = 1.0 + 0x1p-10;
      const double e = sqrt((double)e2 * sc), b = sqrt((double)b2 * sc);
      const double ex = (double)a.q_istats[0], nx = (double)a.q_istats[1], nxb = (double)a.q_istats[2];
      const double gam = kRrGamma * (double)a.Kpad;
      const double eps = ex * b + nx * e + gam * nxb * b;
      const double ep = (eps * (1.0 + 0x1p-20) + 1.01 * (double)hq + Q * (nx * (0x1p-23 + 0x1p-40) + 0x1p-20)) *
                        (1.0 + 0x1p-20);
      a.q_h_out[q] = hq;
      a.q_eps_out[q] = __double2float_ru(ep);
    }
  }
  return hq;
}

// Query operand: 16-B chunk (2u + h) of this lane's query row into qf[u].  Returns the list
// epilogue's code quantum of the raw-query prologue (0 otherwise: the epilogue reads s_h).
template <typename T, int KU, bool F16 = false>
__device__ __forceinline__ float scan2_load_queries(const GemmArgs& a, int q, int h, uint4 (&qf)[KU / 2],
                                                    bool rr_write = false) {
  constexpr int U = KU / 2;
  if (q >= a.M_valid) {
#pragma unroll
    for (int u = 0; u < U; ++u) qf[u] = make_uint4(0, 0, 0, 0);
    return 0.f;
  }
  if constexpr (sizeof(T) == 2 && KU <= kRrMaxD / 8) {
    if (a.q_raw) return scan2_raw_prologue<U, F16>(a, q, h, rr_write, qf);
    if (a.q_istats) {  // exact re-rank operands (GemmArgs.q_f32_out)
      scan2_rr_prologue<U, F16>(a, q, h, rr_write, qf);
      return 0.f;
    }
  }
  if (a.q_ids) {  // similar / hybrid: the stored (normalised, padded) item row of the liked set
    const int64_t lid = a.q_ids[q] - a.q_id_offset;
    const bool ok = lid >= 0 && lid < a.q_n_items;
    const char* row = (const char*)a.q_items_base + (size_t)(ok ? lid : 0) * a.ldx * sizeof(T);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint4 v = *(const uint4*)(row + (2 * u + h) * 16);
      qf[u] = ok ? v : make_uint4(0, 0, 0, 0);
    }
    return 0.f;
  }
  if (a.q_src) {  // raw f32 rows (T == float): normalise here
    const float* row = (const float*)a.q_src + (size_t)q * a.q_src_ld;
    const int d = a.q_d;
    float4 x[U];  // (host guarantees d % 4 == 0, 16-B aligned rows): clamp, load, select
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int k0 = (2 * u + h) * 4;
      const float4 t = *(const float4*)(row + (k0 < d ? k0 : d - 4));
      x[u] = k0 < d ? t : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    if (a.q_normalize) {
      // f32 sum of squares (4 partial sums), as sklearn's einsum does for f32 input; a
      // norm error only scales the whole query row, so it never reorders its items
      float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
#pragma unroll
      for (int u = 0; u < U; ++u) {
        s0 = fmaf(x[u].x, x[u].x, s0);
        s1 = fmaf(x[u].y, x[u].y, s1);
        s2 = fmaf(x[u].z, x[u].z, s2);
        s3 = fmaf(x[u].w, x[u].w, s3);
      }
      float ss = (s0 + s1) + (s2 + s3);
      ss += __shfl_xor(ss, 32);
      const float nrm = __fsqrt_rn(ss);
      const float inv = nrm == 0.f ? 1.f : __fdiv_rn(1.f, nrm);
#pragma unroll
      for (int u = 0; u < U; ++u) {
        x[u].x *= inv;
        x[u].y *= inv;
        x[u].z *= inv;
        x[u].w *= inv;
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
      qf[u] = make_uint4(__float_as_uint(x[u].x), __float_as_uint(x[u].y), __float_as_uint(x[u].z),
                         __float_as_uint(x[u].w));
    return 0.f;
  }
  if (sizeof(T) == 2 && a.q_perm) {  // lane-order operand (scan2_q_offset): 1 KiB per wave load
    const uint4* qp = (const uint4*)a.Q + scan2_q_offset(q, h, U);
#pragma unroll
    for (int u = 0; u < U; ++u) qf[u] = qp[(size_t)u * 64];
    return 0.f;
  }
  const char* qrow = (const char*)a.Q + (size_t)q * a.ldq * sizeof(T);
#pragma unroll
  for (int u = 0; u < U; ++u) qf[u] = *(const uint4*)(qrow + (2 * u + h) * 16);
  return 0.f;
}

// Per-lane half-tile maxima of one 32-item tile (this lane's 16 items): te over eligible
// items (present ∧ mask ∧ ¬excl, in range), tp over present in-range items, as order
// images.  Fast path (wave-uniform): every item of the tile is eligible for every query
// of the wave — a float max3 tree, then one order image (+0.0f folds -0 into +0, so the
// bound stays >= every element's image); otherwise a per-item masked scan.
__device__ __forceinline__ void tile_maxima(const f32x16s& p, int tile0, int n_valid, uint32_t pw, uint32_t ok, int h,
                                            uint32_t& te, uint32_t& tp) {
  if (__all(tile0 + 32 <= n_valid && pw == 0xFFFFFFFFu && ok == 0xFFFFFFFFu)) {
    // v_max3_f32 directly: fmaxf on opaque (inline-asm MFMA) results would canonicalise
    // every input first, doubling the count.  Scores are finite, so NaN rules do not apply.
    auto max3 = [](float x, float y, float z) {
      float m;
      asm("v_max3_f32 %0, %1, %2, %3" : "=v"(m) : "v"(x), "v"(y), "v"(z));
      return m;
    };
    const float m0 = max3(p[0], p[1], p[2]), m1 = max3(p[3], p[4], p[5]), m2 = max3(p[6], p[7], p[8]);
    const float m3 = max3(p[9], p[10], p[11]), m4 = max3(p[12], p[13], p[14]);
    const float m = max3(max3(m0, m1, m2), max3(m3, m4, p[15]), p[15]);
    const uint32_t u = __builtin_bit_cast(uint32_t, m + 0.0f);
    te = tp = u ^ ((uint32_t)((int32_t)u >> 31) | 0x80000000u);  // ord_of
    return;
  }
  uint32_t e = 0, t = 0;
#pragma unroll
  for (int g = 0; g < 16; ++g) {
    const int it = (g & 3) + 8 * (g >> 2) + 4 * h;
    const uint32_t o = ord_of(p[g]);
    const bool in = tile0 + it < n_valid;
    const uint32_t op = (in && ((pw >> it) & 1u)) ? o : 0u;
    const uint32_t oe = (in && ((ok >> it) & 1u)) ? o : 0u;
    t = op > t ? op : t;
    e = oe > e ? oe : e;
  }
  te = e;
  tp = t;
}

// Streaming top-K epilogue (ABL & kScanStream) of one half tile (this lane's 16 items).
// Per lane: the query's bound thr, a private candidate region reg[0..cap) with count n,
// and the running rank-0 key (present arg-max) rkey with its folded order image rp.
struct StreamLane {
  uint32_t thr = 0xFFFFFFFFu;
  uint32_t n = 0;
  uint32_t rp = 0;
  uint64_t rkey = 0;
  uint64_t* reg = nullptr;
};

// Append every eligible item whose order image reaches the bound.  Wave-uniform skip when
// no lane's half-tile maximum reaches it (the common case once the bound is tight).
__device__ __forceinline__ void stream_append(const f32x16s& p, int tile0, int n_valid, uint32_t ok, int h,
                                              uint32_t te, StreamLane& s, uint32_t cap, uint32_t gid0) {
  if (!__any(te >= s.thr)) return;
  if (te >= s.thr) {
#pragma unroll
    for (int g = 0; g < 16; ++g) {
      const int it = (g & 3) + 8 * (g >> 2) + 4 * h;
      const uint32_t o = ord_of(p[g]);
      if (tile0 + it < n_valid && ((ok >> it) & 1u) && o >= s.thr) {
        if (s.n < cap) s.reg[s.n] = make_key(o, gid0 + (uint32_t)(tile0 + it));
        ++s.n;
      }
    }
  }
}

// Rank 0 (similar-sets drops the unmasked arg-max, recommendation_system.py:217): a new
// running present maximum is rare (record values along the scan), so its item is resolved
// only then — the first present in-range item equal (as a float: -0 == +0, numpy argmax)
// to the half-tile maximum; later tiles need a strictly larger maximum (lower id wins ties).
__device__ __forceinline__ void stream_rank0(const f32x16s& p, int tile0, int n_valid, uint32_t pw, int h,
                                             uint32_t tp, StreamLane& s, uint32_t gid0) {
  if (!__any(tp > s.rp)) return;
  if (tp > s.rp) {
    const float mv = float_of_ord(tp);
    bool found = false;
#pragma unroll
    for (int g = 0; g < 16; ++g) {
      const int it = (g & 3) + 8 * (g >> 2) + 4 * h;
      if (!found && tile0 + it < n_valid && ((pw >> it) & 1u) && p[g] == mv) {
        s.rkey = make_key(ord_of(p[g]), gid0 + (uint32_t)(tile0 + it));
        found = true;
      }
    }
    s.rp = tp;
  }
}

// Per-lane streaming state at kernel start: the query's bound is the order image of the
// last key of its pilot top-K list (0 = fewer eligible pilot items than K: take every
// eligible item); padded query rows take nothing.
__device__ __forceinline__ void stream_begin(const GemmArgs& a, int q, size_t region, StreamLane& s) {
  s.reg = a.cand + region * (size_t)a.cand_cap;
  if (q < a.M_valid) {
    const uint32_t o = ordk_of(a.thr_keys[(size_t)q * a.thr_ld + a.thr_ld - 1]);
    s.thr = o ? o : 1u;
  }
}
__device__ __forceinline__ void stream_end(const GemmArgs& a, size_t region, const StreamLane& s) {
  a.cand_cnt[region] = s.n;
  if (a.cand_pmax) a.cand_pmax[region] = s.rkey;
}

// u-step of slice s of the list epilogue's S slices: spread evenly over u = 2 .. U-1
constexpr int list_slice_u(int s, int S, int U) {
  const int span = U > 3 ? U - 2 : 1;
  const int u = 2 + s * span / S;
  return u < U ? u : U - 1;
}

// ABL (tools/scan_probe only): 1 = no epilogue, 2 = no staging after the first tile,
// 4 = no per-tile wait + barrier, 8 = no S stores, 16 = no tile-maxima stores, 32 = no
// order-image / maxima arithmetic.
template <typename T, int KU, int ABL = 0>
__global__ __launch_bounds__(kScanWaves * 64, 1) void scan2_kernel(GemmArgs a, int n_chunks, int tiles_total) {
  constexpr int U = KU / 2;               // u-steps per tile (16-B chunk pairs)
  constexpr int ROWB = KU * 16;
  constexpr int TILE_B = 32 * ROWB;
  constexpr int G = (KU % 16 == 0) ? 8 : 4;  // u-steps sharing one swizzle period
  constexpr int PIECES = KU / 8;          // 1 KiB LDS-DMA pieces per wave per tile
  static_assert(ROWB <= kScanRowMax, "row too wide for the scan kernel");
  static_assert(KU % 8 == 0, "KU must split into whole 1 KiB pieces per wave");
  // three-deep tile ring: two tiles of LDS-DMA in flight behind the one being read.  Small
  // batches (B <= 128: one query group, 256 item chunks) are HBM-latency bound — one tile in
  // flight per CU delivered ~4.3 TB/s on a 10M-row index.
  constexpr int kRing = 3;
  __shared__ __attribute__((aligned(16))) char smem[kRing * TILE_B];

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

  // f16 operands: the re-rank copy of an f32 index (kScanF16); bf16 otherwise
  constexpr bool F16 = (ABL & kScanF16) != 0;
  static_assert(!F16 || sizeof(T) == 2, "f16 operands are 16-bit");
  // LDS fragment bases: chunk (2u + h) ^ swz(r) of row r = rd[u % G] + (u / G)·G·32 bytes
  const int swz = scan_swz<KU>(r);
  int rd[G];
#pragma unroll
  for (int m = 0; m < G; ++m) rd[m] = r * ROWB + (((2 * m + h) ^ swz) << 4);

  // LDS-DMA source offsets of this lane's 16 B in each of its pieces (tile-relative)
  const char* Xg = (const char*)a.X;
  const size_t ldxb = (size_t)a.ldx * sizeof(T);
  uint32_t soff[PIECES];
#pragma unroll
  for (int p = 0; p < PIECES; ++p) {
    const int mine = (wave * PIECES + p) * 1024 + lane * 16;
    const int row = mine / ROWB;
    const int ch = ((mine % ROWB) >> 4) ^ scan_swz<KU>(row);
    soff[p] = (uint32_t)(row * ldxb + ch * 16);
  }
  // Issued as inline asm: the compiler's waitcnt pass would otherwise (conservatively)
  // wait for the LDS-DMA to land before every later ds_read — i.e. expose the whole HBM
  // latency of the next tile inside this one.  Completion is enforced explicitly by the
  // vmcnt(0) + barrier at the end of each tile, before anyone reads the buffer.
  const uint32_t lds_base = (uint32_t)(size_t)((__attribute__((address_space(3))) char*)smem);
  auto stage_piece = [&](int tile, int buf, int p) __attribute__((always_inline)) {
    const char* src = Xg + (size_t)tile * 32 * ldxb + soff[p];
    const uint32_t dst = __builtin_amdgcn_readfirstlane(lds_base + buf * TILE_B + (wave * PIECES + p) * 1024);
    asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off" ::"s"(dst), "v"(src) : "memory");
  };

  // The first two tiles' LDS-DMA goes out before the query operand's loads, so the item
  // rows' latency overlaps the queries' instead of following it (the queries are pinned to
  // AGPRs below, a wait that now also retires these pieces; nothing reads LDS before the
  // explicit wait + barrier ahead of the first tile).
#pragma unroll
  for (int p = 0; p < PIECES; ++p) stage_piece(tile_lo, 0, p);
  {
    const int t1 = tile_lo + 1 < tile_hi ? tile_lo + 1 : tile_lo;
#pragma unroll
    for (int p = 0; p < PIECES; ++p) stage_piece(t1, 1, p);
  }
  // the query's code quantum (prep wrote it with the operand) is loaded ahead of the operand
  // too: one memory round trip for the whole prologue instead of two
  constexpr bool kHs = ((ABL & kScanS16) != 0 || (ABL & kScanList) != 0) && (ABL & kScanStream) == 0;
  float hs_pre = 0.f;
  if constexpr (kHs) {
    constexpr bool kS16b = (ABL & kScanS16) != 0;  // (the image path reads it whatever the prologue)
    if ((kS16b || !a.q_raw) && q < a.M_valid) hs_pre = a.s_h[q];
  }
  uint4 qf[U];
  const float hq_raw = scan2_load_queries<T, KU, F16>(a, q, h, qf, chunk == 0 && a.q_istats != nullptr);
  float qa[sizeof(T) == 4 ? 4 * U : 1];  // f32: the operand as 4U scalars, pinned to AGPRs
  if constexpr (sizeof(T) == 4) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      qa[4 * u + 0] = __uint_as_float(qf[u].x);
      qa[4 * u + 1] = __uint_as_float(qf[u].y);
      qa[4 * u + 2] = __uint_as_float(qf[u].z);
      qa[4 * u + 3] = __uint_as_float(qf[u].w);
    }
#pragma unroll
    for (int i = 0; i < 4 * U; ++i) asm volatile("" : "+a"(qa[i]));
  }
  u32x4v qv[sizeof(T) == 2 ? U : 1];  // bf16: the operand as 4-dword vectors, pinned to AGPRs
  if constexpr (sizeof(T) == 2) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      qv[u] = __builtin_bit_cast(u32x4v, qf[u]);
      asm volatile("" : "+a"(qv[u]));
    }
  }

  const size_t w0 = (size_t)(a.slab_start >> 5);
  const uint32_t* erow = a.excl + (size_t)(q < a.M_valid ? q : a.M_valid - 1) * a.excl_ld;
  // score image: the blocked layout (sblk_quad) — store j of a tile writes the wave's 16
  // accumulator quads j as one contiguous 1-KiB block (512 B as int16), eight full lines,
  // where row-major S took 32 partial lines per store
  const size_t sblk0 = sblk_lane(q, h, a.ldt);  // + (tile·4 + j)·256
  constexpr bool STREAM = (ABL & kScanStream) != 0;
  // int16 score image: this query's code scale 1/(h·32767) (h = 0: zero row, codes 0)
  constexpr bool S16 = (ABL & kScanS16) != 0 && !STREAM;
  float sk = 0.f;
  if constexpr (S16) {
    const float hq = hs_pre;  // (a.s_h[q] for q < M_valid, loaded above)
    sk = hq > 0.f ? 1.0f / (hq * 32767.f) : 0.f;
    asm volatile("" : "+v"(sk));  // consumed before any LDS-DMA is in flight
  }
  // bounded candidate lists (list_epi.h): code scale k2 = 1/(65535·h), the lane's top-5 of
  // the current period, the rank-0 top-2, the period counters (wave-uniform)
  constexpr bool LIST = (ABL & kScanList) != 0 && !STREAM && !S16;
  float k2 = 0.f;
  if constexpr (LIST) {
    const float hq = a.q_raw ? hq_raw : hs_pre;
    k2 = hq > 0.f ? 1.0f / (hq * 65535.f) : 0.f;
    asm volatile("" : "+v"(k2));  // consumed before any LDS-DMA is in flight
  }
  ListTop5 lst;
  ListTop2 r0l;
  uint32_t l_e16 = 0, l_pb2 = 0, l_kodd = 0;
  bool l_full = true;
  int l_cnt = 0, l_period = 0;
  const int l_nb = a.Mpad >> 5, l_blk = q >> 5;
  const bool l_live = __any(q < a.M_valid);  // padded query blocks store nothing
  auto list_store = [&]() __attribute__((always_inline)) {
    if (l_live)
      *(uint4*)(a.lists + 4 * list_slot(chunk, l_period, a.l_np, l_nb, l_blk, lane)) = lst.pack();
    lst.reset();
    l_cnt = 0;
    ++l_period;
  };
  StreamLane sl;
  const size_t region = ((size_t)q * n_chunks + chunk) * 2 + h;
  if constexpr (STREAM) stream_begin(a, q, region, sl);

  // (the first two tiles' LDS-DMA was issued before the query loads, above: both latencies
  // overlap; this wait retires them all)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  asm volatile("s_nop 4");

  f32x16s accE = {}, accO = {};
  uint32_t pw = 0, mw = 0, ew = 0;     // eligibility words of the tile whose epilogue is pending
  uint32_t nw_p = 0, nw_m = 0, nw_e = 0;

  // One tile: ONE accumulation chain (back-to-back dependent MFMAs run at full rate) over
  // LDS buffer BUF into c; woven in: the previous tile's epilogue on p (EPI), this tile's
  // eligibility words, the next tile's staging into BUF^1.  On the f32 MFMA, VALU work does
  // NOT overlap (it holds the SIMD's vector issue), so the epilogue is kept to ~25 VALU in
  // the common all-eligible case (tile_maxima fast path).
  constexpr int kEpiSlices = 8 + PIECES;
  auto tile_body = [&](int buf, auto EPI, int tile, f32x16s& c, const f32x16s& p) __attribute__((always_inline)) {
    const int sbuf = buf == 0 ? 2 : buf - 1;  // (buf + 2) % kRing: the buffer tile-1 used
    constexpr bool epi = decltype(EPI)::value && !(ABL & 1);
    const int ptile = tile - 1;
    const int stile = tile + 2 < tile_hi ? tile + 2 : tile_hi - 1;  // branch-free staging target
    uint32_t te = 0, tp = 0;
    const int ptile0 = ptile * 32;
    // item fragments: ds_read issued two u-steps ahead of their MFMAs
    auto frag = [&](int u) __attribute__((always_inline)) {
      return *(const uint4*)(smem + buf * TILE_B + rd[u % G] + (u / G) * G * 32);
    };
    // 4-slot ring, prefetch distance 2; fragments stay live one step past their MFMAs
    // (see scan3_kernel.h: inline-asm MFMAs are opaque to hazard tracking)
    uint4 fq[4];
    fq[0] = frag(0);
    if constexpr (U > 1) fq[1] = frag(1);
    static_for<U>([&](auto UU) {
      constexpr int u = decltype(UU)::value;
      if constexpr (u + 2 < U) fq[(u + 2) % 4] = frag(u + 2);
      const uint4 fa = fq[u % 4];
      // MFMAs as inline asm so the resident query operand stays in AGPRs (srcB may be an
      // AGPR on gfx950) and the accumulator in VGPRs (read by the epilogue without copies).
      if constexpr (sizeof(T) == 4) {
        const float pa[4] = {__uint_as_float(fa.x), __uint_as_float(fa.y), __uint_as_float(fa.z),
                             __uint_as_float(fa.w)};
#pragma unroll
        for (int cc = 0; cc < 4; ++cc) {
          if (u == 0 && cc == 0)
            asm volatile("v_mfma_f32_32x32x2_f32 %0, %1, %2, 0" : "=&v"(c) : "v"(pa[cc]), "a"(qa[4 * u + cc]));
          else
            asm volatile("v_mfma_f32_32x32x2_f32 %0, %1, %2, %0" : "+v"(c) : "v"(pa[cc]), "a"(qa[4 * u + cc]));
        }
      } else {
        const u32x4v fv = __builtin_bit_cast(u32x4v, fa);
        if constexpr (F16) {
          if constexpr (u == 0)
            asm volatile("v_mfma_f32_32x32x16_f16 %0, %1, %2, 0" : "=&v"(c) : "v"(fv), "a"(qv[u]));
          else
            asm volatile("v_mfma_f32_32x32x16_f16 %0, %1, %2, %0" : "+v"(c) : "v"(fv), "a"(qv[u]));
        } else {
          if constexpr (u == 0)
            asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, 0" : "=&v"(c) : "v"(fv), "a"(qv[u]));
          else
            asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(c) : "v"(fv), "a"(qv[u]));
        }
      }
      if constexpr (u > 0) asm volatile("" ::"v"(__builtin_bit_cast(u32x4v, fq[(u + 3) % 4])));
      // ---- list epilogue (kScanList): eligibility, 16 half-pair slices (codes, keys, top-5
      // inserts), rank 0, the period store, then the next tile's words and staging ----
      if constexpr (LIST) {
        constexpr int kLS = 20 + PIECES;
        static_for<kLS>([&](auto SS) {
          constexpr int s = decltype(SS)::value;
          if constexpr (list_slice_u(s, kLS, U) == u) {
            if constexpr (s == 0) {
              if constexpr (epi) {
                l_e16 = list_elig16(pw & mw & ~ew, ptile0, a.n_valid, h);
                l_full = __all(l_e16 == 0xFFFFu);
                l_pb2 = list_pb2(l_cnt);  // ptile's place in the period
              }
            } else if constexpr (s <= 16) {
              if constexpr (epi) {
                constexpr int pp = (s - 1) >> 1;
                if constexpr (((s - 1) & 1) == 0) {
                  uint32_t w = list_codes(p[2 * pp], p[2 * pp + 1], k2);
                  if (!l_full) {
                    const uint32_t lo = 0u - ((l_e16 >> (2 * pp)) & 1u), hi = 0u - ((l_e16 >> (2 * pp + 1)) & 1u);
                    w &= (lo & 0xFFFFu) | (hi & 0xFFFF0000u);
                  }
                  const uint32_t ix = l_pb2 + list_pair_pos(pp);
                  lst.ins(__builtin_amdgcn_perm(w, ix, 0x05040100u));
                  l_kodd = __builtin_amdgcn_perm(w, ix, 0x07060302u);
                } else {
                  lst.ins(l_kodd);
                }
              }
            } else if constexpr (s == 17) {
              if constexpr (epi) {
                if (a.r0lists) {
                  const float m = list_present_max(p, list_elig16(pw, ptile0, a.n_valid, h));
                  r0l.ins(list_r0_key(m, k2, (uint32_t)(ptile - tile_lo)));
                }
              }
            } else if constexpr (s == 18) {
              if constexpr (epi) {
                if (++l_cnt == a.l_period) list_store();
              }
            } else if constexpr (s == 19) {
              asm volatile("global_load_dword %0, %1, off" : "=v"(nw_p) : "v"(a.present + w0 + tile) : "memory");
              asm volatile("global_load_dword %0, %1, off" : "=v"(nw_m) : "v"(a.mask + w0 + tile) : "memory");
              asm volatile("global_load_dword %0, %1, off" : "=v"(nw_e) : "v"(erow + w0 + tile) : "memory");
            } else {
              if constexpr (!(ABL & 2)) stage_piece(stile, sbuf, s - 20);
            }
          }
        });
        return;
      }
      // ---- slices scheduled on this u-step: slice s runs at u = min(U-1, s+2) ----
      static_for<kEpiSlices>([&](auto SS) {
        constexpr int s = decltype(SS)::value;
        constexpr int su = (s + 2 < U) ? s + 2 : U - 1;
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
              const size_t e = sblk0 + (size_t)(ptile * 4 + j) * 256;
              if constexpr (S16)
                *(uint2*)((int16_t*)a.S + e) =
                    make_uint2(s16_pack(p[4 * j], p[4 * j + 1], sk), s16_pack(p[4 * j + 2], p[4 * j + 3], sk));
              else
                *(float4*)(a.S + e) = make_float4(p[4 * j], p[4 * j + 1], p[4 * j + 2], p[4 * j + 3]);
            }
          } else if constexpr (s == 6) {
            if constexpr (epi && !(ABL & 16) && !STREAM) {
              if (!h || a.pmax) (h ? a.pmax : a.tmax)[(size_t)q * a.ldt + ptile] = h ? tp : te;
            }
          } else if constexpr (s == 7) {
            // as inline asm: a compiler-visible load would get a compiler wait before its
            // first use that also waits for the (asm, invisible) DMA of tile + 2; these
            // complete under the explicit end-of-tile wait (they are older than the DMA)
            asm volatile("global_load_dword %0, %1, off" : "=v"(nw_p) : "v"(a.present + w0 + tile) : "memory");
            asm volatile("global_load_dword %0, %1, off" : "=v"(nw_m) : "v"(a.mask + w0 + tile) : "memory");
            asm volatile("global_load_dword %0, %1, off" : "=v"(nw_e) : "v"(erow + w0 + tile) : "memory");
          } else {
            if constexpr (!(ABL & 2)) stage_piece(stile, sbuf, s - 8);
          }
        }
      });
    });
    // The MFMAs are inline asm, so the compiler cannot see their result latency: this
    // ties the accumulator to a wait long enough for the last MFMA to retire, before any
    // register copy or read of it the compiler may place after this point.
    asm volatile("s_nop 15\n\ts_nop 15\n\ts_nop 15\n\ts_nop 15" : "+v"(c));
    // The eligibility words were loaded by asm (destinations count as written at the asm's
    // end): the wait names them "+v" in the SAME statement, so no use or copy of them moves
    // before it; between the loads and this wait nothing may touch those registers, which
    // tests/test_asm_hazard.py checks on the shipped code object (CFG walk, vmcnt counted).
    if constexpr (!(ABL & 4)) {
      // the last PIECES vector-memory ops are tile + 2's DMA (the staging slices come
      // last, asm "memory" clobbers keep that order): leave them in flight
      if constexpr (ABL & 2)
        asm volatile("s_waitcnt vmcnt(0)" : "+v"(nw_p), "+v"(nw_m), "+v"(nw_e) : : "memory");
      else
        asm volatile("s_waitcnt vmcnt(%3)" : "+v"(nw_p), "+v"(nw_m), "+v"(nw_e) : "n"(PIECES) : "memory");
      __syncthreads();
    } else {
      asm volatile("s_waitcnt vmcnt(0)" : "+v"(nw_p), "+v"(nw_m), "+v"(nw_e) : : "memory");  // (probe)
    }
    pw = nw_p;
    mw = nw_m;
    ew = nw_e;
  };

  // final epilogue of the last tile (not overlapped)
  auto last_epilogue = [&](int tile, const f32x16s& p) __attribute__((always_inline)) {
    if constexpr (ABL & 1) return;
    asm volatile("s_nop 15\n\ts_nop 15\n\ts_nop 15\n\ts_nop 15");  // asm-MFMA result -> VALU read
    if constexpr (LIST) {
      const uint32_t e16 = list_elig16(pw & mw & ~ew, tile * 32, a.n_valid, h);
      const bool full = __all(e16 == 0xFFFFu);
      const uint32_t pb2 = list_pb2(l_cnt);
#pragma unroll
      for (int pp = 0; pp < 8; ++pp) list_pair(lst, p[2 * pp], p[2 * pp + 1], k2, pb2, pp, full, e16);
      if (a.r0lists) {
        const float m = list_present_max(p, list_elig16(pw, tile * 32, a.n_valid, h));
        r0l.ins(list_r0_key(m, k2, (uint32_t)(tile - tile_lo)));
        if (l_live)
          *(uint2*)(a.r0lists + 2 * list_slot(chunk, 0, 1, l_nb, l_blk, lane)) = make_uint2(r0l.k0, r0l.k1);
      }
      list_store();  // the last (possibly partial) period
      return;
    }
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
    for (int j = 0; j < 4; ++j) {
      const size_t e = sblk0 + (size_t)(tile * 4 + j) * 256;
      if constexpr (S16)
        *(uint2*)((int16_t*)a.S + e) =
            make_uint2(s16_pack(p[4 * j], p[4 * j + 1], sk), s16_pack(p[4 * j + 2], p[4 * j + 3], sk));
      else
        *(float4*)(a.S + e) = make_float4(p[4 * j], p[4 * j + 1], p[4 * j + 2], p[4 * j + 3]);
    }
    if (!h || a.pmax) (h ? a.pmax : a.tmax)[(size_t)q * a.ldt + tile] = h ? tp : te;
  };

  using EY = std::integral_constant<bool, true>;
  using EN = std::integral_constant<bool, false>;
  tile_body(0, EN{}, tile_lo, accE, accO);
  int tile = tile_lo + 1, buf = 1;  // tile t reads buffer (t - tile_lo) % kRing
  for (;;) {
    if (tile >= tile_hi) {
      last_epilogue(tile - 1, accE);
      break;
    }
    tile_body(buf, EY{}, tile, accO, accE);
    ++tile;
    buf = buf == kRing - 1 ? 0 : buf + 1;
    if (tile >= tile_hi) {
      last_epilogue(tile - 1, accO);
      break;
    }
    tile_body(buf, EY{}, tile, accE, accO);
    ++tile;
    buf = buf == kRing - 1 ? 0 : buf + 1;
  }
  if constexpr (STREAM) stream_end(a, region, sl);
}

}  // namespace bb
