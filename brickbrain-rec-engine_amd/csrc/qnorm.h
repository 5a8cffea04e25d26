// qnorm.h — the query-row normalisation of the exact re-rank path, shared by prep_kernel
// and the list select's raw-query path (select_list.hip) so both produce the same f32 row
// bit for bit: sklearn.preprocessing.normalize (which cosine_similarity applies to its
// arguments, recommendation_system.py:214) with the sum of squares accumulated in f64.
//
// One wave per row, rows up to 512 wide: lane l holds elements l + 64c (c < 8, zero past the
// row); sum of squares by fma in c order, then the shfl_xor butterfly; norm = sqrt, a zero
// norm becomes 1; element = (float)(x / norm) (a true f64 division, rounded to f32).
#pragma once
#include "common.h"

namespace bb {

constexpr int kQnC = 8;  // elements per lane: rows up to 64·8 = 512 wide

// f64 lane value from `CTRL`'s DPP source lane (both halves moved; every lane active)
template <int CTRL>
__device__ __forceinline__ double qn_dpp(double v) {
  const uint64_t u = __builtin_bit_cast(uint64_t, v);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)u, CTRL, 0xF, 0xF, false);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)(u >> 32), CTRL, 0xF, 0xF, false);
  return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}

// Wave sum by the xor butterfly 32, 16, 8, 4, 2, 1.  The last four steps are DPP row rotations
// (row_ror 8, 4, 2, 1): after the steps above them a lane's value equals its partners' at the
// xor distances already summed, so the rotation reads the same value the xor partner holds —
// the same additions in the same order as __shfl_xor at every step (the same bits), without
// the LDS permute round trips.  Every lane of the wave must be active.
__device__ __forceinline__ double qn_wave_sum(double v) {
  v += __shfl_xor(v, 32);
  v += __shfl_xor(v, 16);
  v += qn_dpp<0x128>(v);  // row_ror:8
  v += qn_dpp<0x124>(v);  // row_ror:4
  v += qn_dpp<0x122>(v);  // row_ror:2
  v += qn_dpp<0x121>(v);  // row_ror:1
  return v;
}

// f64 norm of the wave's row (x[c] = element lane + 64c as f64, zero past the row); 1 for a
// zero row
__device__ __forceinline__ double qn_norm(const double (&x)[kQnC]) {
  double ss = 0.0;
#pragma unroll
  for (int c = 0; c < kQnC; ++c) ss = fma(x[c], x[c], ss);
  ss = qn_wave_sum(ss);
  const double nrm = sqrt(ss);
  return nrm == 0.0 ? 1.0 : nrm;
}

// (float)(x / nrm) — the f64 quotient rounded to f32 — from rinv = 1 / nrm (one division per
// row): q = x·rinv is within 2^-51.9 (relative) of x / nrm and of its correctly rounded f64
// quotient; when q·(1 ∓ 2^-50) round to the same f32, so does that quotient (f32 rounding is
// monotonic), and only a q within that distance of an f32 rounding boundary (a fraction
// ~2^-27 of elements) divides.  The same bits as the division, for ~1/10 of its dependent f64
// latency per element.
__device__ __forceinline__ float qn_elem(double x, double nrm, double rinv) {
  const double q = x * rinv, e = fabs(q) * 0x1p-50;
  const float lo = (float)(q - e), hi = (float)(q + e);
  return lo == hi ? lo : (float)(x / nrm);
}

// Load C elements per lane (i = base + lane + 64c, zero past `d`) with the dtype switch
// outside the loads, so all C loads are in flight together: every load is unconditional (the
// index clamped to the row, d >= 1) and the zero is selected afterwards — a conditional load
// puts each element in a basic block of its own behind its own s_waitcnt vmcnt(0).
template <int C>
__device__ __forceinline__ void load_chunk(const void* p, int dt, size_t sb, int base, int d, int lane,
                                           double (&x)[C]) {
  if (dt == F32) {
    const float* q = (const float*)p + sb;
    float v[C];
#pragma unroll
    for (int c = 0; c < C; ++c) v[c] = q[min(base + lane + 64 * c, d - 1)];
#pragma unroll
    for (int c = 0; c < C; ++c) x[c] = base + lane + 64 * c < d ? (double)v[c] : 0.0;
  } else if (dt == F64) {
    const double* q = (const double*)p + sb;
    double v[C];
#pragma unroll
    for (int c = 0; c < C; ++c) v[c] = q[min(base + lane + 64 * c, d - 1)];
#pragma unroll
    for (int c = 0; c < C; ++c) x[c] = base + lane + 64 * c < d ? v[c] : 0.0;
  } else {
    const uint16_t* q = (const uint16_t*)p + sb;
    uint32_t v[C];
#pragma unroll
    for (int c = 0; c < C; ++c) v[c] = q[min(base + lane + 64 * c, d - 1)];
#pragma unroll
    for (int c = 0; c < C; ++c)
      x[c] = base + lane + 64 * c < d ? (double)__builtin_bit_cast(float, v[c] << 16) : 0.0;
  }
}

}  // namespace bb
