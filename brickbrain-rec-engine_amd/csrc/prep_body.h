// prep_body.h — query preparation, one wave per query row (prep_kernel / prep2_kernel in
// misc.hip, and the query workgroups of compact_kernel, compact.hip): normalise query rows
// (semantic), gather the stored rows of liked sets, or copy CF user rows, into the scan's
// operand (index dtype, f16 re-rank operand with its f32 row + bound, or scan3 planes).
#pragma once
#include "common.h"
#include "qnorm.h"

namespace bb {

__device__ __forceinline__ float load_elem(const void* p, int dtype, size_t i) {
  if (dtype == F32) return ((const float*)p)[i];
  if (dtype == BF16) return __builtin_bit_cast(float, (uint32_t)((const uint16_t*)p)[i] << 16);
  return (float)((const double*)p)[i];
}
__device__ __forceinline__ double load_elem_d(const void* p, int dtype, size_t i) {
  if (dtype == F64) return ((const double*)p)[i];
  return (double)load_elem(p, dtype, i);
}
__device__ __forceinline__ void store_elem(void* p, int dtype, size_t i, float v) {
  if (dtype == BF16)
    ((uint16_t*)p)[i] = to_bf16(v);
  else if (dtype == F16)
    ((uint16_t*)p)[i] = to_f16(v);
  else
    ((float*)p)[i] = v;
}

__device__ __forceinline__ double wave_sum(double v) { return qn_wave_sum(v); }

__device__ __forceinline__ void split3_bits(float v, uint16_t& h, uint16_t& m, uint16_t& l) {
  auto rne = [](float f) -> uint32_t {
    uint32_t u = __float_as_uint(f);
    u += 0x7FFFu + ((u >> 16) & 1u);
    return u >> 16;
  };
  const uint32_t hb = rne(v);
  const float r = v - __uint_as_float(hb << 16);
  const uint32_t mb = rne(r);
  h = (uint16_t)hb;
  m = (uint16_t)mb;
  l = (uint16_t)rne(r - __uint_as_float(mb << 16));
}

// ---------------------------------------------------------------------------------------
// query preparation: normalise query rows (semantic), or gather the stored (already
// normalised) item rows of the liked sets (similar-sets: the query IS feat_matrix[target],
// recommendation_system.py:213), or copy user factor rows (CF, :435).  Rows >= B are zero.
// ---------------------------------------------------------------------------------------
constexpr int kPrepC = kQnC;  // rows up to 512 wide stay in registers (one load round)

// f32 -> three bf16 planes (x = xh + xm + xl exactly) for the split-precision scan

// store element i of output row `row`: index dtype, or SPLIT3 planes in the scan3 fragment
// image (q3f_chunk_offset, scan3_kernel.h), so each query load of the scan is one 1-KiB
// coalesced wave access
__device__ __forceinline__ void store_q(const PrepArgs& a, int row, int i, float v) {
  if (a.out_dtype == SPLIT3) {
    const int U = a.Dpad >> 4;
    uint16_t* o = (uint16_t*)((char*)a.out + q3f_chunk_offset(row, i >> 3, 0, U)) + (i & 7);
    const size_t plane = (size_t)U * 64 * 8;  // bf16 elements between planes of one wave
    uint16_t h, m, l;
    split3_bits(v, h, m, l);
    o[0] = h;
    o[plane] = m;
    o[2 * plane] = l;
  } else if (a.q_perm) {  // bf16 operand in the scan's lane order
    const size_t o = a.q_perm == 2 ? scan2_q_offset(row, i >> 3, a.Dpad >> 4) : scan4_q_offset(row, i >> 3, a.Dpad >> 4);
    ((uint16_t*)a.out)[o * 8 + (i & 7)] = a.out_dtype == F16 ? to_f16(v) : to_bf16(v);
  } else {
    store_elem(a.out, a.out_dtype, (size_t)row * a.Dpad + i, v);
  }
}

// Re-rank outputs of one query row (PrepArgs.out_f32): the f32 element beside the f16
// operand, and ε = E_x·|q̃| + N_x·|q̃−q| + γ·Ñ_x·|q̃| — Cauchy-Schwarz on
// Σ(x̃−x)q̃ + Σx(q̃−q), plus γ = kRrGamma·Dpad for the MFMA f32 accumulation of Σx̃q̃.
struct RrAcc {
  double e2 = 0.0, b2 = 0.0;
  __device__ __forceinline__ void add(const PrepArgs& a, int row, int i, float v) {
    if (i < a.Dpad_f) a.out_f32[(size_t)row * a.Dpad_f + i] = v;
    const double bv = (double)f16_val(to_f16(v));
    e2 += ((double)v - bv) * ((double)v - bv);
    b2 += bv * bv;
  }
  __device__ __forceinline__ void finish(const PrepArgs& a, int row, int lane) {
    const double e = sqrt(wave_sum(e2)), b = sqrt(wave_sum(b2));
    if (lane == 0) {
      const double gam = kRrGamma * (double)a.Dpad;
      const double eps = (double)a.istats[0] * b + (double)a.istats[1] * e + gam * (double)a.istats[2] * b;
      if (a.h_out) {  // int16 score image: its quantum, and ε widened to cover the codes
        rr_quantum(eps * (1.0 + 0x1p-20), b, (double)a.istats[2], a.eps_out[row], a.h_out[row]);
      } else {
        a.eps_out[row] = __double2float_ru(eps * (1.0 + 0x1p-20));
      }
    }
  }
};

__device__ __forceinline__ void prep_rows(const PrepArgs& a, int blk) {
  const int row = blk * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= a.Bpad) return;
  const void* src = a.src;
  int sdt = a.src_dtype, d = a.d, norm_on = a.normalize;
  size_t sb = (size_t)row * a.src_ld;
  bool zero = row >= a.B;
  if (!zero && a.item_ids) {  // stored rows are already normalised and padded
    const int64_t lid = a.item_ids[row] - a.id_offset;
    zero = !(lid >= 0 && lid < a.n_items);
    src = a.items;
    sdt = a.out_dtype == SPLIT3 || a.out_f32 ? F32 : a.out_dtype;
    d = a.out_f32 ? a.Dpad_f : a.Dpad;   // re-rank: the f32 rows (stride Dpad_f)
    norm_on = 0;
    sb = zero ? 0 : (size_t)lid * d;
  }
  if (zero) {
    for (int i = lane; i < a.Dpad; i += 64) store_q(a, row, i, 0.f);
    if (a.out_f32) {
      for (int i = lane; i < a.Dpad_f; i += 64) a.out_f32[(size_t)row * a.Dpad_f + i] = 0.f;
      if (lane == 0) a.eps_out[row] = 0.f;
      if (lane == 0 && a.h_out) a.h_out[row] = 0.f;
    }
    return;
  }
  RrAcc rr;
  if (a.Dpad <= 64 * kPrepC) {
    double x[kPrepC];
    load_chunk<kPrepC>(src, sdt, sb, 0, d, lane, x);
    const double norm = norm_on ? qn_norm(x) : 1.0;  // (qnorm.h: the list select's raw path shares it)
    const double rinv = 1.0 / norm;
#pragma unroll
    for (int c = 0; c < kPrepC; ++c) {
      const int i = lane + 64 * c;
      if (i < a.Dpad) {
        const float v = qn_elem(x[c], norm, rinv);
        store_q(a, row, i, v);
        if (a.out_f32) rr.add(a, row, i, v);
      }
    }
    if (a.out_f32) rr.finish(a, row, lane);
    return;
  }
  double norm = 1.0;
  if (norm_on) {
    double ss = 0.0;
    for (int base = 0; base < d; base += 64 * kPrepC) {
      double x[kPrepC];
      load_chunk<kPrepC>(src, sdt, sb, base, d, lane, x);
#pragma unroll
      for (int c = 0; c < kPrepC; ++c) ss += x[c] * x[c];
    }
    ss = wave_sum(ss);
    norm = sqrt(ss);
    if (norm == 0.0) norm = 1.0;
  }
  for (int base = 0; base < a.Dpad; base += 64 * kPrepC) {
    double x[kPrepC];
    load_chunk<kPrepC>(src, sdt, sb, base, d, lane, x);
#pragma unroll
    for (int c = 0; c < kPrepC; ++c) {
      const int i = base + lane + 64 * c;
      if (i < a.Dpad) {
        const float v = qn_elem(x[c], norm, 1.0 / norm);
        store_q(a, row, i, v);
        if (a.out_f32) rr.add(a, row, i, v);
      }
    }
  }
  if (a.out_f32) rr.finish(a, row, lane);
}

}  // namespace bb
