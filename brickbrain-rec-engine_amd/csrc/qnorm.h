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

__device__ __forceinline__ double qn_wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
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

__device__ __forceinline__ float qn_elem(double x, double nrm) { return (float)(x / nrm); }

}  // namespace bb
