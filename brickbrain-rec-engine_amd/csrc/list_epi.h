// list_epi.h — the bounded candidate-list epilogue of the query-resident scans (kScanList).
//
// Replaces the score image of the exact re-rank path (one slab, f32 index: every 25K-row
// config).  Instead of writing B×N int16 codes that a select kernel re-reads, each lane keeps
// the top-5 keys of its own items in registers and writes them once per list period:
//
//   key  = (code << 16) | pos          code = u16 image of the approximate score,
//                                      c = round(65535·(0.5 + s/(65535·h))) ≈ 32767.5 + s/h
//                                      pos  = (tile within the period << 4) | accumulator
//                                      register g (item (g & 3) + 8 (g >> 2) + 4·half)
//   list = the 5 largest keys over the lane's eligible items of one period (G <= 8 tiles ×
//          16 items), packed into 128 bits: five codes + five 7-bit positions (list_pack5)
//
// The select (select_list.hip) bounds the K-th approximate score by the K-th largest list
// key, takes every key within the re-rank margin of it, and enumerates exhaustively only the
// lists whose 5th key still lies inside the margin (they may have dropped a candidate).
// Rank 0 (similar / hybrid content side): the top-2 present half-tile maxima per lane and
// item chunk, (code << 16) | tile offset.
//
// Codes: |s| <= 16384·h (rr_quantum's floor), so c stays inside (16383, 49152): never 0,
// which marks an empty or ineligible slot.  Encode (fma + v_cvt_pknorm_u16_f32, any rounding)
// and decode (c − 32767.5)·h differ from s by at most 1.01·h (fma / convert rounding of values
// below 1 at 2^-24, ×65535); prep's ε' = (ε + 1.01·h)(1 + 2^-20) bounds |decoded − exact| and
// the select adds two more codes of slack.
#pragma once
#include "common.h"

namespace bb {

__device__ __forceinline__ uint32_t med3u(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t r;
  asm("v_med3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}
__device__ __forceinline__ uint32_t maxu(uint32_t a, uint32_t b) { return a > b ? a : b; }

// two approximate scores -> two u16 codes (lo = a, hi = b); k2 = 1 / (65535·h)
__device__ __forceinline__ uint32_t list_codes(float a, float b, float k2) {
  return __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_pknorm_u16(fmaf(a, k2, 0.5f), fmaf(b, k2, 0.5f)));
}

// per-lane sorted top-5 (k0 >= ... >= k4): one max + four med3, no dependent chain
struct ListTop5 {
  uint32_t k0 = 0, k1 = 0, k2 = 0, k3 = 0, k4 = 0;
  __device__ __forceinline__ void ins(uint32_t x) {
    const uint32_t n0 = maxu(k0, x), n1 = med3u(k0, k1, x), n2 = med3u(k1, k2, x), n3 = med3u(k2, k3, x),
                   n4 = med3u(k3, k4, x);
    k0 = n0;
    k1 = n1;
    k2 = n2;
    k3 = n3;
    k4 = n4;
  }
  __device__ __forceinline__ void reset() { k0 = k1 = k2 = k3 = k4 = 0u; }
  // 128 bits: x = c0:c1, y = c2:c3, z = c4 : p0 (7 b) : p1 (7 b), w = p2 : p3 : p4 (7 b each)
  __device__ __forceinline__ uint4 pack() const {
    return make_uint4((k0 & 0xFFFF0000u) | (k1 >> 16), (k2 & 0xFFFF0000u) | (k3 >> 16),
                      (k4 & 0xFFFF0000u) | ((k0 & 0x7Fu) << 7) | (k1 & 0x7Fu),
                      ((k2 & 0x7Fu) << 14) | ((k3 & 0x7Fu) << 7) | (k4 & 0x7Fu));
  }
};
// unpacked list: codes c[0..4] (descending) and positions p[0..4]
__host__ __device__ inline void list_unpack5(uint4 v, uint32_t c[5], uint32_t p[5]) {
  c[0] = v.x >> 16;
  c[1] = v.x & 0xFFFFu;
  c[2] = v.y >> 16;
  c[3] = v.y & 0xFFFFu;
  c[4] = v.z >> 16;
  p[0] = (v.z >> 7) & 0x7Fu;
  p[1] = v.z & 0x7Fu;
  p[2] = (v.w >> 14) & 0x7Fu;
  p[3] = (v.w >> 7) & 0x7Fu;
  p[4] = v.w & 0x7Fu;
}
constexpr int kListMaxPeriod = 8;  // tiles per period: 7-bit positions
constexpr int kListMaxPerRow = 512;  // lists per query row (2·chunks·periods) the list select takes

struct ListTop2 {
  uint32_t k0 = 0, k1 = 0;
  __device__ __forceinline__ void ins(uint32_t x) {
    const uint32_t n0 = maxu(k0, x), n1 = med3u(k0, k1, x);
    k0 = n0;
    k1 = n1;
  }
};

// positions of accumulator register pair p (registers 2p, 2p+1) of tile t of the period,
// both in one word (lo = register 2p, hi = 2p + 1): list_pb2(t) + list_pair_pos(p)
__host__ __device__ constexpr uint32_t list_pair_pos(int p) { return (uint32_t)(2 * p) * 0x10001u + 0x10000u; }
__host__ __device__ constexpr uint32_t list_pb2(int t_in_period) { return (uint32_t)(t_in_period << 4) * 0x10001u; }

// Insert one register pair of a half tile.  e16: bit g = register g eligible (ignored when
// full).  Masked registers get code 0 (their keys sort below every real key).
__device__ __forceinline__ void list_pair(ListTop5& L, float a, float b, float k2, uint32_t pb2, int p, bool full,
                                          uint32_t e16) {
  uint32_t w = list_codes(a, b, k2);
  if (!full) {
    const uint32_t lo = 0u - ((e16 >> (2 * p)) & 1u), hi = 0u - ((e16 >> (2 * p + 1)) & 1u);
    w &= (lo & 0xFFFFu) | (hi & 0xFFFF0000u);
  }
  const uint32_t ix = pb2 + list_pair_pos(p);
  L.ins(__builtin_amdgcn_perm(w, ix, 0x05040100u));
  L.ins(__builtin_amdgcn_perm(w, ix, 0x07060302u));
}

// This lane's registers of a half tile as a 16-bit mask (bit g = register g): in range and
// set in the item word w (eligibility, or presence for rank 0).
__device__ __forceinline__ uint32_t list_elig16(uint32_t w, int tile0, int n_valid, int h) {
  const int rem = n_valid - tile0;
  const uint32_t inr = rem >= 32 ? 0xFFFFFFFFu : rem <= 0 ? 0u : ((1u << rem) - 1u);
  const uint32_t v = (w & inr) >> (4 * h);  // register g <-> item (g & 3) + 8 (g >> 2) + 4h
  return (v & 0xFu) | ((v >> 4) & 0xF0u) | ((v >> 8) & 0xF00u) | ((v >> 12) & 0xF000u);
}

// Present maximum of this lane's half tile as a float (-inf when none): rank-0 tracking.
// pe16: bit g = register g present and in range.
template <typename V>
__device__ __forceinline__ float list_present_max(const V& p, uint32_t pe16) {
  auto max3 = [](float x, float y, float z) {
    float m;
    asm("v_max3_f32 %0, %1, %2, %3" : "=v"(m) : "v"(x), "v"(y), "v"(z));
    return m;
  };
  if (__all(pe16 == 0xFFFFu)) {
    const float m0 = max3(p[0], p[1], p[2]), m1 = max3(p[3], p[4], p[5]), m2 = max3(p[6], p[7], p[8]);
    const float m3 = max3(p[9], p[10], p[11]), m4 = max3(p[12], p[13], p[14]);
    return max3(max3(m0, m1, m2), max3(m3, m4, p[15]), p[15]);
  }
  float m = -__builtin_inff();
#pragma unroll
  for (int g = 0; g < 16; ++g) m = ((pe16 >> g) & 1u) ? fmaxf(m, p[g]) : m;
  return m;
}

// rank-0 key of a half tile: (code << 16) | tile offset; 0 when nothing is present
__device__ __forceinline__ uint32_t list_r0_key(float m, float k2, uint32_t toff) {
  const uint32_t c = list_codes(m, m, k2) & 0xFFFFu;
  return c ? (c << 16) | toff : 0u;
}

// Tiles of item chunk c (the scans' balanced split) and list geometry shared by host and
// device: lists of chunk c, period p, lane (h, r) of 32-query block b at
// ((c·np + p)·NB + b)·64 + h·32 + r (uint4); rank-0 pairs at (c·NB + b)·64 + h·32 + r (uint2).
// (32-bit: the list geometry keeps chunks <= 256 and tiles < 2^24, so c·tiles < 2^32; the
// scans' 64-bit split gives the same value)
__host__ __device__ inline int chunk_tile_lo(int c, int tiles, int n_chunks) {
  return (int)((uint32_t)c * (uint32_t)tiles / (uint32_t)n_chunks);
}
__host__ __device__ inline size_t list_slot(int c, int p, int np, int nb, int b, int lane) {
  return (((size_t)c * np + p) * nb + b) * 64 + lane;
}

}  // namespace bb
