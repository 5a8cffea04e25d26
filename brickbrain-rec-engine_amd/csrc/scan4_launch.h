// scan4_launch.h — launch bodies of the 64-queries-per-wave scan (scan4_kernel.h), one template
// per kernel family; each scan4_*.hip translation unit instantiates a few row widths, so the
// instances (minutes each at d = 384 / 768) compile in parallel.
#pragma once
#include "scan4_kernel.h"

namespace bb {

// the exact re-rank path (the f16 copy of an f32 index): list / int16-image / f32-slab scans
template <int KU>
bool launch_scan4_rr_t(const GemmArgs& a, hipStream_t s) {
  const int tiles = a.Ncols / 32;
  const int n_chunks = a.lists ? scan4_list_chunks(a.Mpad, tiles, KU) : scan4_n_chunks(a.Mpad, tiles);
  const int blocks = a.Mpad / kScan4Queries * n_chunks;
  if (a.lists) {  // bounded candidate lists
    bb_launch((scan4_kernel<KU, kScanList | kScanF16>), dim3(blocks), dim3(kScanWaves * 64), 0, s, a, n_chunks, tiles);
    return true;
  }
  if (a.s_h && !a.cand) {  // int16 score image
    bb_launch((scan4_kernel<KU, kScanS16 | kScanF16>), dim3(blocks), dim3(kScanWaves * 64), 0, s, a, n_chunks, tiles);
    return true;
  }
  if (a.f16) {  // f32 score slab
    bb_launch((scan4_kernel<KU, kScanF16>), dim3(blocks), dim3(kScanWaves * 64), 0, s, a, n_chunks, tiles);
    return true;
  }
  return false;
}

// bf16 indexes: streaming appends, the streaming pilot, or the f32 score slab
template <int KU>
void launch_scan4_bf_t(const GemmArgs& a, hipStream_t s) {
  const int tiles = a.Ncols / 32;
  const int n_chunks = scan4_n_chunks(a.Mpad, tiles);
  const int blocks = a.Mpad / kScan4Queries * n_chunks;
  if (a.cand)
    bb_launch((scan4_kernel<KU, kScanStream>), dim3(blocks), dim3(kScanWaves * 64), 0, s, a, n_chunks, tiles);
  else if (a.pilot_top)  // streaming pilot: top-m half-tile maxima, no image
    bb_launch((scan4_kernel<KU, kScanPilot>), dim3(blocks), dim3(kScanWaves * 64), 0, s, a, n_chunks, tiles);
  else
    bb_launch((scan4_kernel<KU>), dim3(blocks), dim3(kScanWaves * 64), 0, s, a, n_chunks, tiles);
}

// per-TU entry points (scan4_rr_*.hip, scan4_bf_*.hip): false when the TU has no instance of ku
bool launch_scan4_rr_lo(const GemmArgs& a, int ku, hipStream_t s, bool& launched);   // KU 8..32
bool launch_scan4_rr_hi(const GemmArgs& a, int ku, hipStream_t s, bool& launched);   // KU 48, 64
bool launch_scan4_bf_lo(const GemmArgs& a, int ku, hipStream_t s);                   // KU 8..32
bool launch_scan4_bf_48(const GemmArgs& a, int ku, hipStream_t s);
bool launch_scan4_bf_64(const GemmArgs& a, int ku, hipStream_t s);
bool launch_scan4_bf_96(const GemmArgs& a, int ku, hipStream_t s);

}  // namespace bb
