// scan4.hip — launcher of the 64-queries-per-wave bf16 scan (scan4_kernel.h): shape rules, the
// hybrid dual-scan instances, and dispatch to the per-width instance units (scan4_launch.h).
#include <cstdlib>

#include "scan4_launch.h"

namespace bb {

static bool scan4_env_off() {
  static const bool off = ab_env("BB_NO_SCAN4") != nullptr;
  return off;
}

// bf16 scan, query rows padded to whole 256-query groups and at least BB_SCAN4_MIN rows
// (default 512): the 64-queries-per-wave scan.  A single 256-query group runs scan2
// (measured at 25,216 x 384, B=256: 20.5 vs 23.6 us per launch, 13.3M vs 7.4M q/s with
// three batches in flight, profiles/r02c_b2.jsonl).
bool scan4_used(int dtype, int Mpad) {
  static const int min_rows = ab_env("BB_SCAN4_MIN") ? atoi(ab_env("BB_SCAN4_MIN")) : 512;
  return dtype == BF16 && Mpad % kScan4Queries == 0 && Mpad >= min_rows && !scan4_env_off();
}

int scan_chunks(int dtype, int Mpad, int tiles, bool split, int list_ku) {
  if (split || !scan4_used(dtype, Mpad)) return scan_n_chunks(Mpad, tiles, list_ku > 0 ? kScanListWg : 256);
  return list_ku > 0 ? scan4_list_chunks(Mpad, tiles, list_ku) : scan4_n_chunks(Mpad, tiles);
}

// The hybrid's two re-rank scans (int16 image) in one launch: content rows of 192..512
// (KU0 in {24, 32, 48, 64}), CF factors up to 128 wide (KU1 in {8, 16}).
template <int KU0, int KU1>
static void launch_dual_t(const GemmArgs& a0, const GemmArgs& a1, hipStream_t s) {
  const int t0 = a0.Ncols / 32, t1 = a1.Ncols / 32;
  const int nc0 = a0.lists ? scan4_list_chunks(a0.Mpad, t0, KU0) : scan4_n_chunks(a0.Mpad, t0);
  const int nc1 = a1.lists ? scan4_list_chunks(a1.Mpad, t1, KU1) : scan4_n_chunks(a1.Mpad, t1);
  const int nb0 = a0.Mpad / kScan4Queries * nc0, nb1 = a1.Mpad / kScan4Queries * nc1;
  if (a0.lists)  // bounded candidate lists on both sides (the f16 re-rank copies)
    bb_launch((scan4_dual_kernel<KU0, KU1, kScanList | kScanF16>), dim3(nb0 + nb1), dim3(kScanWaves * 64), 0,
                       s, a0, a1, nc0, t0, nc1, t1, nb0);
  else
    bb_launch((scan4_dual_kernel<KU0, KU1, kScanS16 | kScanF16>), dim3(nb0 + nb1), dim3(kScanWaves * 64), 0,
                       s, a0, a1, nc0, t0, nc1, t1, nb0);
}
template <int KU0>
static bool launch_dual_k1(const GemmArgs& a0, const GemmArgs& a1, int ku1, hipStream_t s) {
  switch (ku1) {
    case 8: launch_dual_t<KU0, 8>(a0, a1, s); return true;
    case 16: launch_dual_t<KU0, 16>(a0, a1, s); return true;
    default: return false;
  }
}
bool scan4_dual_supported(int ku0, int ku1) {
  return (ku0 == 24 || ku0 == 32 || ku0 == 48 || ku0 == 64) && (ku1 == 8 || ku1 == 16);
}
// The dual launcher's shape rules; *why names the first one broken (nullptr: all hold).
bool scan4_dual_args_ok(const GemmArgs& a0, const GemmArgs& a1, const char** why) {
  const int ku0 = a0.Kpad * 2 / 16, ku1 = a1.Kpad * 2 / 16;
  const char* w = nullptr;
  if (a0.ldx <= 0 || a0.ldx >= (int64_t(1) << 23) || a1.ldx <= 0 || a1.ldx >= (int64_t(1) << 23))
    w = "item row stride outside (0, 2^23): the LDS-DMA source offsets are 24-bit (scan4_kernel.h)";
  else if (!scan4_dual_supported(ku0, ku1))
    w = "row widths outside the dual instances (content 192..512, CF up to 128)";
  else if (!a0.s_h || !a1.s_h || !a0.f16 || !a1.f16 || a0.cand || a1.cand || !scan4_used(BF16, a0.Mpad) ||
           a0.Mpad != a1.Mpad)
    w = "not an f16 re-rank scan pair of equal query rows";
  else if (!a0.lists != !a1.lists || (a0.lists && (a0.l_period <= 0 || a0.l_np <= 0 || a1.l_period <= 0 || a1.l_np <= 0)))
    w = "list geometry";
  else if (a0.Ncols % 32 || a1.Ncols % 32 || (a0.slab_start & 31) || (a1.slab_start & 31))
    w = "slab not tile-aligned";
  else if (a0.q_ids || a0.q_src || a0.q_istats || a1.q_ids || a1.q_src || a1.q_istats)
    w = "fused query prologue";
  if (why) *why = w;
  return w == nullptr;
}

hipError_t launch_scan4_dual(const GemmArgs& a0, const GemmArgs& a1, hipStream_t s) {
  const int ku0 = a0.Kpad * 2 / 16, ku1 = a1.Kpad * 2 / 16;
  if (!scan4_dual_args_ok(a0, a1, nullptr)) return hipErrorInvalidValue;
  bool ok = false;
  switch (ku0) {
    case 24: ok = launch_dual_k1<24>(a0, a1, ku1, s); break;
    case 32: ok = launch_dual_k1<32>(a0, a1, ku1, s); break;
    case 48: ok = launch_dual_k1<48>(a0, a1, ku1, s); break;
    case 64: ok = launch_dual_k1<64>(a0, a1, ku1, s); break;
  }
  return ok ? hipGetLastError() : hipErrorInvalidValue;
}

// top-m per lane of a kScanPilot scan4 launch of this row width (the interleaved schedule has
// registers for 8, the chained d = 768 one for 4)
int scan4_pilot_m(int kpad) { return kpad * 2 / 16 <= 64 ? 8 : 4; }

bool launch_scan4(const GemmArgs& a, int ku, hipStream_t s) {
  if (a.ldx <= 0 || a.ldx >= (int64_t(1) << 23)) return false;  // 24-bit DMA offsets (scan4_kernel.h)
  if (ku <= kRrMaxD / 8) {  // the exact re-rank path first (the f16 copy of an f32 index)
    bool launched = false;
    if ((launch_scan4_rr_lo(a, ku, s, launched) || launch_scan4_rr_hi(a, ku, s, launched)) && launched) return true;
  }
  return launch_scan4_bf_lo(a, ku, s) || launch_scan4_bf_48(a, ku, s) || launch_scan4_bf_64(a, ku, s) ||
         launch_scan4_bf_96(a, ku, s);
}

}  // namespace bb
