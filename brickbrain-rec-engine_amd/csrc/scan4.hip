// scan4.hip — launcher of the 64-queries-per-wave bf16 scan (scan4_kernel.h); its own
// translation unit so the template instances compile in parallel with gemm.hip.
#include <cstdlib>

#include "scan4_kernel.h"

namespace bb {

static bool scan4_env_off() {
  static const bool off = getenv("BB_NO_SCAN4") != nullptr;
  return off;
}

// bf16 scan, query rows padded to whole 256-query groups and at least BB_SCAN4_MIN rows
// (default 512): the 64-queries-per-wave scan.  A single 256-query group runs scan2
// (measured at 25,216 x 384, B=256: 20.5 vs 23.6 us per launch, 13.3M vs 7.4M q/s with
// three batches in flight, profiles/r02c_b2.jsonl).
bool scan4_used(int dtype, int Mpad) {
  static const int min_rows = getenv("BB_SCAN4_MIN") ? atoi(getenv("BB_SCAN4_MIN")) : 512;
  return dtype == BF16 && Mpad % kScan4Queries == 0 && Mpad >= min_rows && !scan4_env_off();
}

int scan_chunks(int dtype, int Mpad, int tiles, bool split) {
  return !split && scan4_used(dtype, Mpad) ? scan4_n_chunks(Mpad, tiles) : scan_n_chunks(Mpad, tiles);
}

template <int KU>
static void launch_t(const GemmArgs& a, hipStream_t s) {
  const int tiles = a.Ncols / 32;
  const int n_chunks = scan4_n_chunks(a.Mpad, tiles);
  const int blocks = a.Mpad / kScan4Queries * n_chunks;
  if constexpr (KU <= kRrMaxD / 8) {
    if (a.s_h && !a.cand) {  // exact re-rank path: int16 score image
      hipLaunchKernelGGL((scan4_kernel<KU, kScanS16>), dim3(blocks), dim3(kScanWaves * 64), 0, s, a, n_chunks, tiles);
      return;
    }
  }
  if (a.cand)
    hipLaunchKernelGGL((scan4_kernel<KU, kScanStream>), dim3(blocks), dim3(kScanWaves * 64), 0, s, a, n_chunks, tiles);
  else
    hipLaunchKernelGGL((scan4_kernel<KU>), dim3(blocks), dim3(kScanWaves * 64), 0, s, a, n_chunks, tiles);
}

bool launch_scan4(const GemmArgs& a, int ku, hipStream_t s) {
  switch (ku) {
    case 8: launch_t<8>(a, s); return true;
    case 16: launch_t<16>(a, s); return true;
    case 24: launch_t<24>(a, s); return true;
    case 32: launch_t<32>(a, s); return true;
    case 48: launch_t<48>(a, s); return true;
    case 64: launch_t<64>(a, s); return true;
    case 96: launch_t<96>(a, s); return true;
    default: return false;
  }
}

}  // namespace bb
