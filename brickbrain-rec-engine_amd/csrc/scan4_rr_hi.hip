// scan4_rr_hi.hip — re-rank scan4 instances, rows of 384 / 512 f16 (scan4_launch.h)
#include "scan4_launch.h"

namespace bb {
bool launch_scan4_rr_hi(const GemmArgs& a, int ku, hipStream_t s, bool& launched) {
  switch (ku) {
    case 48: launched = launch_scan4_rr_t<48>(a, s); return true;
    case 64: launched = launch_scan4_rr_t<64>(a, s); return true;
    default: return false;
  }
}
}  // namespace bb
