// scan4_rr_lo.hip — re-rank scan4 instances, rows up to 256 f16 wide (scan4_launch.h)
#include "scan4_launch.h"

namespace bb {
bool launch_scan4_rr_lo(const GemmArgs& a, int ku, hipStream_t s, bool& launched) {
  switch (ku) {
    case 8: launched = launch_scan4_rr_t<8>(a, s); return true;
    case 16: launched = launch_scan4_rr_t<16>(a, s); return true;
    case 24: launched = launch_scan4_rr_t<24>(a, s); return true;
    case 32: launched = launch_scan4_rr_t<32>(a, s); return true;
    default: return false;
  }
}
}  // namespace bb
