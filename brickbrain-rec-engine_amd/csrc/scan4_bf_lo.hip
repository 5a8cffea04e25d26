// scan4_bf_lo.hip — bf16 scan4 instances, rows up to 256 wide (scan4_launch.h)
#include "scan4_launch.h"

namespace bb {
bool launch_scan4_bf_lo(const GemmArgs& a, int ku, hipStream_t s) {
  switch (ku) {
    case 8: launch_scan4_bf_t<8>(a, s); return true;
    case 16: launch_scan4_bf_t<16>(a, s); return true;
    case 24: launch_scan4_bf_t<24>(a, s); return true;
    case 32: launch_scan4_bf_t<32>(a, s); return true;
    default: return false;
  }
}
}  // namespace bb
