// scan4_bf_64.hip — bf16 scan4 instances, KU = 64 (scan4_launch.h)
#include "scan4_launch.h"

namespace bb {
bool launch_scan4_bf_64(const GemmArgs& a, int ku, hipStream_t s) {
  if (ku != 64) return false;
  launch_scan4_bf_t<64>(a, s);
  return true;
}
}  // namespace bb
