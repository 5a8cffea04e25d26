// scan4_bf_96.hip — bf16 scan4 instances, KU = 96 (scan4_launch.h)
#include "scan4_launch.h"

namespace bb {
bool launch_scan4_bf_96(const GemmArgs& a, int ku, hipStream_t s) {
  if (ku != 96) return false;
  launch_scan4_bf_t<96>(a, s);
  return true;
}
}  // namespace bb
