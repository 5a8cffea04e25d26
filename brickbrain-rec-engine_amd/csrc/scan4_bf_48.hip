// scan4_bf_48.hip — bf16 scan4 instances, KU = 48 (scan4_launch.h)
#include "scan4_launch.h"

namespace bb {
bool launch_scan4_bf_48(const GemmArgs& a, int ku, hipStream_t s) {
  if (ku != 48) return false;
  launch_scan4_bf_t<48>(a, s);
  return true;
}
}  // namespace bb
