// dp_gemm_big320.hip: the big-tile engine at 320 x 256 and 512 x 128.
#include "dp_gemm_impl.h"

namespace dpg {
int launch_part_big320(const GemmP& p, int tile, bool conv, bool bf16, hipStream_t s) {
  if (tile == DP_TILE_BIG_512x128) return (bf16 ? launch_big<KBF16, 512, 128, 64, 2, false>(p, conv, s) : launch_big<KF16, 512, 128, 64, 2, false>(p, conv, s));
  return (bf16 ? launch_big<KBF16, 320, 256, 64, 2, false>(p, conv, s) : launch_big<KF16, 320, 256, 64, 2, false>(p, conv, s));
}
}  // namespace dpg
