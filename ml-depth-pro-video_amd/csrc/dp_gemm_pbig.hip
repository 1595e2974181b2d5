// dp_gemm_pbig.hip: the persistent data-parallel engine (320 x 256, 256 x 256).
#include "dp_gemm_impl.h"

namespace dpg {
int launch_part_pbig(const GemmP& p, int tile, bool conv, bool bf16, hipStream_t s) {
  if (tile == DP_TILE_PBIG_320x256) return (bf16 ? launch_pbig<KBF16, 320, 256>(p, conv, s) : launch_pbig<KF16, 320, 256>(p, conv, s));
  return (bf16 ? launch_pbig<KBF16, 256, 256>(p, conv, s) : launch_pbig<KF16, 256, 256>(p, conv, s));
}
}  // namespace dpg
