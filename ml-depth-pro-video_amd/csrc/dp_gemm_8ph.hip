// dp_gemm_8ph.hip: the 8-phase 256 x 256 engine.
#include "dp_gemm_impl.h"

namespace dpg {
int launch_part_8ph(const GemmP& p, int tile, bool conv, bool bf16, hipStream_t s) {
  if (tile == DP_TILE_P8PH_256x256) {
    if (conv) return DP_ERR_ARG;
    return bf16 ? launch_p8ph<KBF16>(p, s) : launch_p8ph<KF16>(p, s);
  }
  return (bf16 ? launch_8ph<KBF16>(p, conv, s) : launch_8ph<KF16>(p, conv, s));
}
}  // namespace dpg
