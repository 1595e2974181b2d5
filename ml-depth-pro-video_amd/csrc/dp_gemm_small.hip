// dp_gemm_small.hip: the register-staged small-tile engines and the 2-workgroup-per-CU 256 x 128 engine.
#include "dp_gemm_impl.h"

namespace dpg {
int launch_part_small(const GemmP& p, int tile, bool conv, bool bf16, hipStream_t s) {
  switch (tile) {
    case DP_TILE_256x64: return (bf16 ? launch_small<KBF16, 256, 64, 4, 1>(p, conv, s) : launch_small<KF16, 256, 64, 4, 1>(p, conv, s));
    case DP_TILE_256x32: return (bf16 ? launch_small<KBF16, 256, 32, 4, 1>(p, conv, s) : launch_small<KF16, 256, 32, 4, 1>(p, conv, s));
    case DP_TILE_DUAL_256x128: return (bf16 ? launch_dual<KBF16>(p, conv, s) : launch_dual<KF16>(p, conv, s));
    default: return (bf16 ? launch_small<KBF16, 128, 128, 2, 2>(p, conv, s) : launch_small<KF16, 128, 128, 2, 2>(p, conv, s));
  }
}
}  // namespace dpg
