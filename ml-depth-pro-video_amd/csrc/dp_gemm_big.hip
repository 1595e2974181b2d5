// dp_gemm_big.hip: the big-tile engine at 256 x 256 / 256 x 128 (incl. grouped launches).
#include "dp_gemm_impl.h"

namespace dpg {
int launch_part_big(const GemmP& p, int tile, bool conv, bool bf16, hipStream_t s) {
  switch (tile) {
    case TILE_GRP_128x128: return (bf16 ? launch_big<KBF16, 128, 128, 64, 3, true>(p, conv, s) : launch_big<KF16, 128, 128, 64, 3, true>(p, conv, s));
    case DP_TILE_BIG_256x128: return (bf16 ? launch_big<KBF16, 256, 128, 64, 3, true>(p, conv, s) : launch_big<KF16, 256, 128, 64, 3, true>(p, conv, s));
    case DP_TILE_BIG_256x128_K32: return (bf16 ? launch_big<KBF16, 256, 128, 32, 6, true>(p, conv, s) : launch_big<KF16, 256, 128, 32, 6, true>(p, conv, s));
    case DP_TILE_BIG_256x256_K32: return (bf16 ? launch_big<KBF16, 256, 256, 32, 2, false>(p, conv, s) : launch_big<KF16, 256, 256, 32, 2, false>(p, conv, s));
    case DP_TILE_DEEP4_256x256: return (bf16 ? launch_big<KBF16, 256, 256, 32, 4, false>(p, conv, s) : launch_big<KF16, 256, 256, 32, 4, false>(p, conv, s));
    case DP_TILE_DEEP5_256x256: return (bf16 ? launch_big<KBF16, 256, 256, 32, 5, false>(p, conv, s) : launch_big<KF16, 256, 256, 32, 5, false>(p, conv, s));
    case DP_TILE_DEEP_256x128: return (bf16 ? launch_big<KBF16, 256, 128, 32, 6, false>(p, conv, s) : launch_big<KF16, 256, 128, 32, 6, false>(p, conv, s));
    default: return (bf16 ? launch_big<KBF16, 256, 256, 64, 2, false>(p, conv, s) : launch_big<KF16, 256, 256, 64, 2, false>(p, conv, s));
  }
}
}  // namespace dpg

#ifdef DP_STAMPS
// timing-only builds: the stamps of the big engine's last launch (tools/gemm_stamps.py)
extern "C" int dp_gemm_stamps(void* host_dst, int n_wg) {
  return (int)hipMemcpyFromSymbol(host_dst, HIP_SYMBOL(g_stamps), (size_t)n_wg * 5 * 8, 0, hipMemcpyDeviceToHost);
}
#endif
